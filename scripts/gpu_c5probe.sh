#!/bin/bash
# C5 bench of the product build and each build/probe variant (kernel times only), then C5 parity tests
mkdir -p gpurun_out
for lib in kart_amd/libkartdiff.so $(ls build/probe/*.so 2>/dev/null); do
  name=$(basename $lib .so)
  KART_AMD_LIB=$(pwd)/$lib timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --time-all \
     > gpurun_out/c5_$name.json 2> gpurun_out/c5_$name.err || { echo "$name failed"; tail -3 gpurun_out/c5_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c5_$name.json')); print('$name', d['ms_per_step'], d['kernels_avg_ms'], d['roofline']['frac'])"
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "env or spatial or c5" --timeout 120 --timeout-method thread 2>&1 | tail -2
