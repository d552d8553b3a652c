#!/bin/bash
# bench each profiling variant of libkartdiff (build/probe/*.so) and the product build
mkdir -p gpurun_out
for lib in kart_amd/libkartdiff.so $(ls build/probe/*.so 2>/dev/null); do
  name=$(basename $lib .so)
  KART_AMD_LIB=$(pwd)/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check --time-all \
     > gpurun_out/probe_$name.json 2> gpurun_out/probe_$name.err
  rc=$?; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -5 gpurun_out/probe_$name.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/probe_$name.json')); print('$name', d['ms_per_step'], d['kernels_avg_ms'])"
done
