#!/bin/bash
# fielddiff cost split on C3 (20M polygons): product, no parse (E1), no byte-payload compare (E2)
mkdir -p gpurun_out
for v in prod fdg8 fdg32; do
  if [ $v != prod ]; then export KART_AMD_LIB=$(pwd)/build/probe/libkartdiff_$v.so; else unset KART_AMD_LIB; fi
  timeout -k 10 300 python bench.py --workload c3 --n ${N:-20000000} --steps 5 --warmup 1 --no-cpu-baseline --no-check --time-all \
    > gpurun_out/fdexp_$v.json 2> gpurun_out/fdexp_$v.err || { tail -3 gpurun_out/fdexp_$v.err; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/fdexp_$v.json'));print(d['kernels_avg_ms'])")"
done
# C2 (points) with the same variants
for v in prod fdg8 fdg32; do
  if [ $v != prod ]; then export KART_AMD_LIB=$(pwd)/build/probe/libkartdiff_$v.so; else unset KART_AMD_LIB; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --time-all > gpurun_out/fdexp2_$v.json 2> gpurun_out/fdexp2_$v.err || { tail -3 gpurun_out/fdexp2_$v.err; exit 1; }
  echo "c2 $v $(python3 -c "import json;d=json.load(open('gpurun_out/fdexp2_$v.json'));print(d['kernels_avg_ms'])")"
done
