#!/bin/bash
# k_hex: default (plain x4) vs probe builds 0 (NT x1), 4 (plain x8), 5 (plain x2); then the output tests
mkdir -p gpurun_out/hexvar2
A="--workload c6 --steps 20 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $A > gpurun_out/hexvar2/d.json 2> gpurun_out/hexvar2/d.err || exit 1
for v in 0 4 5; do
  KART_AMD_LIB=$PWD/build/probe/libkartdiff_hex$v.so timeout -k 10 300 python -u bench.py $A > gpurun_out/hexvar2/v$v.json 2> gpurun_out/hexvar2/v$v.err || exit 1
done
for v in d v0 v4 v5; do python3 -c "import json,sys; d=json.load(open('gpurun_out/hexvar2/$v.json')); print('$v', d['ms_per_step'], d['kernels_avg_ms'], d['roofline']['frac'])"; done
timeout -k 10 300 python -u -m pytest tests/test_output.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_output2.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_output2.log; exit $rc
