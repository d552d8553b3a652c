#!/bin/bash
# k_hex variants (KD_HEX_VARIANT probe builds): 0 NT x1 (default), 1 plain x1, 2 NT x4, 3 plain x4
mkdir -p gpurun_out/hexvar
A="--workload c6 --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $A > gpurun_out/hexvar/v0.json 2> gpurun_out/hexvar/v0.err || exit 1
for v in 1 2 3; do
  KART_AMD_LIB=$PWD/build/probe/libkartdiff_hex$v.so timeout -k 10 300 python -u bench.py $A > gpurun_out/hexvar/v$v.json 2> gpurun_out/hexvar/v$v.err || exit 1
done
for v in 0 1 2 3; do python3 -c "import json,sys; d=json.load(open('gpurun_out/hexvar/v$v.json')); print('v$v', d['ms_per_step'], d['kernels_avg_ms'], d['roofline']['frac'])"; done
