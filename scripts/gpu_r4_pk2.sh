#!/bin/bash
# round 4: k_pkm_scan with a one-round-trip tail — pk-order tests, then C3 A/B (16 / 8 masks per thread)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py -x -q --timeout 300 --timeout-method thread -m gpu -k "not 100000000" > gpurun_out/r4pk2_parity.log 2>&1 || { tail -30 gpurun_out/r4pk2_parity.log; exit 1; }
tail -1 gpurun_out/r4pk2_parity.log
for v in base pk8t; do
  if [ $v = base ]; then lib=kart_amd/libkartdiff.so; else lib=kart_amd/probe/libkartdiff_$v.so; fi
  KART_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-host-timing --no-sort --time-all \
      > gpurun_out/r4pk2_$v.json 2> gpurun_out/r4pk2_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4pk2_$v.json'));k=d['step_kernels_avg_ms'];print('$v', d['ms_per_step'], d['pk_order']['ms_per_step_events'], {x:k[x] for x in k if 'pkm' in x})"
done
