#!/bin/bash
# k_fielddiff at 3 waves per SIMD (smaller rounds, two payloads per pass): parity, then C3 / C3v A/B
set -o pipefail
mkdir -p gpurun_out
PK="diff2_golden or (device_pipeline and polygons and not 100000000)"
for V in default ${VARS:-w40 w36 w44}; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "$PK" > gpurun_out/r3w_$V.log 2>&1 || { echo "$V parity FAILED"; tail -5 gpurun_out/r3w_$V.log; continue; }
  tail -1 gpurun_out/r3w_$V.log
  for WL in c3 c3v; do
    KART_AMD_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --workload $WL --steps 20 --no-sort --no-cpu-baseline --no-host-timing > gpurun_out/r3w_${V}_$WL.json 2> gpurun_out/r3w_${V}_$WL.err || { tail -5 gpurun_out/r3w_${V}_$WL.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r3w_${V}_$WL.json'));print('$V $WL', d['value'], d['ms_per_step'], d['kernels_avg_ms'])"
  done
done
