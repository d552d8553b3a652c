#!/bin/bash
# k_resolve3 ancestor samples per chunk (2^8 / 2^9 / 2^10 default / 2^11): parity, then C4 timing
set -o pipefail
mkdir -p gpurun_out
for V in default ns8 ns9 ns11; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread \
      -k "merge3 and not rejects" > gpurun_out/r3af_$V.log 2>&1 || { echo "$V parity FAILED"; tail -5 gpurun_out/r3af_$V.log; continue; }
  tail -1 gpurun_out/r3af_$V.log
  KART_AMD_LIB=$PWD/$L timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --time-all --no-cpu-baseline --no-host-timing \
      > gpurun_out/r3af_${V}_c4.json 2> gpurun_out/r3af_${V}_c4.err || { tail -5 gpurun_out/r3af_${V}_c4.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3af_${V}_c4.json'));print('$V', d['value'], d['kernels_avg_ms']['k_resolve3'])"
done
