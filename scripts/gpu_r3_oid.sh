#!/bin/bash
# int-key join with the tile's OIDs staged in LDS (probe oidlds): parity, then C3 and C2 A/B
set -o pipefail
mkdir -p gpurun_out
KART_AMD_LIB=$PWD/kart_amd/probe/libkartdiff_oidlds.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
    --timeout 300 --timeout-method thread -k "diff2 or (device_pipeline and not 100000000)" > gpurun_out/r3s_pytest.log 2>&1 \
    || { tail -30 gpurun_out/r3s_pytest.log; exit 1; }
tail -2 gpurun_out/r3s_pytest.log
for WL in c3 c2; do
for V in default oidlds default; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 400 python -u bench.py --workload $WL --steps 20 --time-all --no-cpu-baseline --no-host-timing \
      > gpurun_out/r3s_${V}_$WL.json 2> gpurun_out/r3s_${V}_$WL.err || { tail -5 gpurun_out/r3s_${V}_$WL.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3s_${V}_$WL.json'));print('$V $WL', d['value'], d['ms_per_step'], d['kernels_avg_ms'])"
done
done
