#!/bin/bash
# flat payload-compare probes (parity, then C3 and C3v bench lines), then the blob-reader A/B at 3M
set -o pipefail
mkdir -p gpurun_out
PK="diff2_golden or diff2_synthetic or (device_pipeline and polygons and not 100000000)"
for V in default ${VARS:-flat4 flat6}; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "$PK" > gpurun_out/r3k_$V.log 2>&1 || { echo "$V parity FAILED"; tail -5 gpurun_out/r3k_$V.log; continue; }
  tail -1 gpurun_out/r3k_$V.log
  for WL in c3 c3v; do
    KART_AMD_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --workload $WL --steps 20 --time-all --no-cpu-baseline --no-host-timing > gpurun_out/r3k_${V}_$WL.json 2> gpurun_out/r3k_${V}_$WL.err || { tail -5 gpurun_out/r3k_${V}_$WL.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r3k_${V}_$WL.json'));print('$V $WL', d['value'], d['ms_per_step'], d['kernels_avg_ms'])"
  done
done
timeout -k 10 500 python -u scripts/odb_ab.py 3000000 kart_amd/libkartdiff.so kart_amd/probe/libkartdiff_odbold.so > gpurun_out/r3k_odb_ab.jsonl 2> gpurun_out/r3k_odb_ab.err || { tail -5 gpurun_out/r3k_odb_ab.err; exit 1; }
cat gpurun_out/r3k_odb_ab.jsonl
