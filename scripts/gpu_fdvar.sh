#!/bin/bash
# probe-build sweep: each build's parity (pytest -k $PK), then the bench line of workload $WL at N
# usage: [TF=tests/file.py] VARS="a b" WL=c3 N=20000000 PK="device_pipeline and polygons and not 100000000" bash scripts/gpu_fdvar.sh
mkdir -p gpurun_out
WL=${WL:-c3}
PK=${PK:-"device_pipeline and polygons and not 100000000"}
for V in default ${VARS:-}; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 200 python -u -m pytest ${TF:-tests/test_gpu_parity.py} -x -q --timeout 150 --timeout-method thread -m gpu -k "$PK" > gpurun_out/fdv_$V.log 2>&1 || { echo "$V parity FAILED"; tail -5 gpurun_out/fdv_$V.log; continue; }
  KART_AMD_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload $WL ${N:+--n $N} --steps 20 --time-all --no-cpu-baseline --no-host-timing > gpurun_out/fdv_$V.json 2> gpurun_out/fdv_$V.err || { tail -5 gpurun_out/fdv_$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fdv_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels_avg_ms'])"
done
