#!/bin/bash
# fielddiff: 16-B LDS reads (product) vs dword reads (fdb32): parity suite, then C3 (20M) and C2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fdb.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_fdb.log; [ $rc -eq 0 ] || exit $rc
for v in prod fdb32; do
  if [ $v != prod ]; then export KART_AMD_LIB=$(pwd)/build/probe/libkartdiff_$v.so; else unset KART_AMD_LIB; fi
  timeout -k 10 300 python bench.py --workload c3 --n 20000000 --steps 5 --warmup 1 --no-cpu-baseline --time-all > gpurun_out/fdb3_$v.json 2> gpurun_out/fdb3_$v.err || { tail -3 gpurun_out/fdb3_$v.err; exit 1; }
  echo "c3 $v $(python3 -c "import json;d=json.load(open('gpurun_out/fdb3_$v.json'));print(d['kernels_avg_ms'])")"
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --time-all > gpurun_out/fdb2_$v.json 2> gpurun_out/fdb2_$v.err || { tail -3 gpurun_out/fdb2_$v.err; exit 1; }
  echo "c2 $v $(python3 -c "import json;d=json.load(open('gpurun_out/fdb2_$v.json'));print(d['kernels_avg_ms'])")"
done
