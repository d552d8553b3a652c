#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_e9.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_e9.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_e9.json 2> gpurun_out/bench_e9.err || exit 1
cat gpurun_out/bench_e9.json
bash scripts/probe_variants.sh 2>&1 | grep -v "Traceback\|File \|raise\|obj, end\|JSONDecodeError\|json.load\|return \|^ *\^"
for v in; do
KART_AMD_LIB=$(pwd)/build/probe/libkartdiff_$v.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/$v.txt 2> gpurun_out/$v.err || exit 1
grep "^JT\|^FD" gpurun_out/$v.txt | tail -30
done
