#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 3 --cpu-seconds 2 --time-all > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
