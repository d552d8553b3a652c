#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "merge3" --timeout 200 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload c4 --steps 10 --warmup 2 --cpu-seconds 5 --time-all > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
