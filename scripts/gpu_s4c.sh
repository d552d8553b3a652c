#!/bin/bash
# hash-name checks + merge parity, then the C4 bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "merge3 or hash" --timeout 200 --timeout-method thread > gpurun_out/pytest_s4c.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_s4c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --time-all > gpurun_out/bench_s4c_c4.json 2> gpurun_out/bench_s4c_c4.err || { tail gpurun_out/bench_s4c_c4.err; exit 1; }
cat gpurun_out/bench_s4c_c4.json
