#!/bin/bash
# full parity suite, then C2 and C3 bench lines
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_s4e.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_s4e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --time-all > gpurun_out/bench_s4e_c2.json 2> gpurun_out/bench_s4e_c2.err && cat gpurun_out/bench_s4e_c2.json || exit 1
timeout -k 10 900 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --time-all > gpurun_out/bench_s4e_c3.json 2> gpurun_out/bench_s4e_c3.err || { tail gpurun_out/bench_s4e_c3.err; exit 1; }
cat gpurun_out/bench_s4e_c3.json
