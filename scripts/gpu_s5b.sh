#!/bin/bash
# session 5: hex-WKB writer formatting (kd_hex_encode) on the GPU: its tests, the full suite, the C6
# bench line and its rocprof kernel stats
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_output.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_output.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_output.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_s5b.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s5b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c6 > gpurun_out/bench_c6.json 2> gpurun_out/bench_c6.err || { tail gpurun_out/bench_c6.err; exit 1; }
cat gpurun_out/bench_c6.json
WL=c6 KERN=k_hex NPTS=20000000 bash scripts/profile_gpu.sh r01s5_c6
