#!/bin/bash
# classify3 rewrite: merge parity first, then the whole suite, then the C4 bench + rocprof stats
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "merge3" --timeout 200 --timeout-method thread > gpurun_out/pytest_s4b_merge.log 2>&1
rc=$?; echo "pytest merge exit $rc"; tail -4 gpurun_out/pytest_s4b_merge.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_s4b.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_s4b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_s4b_c2.json 2> gpurun_out/bench_s4b_c2.err && cat gpurun_out/bench_s4b_c2.json || exit 1
timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --warmup 3 --cpu-seconds 5 --time-all > gpurun_out/bench_s4b_c4.json 2> gpurun_out/bench_s4b_c4.err || { tail gpurun_out/bench_s4b_c4.err; exit 1; }
cat gpurun_out/bench_s4b_c4.json
R=$(pwd); export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof_s4b_c4 -o run -- \
    python3 $R/bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_s4b_c4.json 2> $R/gpurun_out/prof_s4b_c4.err
rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
cut -d, -f1-6 $R/gpurun_out/prof_s4b_c4/run_kernel_stats.csv
