#!/bin/bash
# session-5 closing check: full GPU suite, smoke(), default (C2) and C6 bench lines, C6 kernel stats
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_s5c.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s5c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s5c.log 2>&1 || { tail gpurun_out/smoke_s5c.log; exit 1; }
tail -1 gpurun_out/smoke_s5c.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_s5c_c2.json 2> gpurun_out/bench_s5c_c2.err || { tail gpurun_out/bench_s5c_c2.err; exit 1; }
cat gpurun_out/bench_s5c_c2.json
timeout -k 10 400 python -u bench.py --workload c6 > gpurun_out/bench_s5c_c6.json 2> gpurun_out/bench_s5c_c6.err || { tail gpurun_out/bench_s5c_c6.err; exit 1; }
cat gpurun_out/bench_s5c_c6.json
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof_s5c_c6 -o run -- \
    python3 $R/bench.py --workload c6 --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_s5c_c6.json 2> $R/gpurun_out/prof_s5c_c6.err
