#!/bin/bash
# round 4, first GPU pass: the walk-order tests, the pipeline/sort parity cases, smoke, a short C3 bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -x -v --timeout 300 --timeout-method thread \
    -k "not 50_000_000" > gpurun_out/r4a_walk.log 2>&1
rc=$?; tail -3 gpurun_out/r4a_walk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread \
    -k "pipeline or sort or pack_side or perm" > gpurun_out/r4a_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r4a_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1 || { tail gpurun_out/r4a_smoke.log; exit 1; }
tail -1 gpurun_out/r4a_smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --no-cpu-baseline --no-host-timing > gpurun_out/r4a_bench_c3.json 2> gpurun_out/r4a_bench_c3.err
rc=$?; tail -2 gpurun_out/r4a_bench_c3.err; exit $rc
