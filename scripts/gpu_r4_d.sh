#!/bin/bash
# round 4: walk tests, perm/hash/merge3/pipeline parity, C5 mix, benches C3/C4/C5
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r4d_walk.log 2>&1
rc=$?; tail -3 gpurun_out/r4d_walk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_spatial_diff.py -x -v --timeout 600 \
    --timeout-method thread -k "pipeline or perm or hash or merge3 or c5_mix or geom_filter" > gpurun_out/r4d_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r4d_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-timing --no-sort > gpurun_out/r4d_bench_c3.json 2> gpurun_out/r4d_bench_c3.err
rc=$?; tail -1 gpurun_out/r4d_bench_c3.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline > gpurun_out/r4d_bench_c4.json 2> gpurun_out/r4d_bench_c4.err
rc=$?; tail -1 gpurun_out/r4d_bench_c4.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload c5 --steps 20 --no-cpu-baseline > gpurun_out/r4d_bench_c5.json 2> gpurun_out/r4d_bench_c5.err
rc=$?; tail -1 gpurun_out/r4d_bench_c5.err; exit $rc
