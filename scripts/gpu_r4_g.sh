#!/bin/bash
# round 4: k_join3 with the differing paths compacted (parity + C4 A/B), deferred head fallbacks (C5)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py tests/test_gpu_dropin_perm.py \
    tests/test_spatial_diff.py -x -v --timeout 600 --timeout-method thread -m gpu \
    -k "merge3 or hash_names or late_materialised or falls_back or c5_mix or geom_filter or heads" > gpurun_out/r4g_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r4g_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline > gpurun_out/r4g_bench_c4.json 2> gpurun_out/r4g_bench_c4.err
rc=$?; tail -1 gpurun_out/r4g_bench_c4.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload c5 --steps 20 --no-cpu-baseline > gpurun_out/r4g_bench_c5.json 2> gpurun_out/r4g_bench_c5.err
rc=$?; tail -1 gpurun_out/r4g_bench_c5.err; exit $rc
