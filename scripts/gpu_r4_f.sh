#!/bin/bash
# round 4: one-pass three-way join (k_join3) — merge3 parity (golden, synthetic, edges, unsorted, hash
# names, C4 layer incl. 50M, walk-order segmented), then C4 bench: k_join3 vs the two-step path
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py tests/test_merge_index.py tests/test_gpu_dropin_perm.py -x -v --timeout 600 \
    --timeout-method thread -m gpu -k "merge or hash_names or late_materialised or falls_back" > gpurun_out/r4f_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r4f_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline > gpurun_out/r4f_bench_c4.json 2> gpurun_out/r4f_bench_c4.err
rc=$?; tail -1 gpurun_out/r4f_bench_c4.err; [ $rc -eq 0 ] || exit $rc
KD_MERGE3_JOIN=0 timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline > gpurun_out/r4f_bench_c4_2step.json 2> gpurun_out/r4f_bench_c4_2step.err
rc=$?; tail -1 gpurun_out/r4f_bench_c4_2step.err; exit $rc
