#!/bin/bash
# round 4: split k_join3 + k_resolve3<HAVE_A> — merge parity, C4 A/B (split vs in-join rule), then the
# 10M-feature end-to-end diff
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py tests/test_gpu_dropin_perm.py \
    tests/test_merge_index.py -x -q --timeout 400 --timeout-method thread -m gpu \
    -k "merge or hash_names or late_materialised or falls_back" > gpurun_out/r4m_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r4m_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline > gpurun_out/r4m_bench_c4.json 2> gpurun_out/r4m_bench_c4.err
rc=$?; tail -1 gpurun_out/r4m_bench_c4.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/r4m_bench_c4.json'));print(d['ms_per_step'], d['step_kernels_avg_ms'], d['presorted'])"
KD_MERGE3_SPLIT=0 timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline > gpurun_out/r4m_bench_c4_nosplit.json 2> gpurun_out/r4m_bench_c4_nosplit.err
rc=$?; tail -1 gpurun_out/r4m_bench_c4_nosplit.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/r4m_bench_c4_nosplit.json'));print(d['ms_per_step'], d['step_kernels_avg_ms'], d['presorted'])"
echo "m done"
