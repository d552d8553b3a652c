#!/bin/bash
# round 4: persistent register-prefetched k_join2r — classify2 parity (the OID-in-LDS join forced at
# every size), the pipeline incl. C3 at 100M, then C3 A/B (KD_J2R=0) and C5
mkdir -p gpurun_out
KD_J2_OIDLDS_MIN=0 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py -x -q --timeout 600 \
    --timeout-method thread -m gpu -k "diff2 or pipeline or pk_order" > gpurun_out/r4o_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r4o_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-timing --no-sort > gpurun_out/r4o_bench_c3.json 2> gpurun_out/r4o_bench_c3.err
rc=$?; tail -1 gpurun_out/r4o_bench_c3.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/r4o_bench_c3.json'));print(d['value'], d['ms_per_step'], d['step_kernels_avg_ms'])"
KD_J2R=0 timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-timing --no-sort > gpurun_out/r4o_bench_c3_nor.json 2> gpurun_out/r4o_bench_c3_nor.err
rc=$?; tail -1 gpurun_out/r4o_bench_c3_nor.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/r4o_bench_c3_nor.json'));print(d['value'], d['ms_per_step'], d['step_kernels_avg_ms'])"
