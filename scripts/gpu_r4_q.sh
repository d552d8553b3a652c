#!/bin/bash
# round 4: dropin GPU tests (streaming contract through the Promise builder) + the 10M end-to-end diff
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dropin.py tests/test_merge_index.py -x -q --timeout 300 \
    --timeout-method thread -m gpu > gpurun_out/r4q_dropin.log 2>&1
rc=$?; tail -2 gpurun_out/r4q_dropin.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r4_i.sh
