#!/bin/bash
# round 4: host transfer paths (pageable / pinned chunks / k_to_host) at every size class
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_staging.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4st.log 2>&1
rc=$?; tail -5 gpurun_out/r4st.log; exit $rc
