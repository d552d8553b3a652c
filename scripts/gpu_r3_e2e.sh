#!/bin/bash
# drop-in GPU tests, then the end-to-end repository diffs at 3M and 10M features
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dropin.py tests/test_output.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r3j_pytest.log 2>&1 || { tail -30 gpurun_out/r3j_pytest.log; exit 1; }
tail -2 gpurun_out/r3j_pytest.log
bash scripts/gpu_e2e.sh r3j 3000000 10000000
