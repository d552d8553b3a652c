#!/bin/bash
# spatial indexer on heads, C3v parity (2M and 100M)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_spatial_diff.py tests/test_spatial_index.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r3m_spatial.log 2>&1 || { tail -30 gpurun_out/r3m_spatial.log; exit 1; }
tail -2 gpurun_out/r3m_spatial.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 500 --timeout-method thread -k "polygons_same" \
    > gpurun_out/r3m_c3v.log 2>&1 || { tail -30 gpurun_out/r3m_c3v.log; exit 1; }
tail -5 gpurun_out/r3m_c3v.log
