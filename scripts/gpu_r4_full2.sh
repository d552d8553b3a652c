#!/bin/bash
# round 4: the full-size -m gpu cases (C3 / C3v 100M, C4 50M, C5 100M polygons and mix)
mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
    -k "100000000 or 100_000_000 or c4_layer or 50_000_000" > gpurun_out/r4f2_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r4f2_pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/r4f2_pytest_gpu.log | head; exit $rc
