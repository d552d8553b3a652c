#!/bin/bash
# round 4: k_gf_dense variants on tiny delta lists (one partial 64-delta chunk)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_spatial_diff.py -x -v --timeout 300 --timeout-method thread -m gpu -k "dense_variants" > gpurun_out/r4gfe.log 2>&1
rc=$?; tail -6 gpurun_out/r4gfe.log; exit $rc
