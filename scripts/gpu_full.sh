#!/bin/bash
# parity tests, then the bench, then the profile passes (trace, FETCH, WRITE, SQ)
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || { tail gpurun_out/bench_$TAG.err; exit $rc; }
bash scripts/profile_gpu.sh $TAG
