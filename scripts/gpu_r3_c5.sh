#!/bin/bash
# heads kernel: parity, C5 bench line, then its own rocprof summary + traffic (pipeline launches only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spatial_diff.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r3i_pytest.log 2>&1 || { tail -30 gpurun_out/r3i_pytest.log; exit 1; }
tail -2 gpurun_out/r3i_pytest.log
timeout -k 10 500 python -u bench.py --workload c5 > gpurun_out/r3i_bench_c5.json 2> gpurun_out/r3i_bench_c5.err || { tail gpurun_out/r3i_bench_c5.err; exit 1; }
cat gpurun_out/r3i_bench_c5.json
WL=c5 KERN=k_gf_heads NUNITS=100000000 BENCH_ARGS="--workload c5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-timing --no-arena-timing --no-delta-order" bash scripts/profile_gpu.sh r3i_c5
