#!/bin/bash
# round 4: C3v rocprofv3 kernel stats + FETCH/WRITE passes
set -e
WL=c3v KERN=k_fielddiff NUNITS=100000000 BENCH_ARGS="--workload c3v --steps 5 --warmup 1 --no-cpu-baseline --no-host-timing --no-sort" bash scripts/profile_gpu.sh r4_c3v
