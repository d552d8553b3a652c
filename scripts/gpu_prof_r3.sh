#!/bin/bash
# round-3 profiles: rocprofv3 kernel stats + FETCH_SIZE + WRITE_SIZE passes per workload
set -e
WL=c3 KERN=k_fielddiff NUNITS=100000000 bash scripts/profile_gpu.sh r3_c3
WL=c5 KERN=k_gf_heads NUNITS=100000000 BENCH_ARGS="--workload c5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-timing --no-arena-timing --no-delta-order" bash scripts/profile_gpu.sh r3_c5
WL=c3v KERN=k_fielddiff NUNITS=100000000 BENCH_ARGS="--workload c3v --steps 5 --warmup 1 --no-cpu-baseline --no-host-timing --no-sort" bash scripts/profile_gpu.sh r3_c3v
