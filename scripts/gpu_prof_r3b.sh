#!/bin/bash
# round-3 final profiles: rocprofv3 kernel stats + FETCH_SIZE + WRITE_SIZE passes (C3, C5, C4)
set -e
WL=c3 KERN=k_fielddiff NUNITS=100000000 bash scripts/profile_gpu.sh r3f_c3
WL=c5 KERN=k_gf_heads NUNITS=100000000 BENCH_ARGS="--workload c5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-timing --no-arena-timing --no-delta-order" bash scripts/profile_gpu.sh r3f_c5
WL=c4 KERN=k_join2 NUNITS=150000000 BENCH_ARGS="--workload c4 --steps 5 --warmup 1 --no-cpu-baseline --no-host-timing" bash scripts/profile_gpu.sh r3f_c4
