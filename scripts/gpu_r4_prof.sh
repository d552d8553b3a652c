#!/bin/bash
# round 4 rocprofv3 evidence: per-kernel stats + FETCH/WRITE passes for C3 (with the fallback-sort
# steps of the same bench run), C4 (k_join3) and C5 (k_gf_heads + k_gh_gather + k_gf_fb)
set -e
WL=c3 KERN=k_fielddiff NUNITS=100000000 bash scripts/profile_gpu.sh r4_c3
WL=c4 KERN=k_join3 NUNITS=50000000 bash scripts/profile_gpu.sh r4_c4
WL=c5 KERN=k_gf_heads NUNITS=100000000 bash scripts/profile_gpu.sh r4_c5
echo "all profiles done"
