#!/bin/bash
# round 4 evidence, part 2: C4 (k_join3) and C5 (k_gf_heads) rocprofv3 kernel stats + FETCH/WRITE passes
set -e
WL=c4 KERN=k_join3 NUNITS=50000000 bash scripts/profile_gpu.sh r4_c4
WL=c5 KERN=k_gf_dense NUNITS=100000000 bash scripts/profile_gpu.sh r4_c5d
echo "prof2 done"
