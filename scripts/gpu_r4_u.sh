#!/bin/bash
# round 4: 10M end-to-end diff (slab + staging set up at kd_init), then the C4 / C5 profiles
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/e2e_repo_bench.py --n 10000000 --out gpurun_out/r4u_e2e_10m.json > gpurun_out/r4u_e2e_10m.log 2>&1
python3 -c "
import json;d=json.load(open('gpurun_out/r4u_e2e_10m.json'))
for k in ('pruned walk (cold)','pruned walk (warm)'): print(k, d[k]['diff_s'], d[k].get('diff_parts_s'))
print('init', d.get('engine_init_s'))"
bash scripts/gpu_r4_prof2.sh
