#!/bin/bash
# round 4: where the first kd_diff2 of a process spends its time (host phase marks, KD_TRACE_HOST=1)
set -e
mkdir -p gpurun_out
KD_TRACE_HOST=1 timeout -k 10 600 python -u scripts/e2e_repo_bench.py --n 3000000 --out gpurun_out/r4x_e2e_3m.json > gpurun_out/r4x_e2e_3m.log 2> gpurun_out/r4x_e2e_3m.err
grep "\[kd\]" gpurun_out/r4x_e2e_3m.err | head -40
python3 -c "
import json;d=json.load(open('gpurun_out/r4x_e2e_3m.json'))
for k in ('pruned walk (cold)','pruned walk (warm)','full walk'): print(k, d[k]['diff_s'], d[k].get('diff_parts_s'))"
