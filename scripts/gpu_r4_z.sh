#!/bin/bash
# round 4: the first kd_diff2's result copy (trace marks); the C5-envelopes step at 5 / 200 steps
set -e
mkdir -p gpurun_out
KD_TRACE_HOST=1 timeout -k 10 600 python -u scripts/e2e_repo_bench.py --n 3000000 --out gpurun_out/r4z_e2e_3m.json > gpurun_out/r4z_e2e_3m.log 2> gpurun_out/r4z_e2e_3m.err
grep "\[kd\]" gpurun_out/r4z_e2e_3m.err | head -24
for k in 5 200; do
  timeout -k 10 300 python -u bench.py --workload c5env --steps $k --no-cpu-baseline --no-events --no-heads-path > gpurun_out/r4z_c5env_$k.json 2> gpurun_out/r4z_c5env_$k.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4z_c5env_$k.json'));print('c5env steps $k', d['ms_per_step'])"
done
