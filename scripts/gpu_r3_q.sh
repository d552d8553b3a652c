#!/bin/bash
# the default bench line, then the end-to-end repository diffs at 3M and 10M
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r3q_bench.json 2> gpurun_out/r3q_bench.err || { tail gpurun_out/r3q_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r3q_bench.json'));print(d['value'], d['ms_per_step'], d['kernels_avg_ms'], d.get('value_with_sort'))"
bash scripts/gpu_e2e.sh r3q 3000000 10000000
