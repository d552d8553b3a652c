#!/bin/bash
# round 4: first-diff warm-up at kd_init — drop-in GPU tests, the 3M trace, the 10M end-to-end diff
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dropin.py tests/test_merge_index.py tests/test_spatial_diff.py -x -q \
    --timeout 300 --timeout-method thread -m gpu -k "not 100000000" > gpurun_out/r4y_parity.log 2>&1 || { tail -30 gpurun_out/r4y_parity.log; exit 1; }
tail -1 gpurun_out/r4y_parity.log
KD_TRACE_HOST=1 timeout -k 10 600 python -u scripts/e2e_repo_bench.py --n 3000000 --out gpurun_out/r4y_e2e_3m.json > gpurun_out/r4y_e2e_3m.log 2> gpurun_out/r4y_e2e_3m.err
grep "\[kd\]" gpurun_out/r4y_e2e_3m.err | head -14
timeout -k 10 600 python -u scripts/e2e_repo_bench.py --n 10000000 --out gpurun_out/r4y_e2e_10m.json > gpurun_out/r4y_e2e_10m.log 2>&1
python3 -c "
import json
for f in ('gpurun_out/r4y_e2e_3m.json','gpurun_out/r4y_e2e_10m.json'):
    d=json.load(open(f)); print(f, 'init', d.get('engine_init_s'))
    for k in ('pruned walk (cold)','pruned walk (warm)','full walk'): print(' ', k, d[k]['diff_s'], d[k].get('diff_parts_s'), d[k]['field_diff_s'], d[k]['total_s'])"
