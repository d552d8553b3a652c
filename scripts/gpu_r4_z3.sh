#!/bin/bash
# round 4: the first kd_diff2's result copy through k_to_host (trace marks), then the drop-in tests
set -e
mkdir -p gpurun_out
KD_TRACE_HOST=1 timeout -k 10 600 python -u scripts/e2e_repo_bench.py --n 3000000 --out gpurun_out/r4z3_e2e_3m.json > gpurun_out/r4z3_e2e_3m.log 2> gpurun_out/r4z3_e2e_3m.err
grep "\[kd\]" gpurun_out/r4z3_e2e_3m.err | head -12
python3 -c "
import json;d=json.load(open('gpurun_out/r4z3_e2e_3m.json'));print('init', d.get('engine_init_s'))
for k in ('pruned walk (cold)','pruned walk (warm)','full walk'): print(' ', k, d[k]['diff_s'], d[k].get('diff_parts_s'), d[k]['field_diff_s'], d[k]['total_s'])"
timeout -k 10 600 python -u -m pytest tests/test_dropin.py tests/test_merge_index.py tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread -m gpu -k "not 100000000 and not 100_000_000" > gpurun_out/r4z3_parity.log 2>&1 || { tail -30 gpurun_out/r4z3_parity.log; exit 1; }
tail -1 gpurun_out/r4z3_parity.log
