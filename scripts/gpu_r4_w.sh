#!/bin/bash
# round 4: k_gf_dense (delta-order heads without the pair dependency) parity + A/B on the C5 mix;
# the pinned host staging through the drop-in tests and the 10M end-to-end diff
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spatial_diff.py tests/test_dropin.py tests/test_merge_index.py -x -v \
    --timeout 300 --timeout-method thread -m gpu -k "not 100000000" > gpurun_out/r4w_parity.log 2>&1 || { tail -30 gpurun_out/r4w_parity.log; exit 1; }
tail -2 gpurun_out/r4w_parity.log
timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --no-cpu-baseline --no-arena-timing \
    --ab KD_GF_DENSE=0,KD_GFD=1s,KD_GFD=1t,KD_GFD=2s,KD_GFD=2t > gpurun_out/r4w_c5.json 2> gpurun_out/r4w_c5.err || { tail -20 gpurun_out/r4w_c5.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4w_c5.json'));print(d['ms_per_step'], d['kernels_avg_ms'], d['roofline']['frac']);print(d['ab'])"
timeout -k 10 300 python -u bench.py --workload c5env --steps 20 --no-cpu-baseline --no-events --no-heads-path > gpurun_out/r4w_c5env_noev.json 2> gpurun_out/r4w_c5env_noev.err
python3 -c "import json;d=json.load(open('gpurun_out/r4w_c5env_noev.json'));print('c5env no events', d['ms_per_step'])"
timeout -k 10 600 python -u scripts/e2e_repo_bench.py --n 10000000 --out gpurun_out/r4w_e2e_10m.json > gpurun_out/r4w_e2e_10m.log 2>&1
python3 -c "
import json;d=json.load(open('gpurun_out/r4w_e2e_10m.json'))
for k in ('pruned walk (cold)','pruned walk (warm)','full walk'): print(k, d[k]['diff_s'], d[k].get('diff_parts_s'), d[k]['field_diff_s'], d[k]['total_s'])
print('init', d.get('engine_init_s'))"
