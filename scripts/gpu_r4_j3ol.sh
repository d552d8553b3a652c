#!/bin/bash
# round 4: k_join3 with ours'/theirs' OIDs staged in LDS (KD_J3_OL=1) — merge parity, then C4 A/B
set -e
mkdir -p gpurun_out
KD_J3_OL=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_merge_index.py tests/test_gpu_walk.py -x -q --timeout 300 \
    --timeout-method thread -m gpu -k "merge and not 50000000" > gpurun_out/r4j3ol_parity.log 2>&1 || { tail -30 gpurun_out/r4j3ol_parity.log; exit 1; }
tail -1 gpurun_out/r4j3ol_parity.log
for ol in 0 1; do
  KD_J3_OL=$ol timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline > gpurun_out/r4j3ol_$ol.json 2> gpurun_out/r4j3ol_$ol.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4j3ol_$ol.json'));print('ol $ol', d['ms_per_step'], d['presorted'], d['kernels_avg_ms'])"
done
