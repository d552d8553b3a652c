#!/bin/bash
# round 4: k_place2 with 4 tiles per workgroup — classify2 parity, then C3 A/B (1 vs 4 waves per workgroup)
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py tests/test_dropin.py -x -q --timeout 300 \
    --timeout-method thread -m gpu -k "not 100000000" > gpurun_out/r4pl_parity.log 2>&1 || { tail -30 gpurun_out/r4pl_parity.log; exit 1; }
tail -1 gpurun_out/r4pl_parity.log
for w in 1 4 1 4; do
  KD_PLACE_WPB=$w timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-host-timing --no-sort --time-all > gpurun_out/r4pl_$w.json 2> gpurun_out/r4pl_$w.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4pl_$w.json'));k=d['step_kernels_avg_ms'];print('wpb $w', d['ms_per_step'], k['k_place2'], k['k_join2'], k['k_fielddiff'])"
done
