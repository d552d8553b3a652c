#!/bin/bash
# the join's LDS-staged OIDs forced on at every size (parity), then the default C3 and C5 lines
set -o pipefail
mkdir -p gpurun_out
KD_J2_OIDLDS_MIN=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py -m gpu -x -v \
    --timeout 300 --timeout-method thread -k "diff2 or device_pipeline or golden" > gpurun_out/r3t_pytest.log 2>&1 \
    || { tail -30 gpurun_out/r3t_pytest.log; exit 1; }
tail -2 gpurun_out/r3t_pytest.log
for WL in c3 c5; do
  timeout -k 10 400 python -u bench.py --workload $WL --no-cpu-baseline --no-host-timing > gpurun_out/r3t_$WL.json 2> gpurun_out/r3t_$WL.err || { tail -5 gpurun_out/r3t_$WL.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3t_$WL.json'));print('$WL', d['value'], d['ms_per_step'], d['kernels_avg_ms'], d.get('value_with_sort'))"
done
