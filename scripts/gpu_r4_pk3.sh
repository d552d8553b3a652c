#!/bin/bash
# round 4: k_pkm_mark without the pk write (place recomputes it from the record keys)
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
    -k "(pk_order or device_pipeline or walk) and not 100000000" > gpurun_out/r4pk3_parity.log 2>&1 || { tail -30 gpurun_out/r4pk3_parity.log; exit 1; }
tail -1 gpurun_out/r4pk3_parity.log
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-host-timing --no-sort --time-all > gpurun_out/r4pk3.json 2> gpurun_out/r4pk3.err
python3 -c "import json;d=json.load(open('gpurun_out/r4pk3.json'));k=d['step_kernels_avg_ms'];print('new', d['ms_per_step'], d['pk_order']['ms_per_step_events'], {x:k[x] for x in k if 'pkm' in x})"
