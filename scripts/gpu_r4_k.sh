#!/bin/bash
# round 4: persistent k_gf_heads — spatial parity + C5 bench; then the 10M-feature end-to-end diff
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_spatial_diff.py tests/test_gpu_parity.py tests/test_spatial_index.py \
    tests/test_sf_filter.py -x -q --timeout 500 --timeout-method thread -m gpu \
    -k "c5 or geom_filter or heads or envelopes or index" > gpurun_out/r4k_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r4k_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload c5 --steps 20 --no-cpu-baseline > gpurun_out/r4k_bench_c5.json 2> gpurun_out/r4k_bench_c5.err
rc=$?; tail -1 gpurun_out/r4k_bench_c5.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/r4k_bench_c5.json'));print(d['ms_per_step'], d['step_kernels_avg_ms'], d['roofline']['frac'])"
echo "k done"
