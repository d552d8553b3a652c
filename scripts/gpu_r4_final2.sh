#!/bin/bash
# round 4 final bench lines, part 2: C4, C5 (k_gf_dense), C5-envelopes; then the C5 rocprof passes
set -e
mkdir -p gpurun_out
for wl in c4 c5 c5env; do
  timeout -k 10 400 python -u bench.py --workload $wl > gpurun_out/r4F_bench_$wl.json 2> gpurun_out/r4F_bench_$wl.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4F_bench_$wl.json'));print('$wl', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 python -u bench.py --workload c5env --steps 20 --warmup 300 --no-cpu-baseline --no-heads-path > gpurun_out/r4F_c5env_w300.json 2> gpurun_out/r4F_c5env_w300.err
python3 -c "import json;d=json.load(open('gpurun_out/r4F_c5env_w300.json'));print('c5env warmup 300', d['ms_per_step'], d['kernels_avg_ms'])"
WL=c5 KERN=k_gf_dense NUNITS=100000000 BENCH_ARGS="--workload c5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-timing --no-arena-timing" bash scripts/profile_gpu.sh r4_c5d
