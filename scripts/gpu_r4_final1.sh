#!/bin/bash
# round 4 final bench lines, part 1: the driver's default (C3), C3v, C2, C6
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r4F_bench_default.json 2> gpurun_out/r4F_bench_default.err
python3 -c "import json;d=json.load(open('gpurun_out/r4F_bench_default.json'));print('default', d['value'], d['ms_per_step'], d['roofline']['frac'])"
for wl in c3v c2 c6; do
  timeout -k 10 400 python -u bench.py --workload $wl > gpurun_out/r4F_bench_$wl.json 2> gpurun_out/r4F_bench_$wl.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4F_bench_$wl.json'));print('$wl', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
