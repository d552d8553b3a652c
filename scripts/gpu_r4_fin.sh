#!/bin/bash
# round 4: bench after the rank-consistent burst — C5-envelopes, C2, then the driver's default (C3)
set -e
mkdir -p gpurun_out
for wl in c5env c2; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline > gpurun_out/r4fin_$wl.json 2> gpurun_out/r4fin_$wl.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4fin_$wl.json'));print('$wl', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 500 python -u bench.py > gpurun_out/r4fin_default.json 2> gpurun_out/r4fin_default.err
python3 -c "import json;d=json.load(open('gpurun_out/r4fin_default.json'));print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['fallback_sort']['value'])"
