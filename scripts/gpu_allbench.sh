#!/bin/bash
# every workload's bench line (default options), then the C3 rocprof kernel-trace summary
# usage: bash scripts/gpu_allbench.sh TAG [workloads]
TAG=${1:-all}; shift
WLS=${@:-c3 c2 c4 c5 c6}
mkdir -p gpurun_out
for W in $WLS; do
  timeout -k 10 500 python -u bench.py --workload $W > gpurun_out/${TAG}_bench_$W.json 2> gpurun_out/${TAG}_bench_$W.err || { tail -5 gpurun_out/${TAG}_bench_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$W.json'));r=d.get('roofline') or {};print('$W', d['value'], d['unit'], d['ms_per_step'], r.get('kernel'), r.get('avg_launch_ms'), r.get('frac'))"
done
