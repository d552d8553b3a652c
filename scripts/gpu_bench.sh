#!/bin/bash
# bench lines for the workloads given, each under its own limit; extra bench options in BENCH_ARGS
# usage: bash scripts/gpu_bench.sh TAG workload [workload ...]
TAG=${1:-b}; shift
mkdir -p gpurun_out
for W in "$@"; do
  timeout -k 10 ${T:-600} python -u bench.py --workload $W $BENCH_ARGS > gpurun_out/${TAG}_bench_$W.json \
      2> gpurun_out/${TAG}_bench_$W.err || { tail -5 gpurun_out/${TAG}_bench_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$W.json'));r=d.get('roofline') or {};print('$W', d['value'], d['unit'], d['ms_per_step'], r.get('kernel'), r.get('avg_launch_ms'), r.get('frac'))"
done
