#!/bin/bash
# the final bench line of every workload (default options: CPU baselines, host timings and the
# fallback / arena / heads legs included), each under its own limit; lines collected under
# gpurun_out/<TAG>/bench_<wl>.json.  Extra lines: c3 through the join's pairs over per-entry arenas,
# c5 with the device gather of the heads.
# usage: bash scripts/gpu_bench_all.sh TAG workload [workload ...]   (c3pairs, c5gather: the extra lines)
set -o pipefail
TAG=${1:-r06}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for W in "$@"; do
  case $W in
    c3pairs) A="--workload c3 --pair-arenas --no-sort --no-radix" ;;
    c5gather) A="--workload c5 --gh-gather --no-arena-timing" ;;
    *) A="--workload $W" ;;
  esac
  timeout -k 10 ${T:-600} python -u bench.py $A > $OUT/bench_$W.json 2> $OUT/bench_$W.err || { tail -5 $OUT/bench_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$W.json'));r=d.get('roofline') or {};print('$W', d['value'], d['unit'], d['ms_per_step'], r.get('kernel'), r.get('avg_launch_ms'), r.get('frac'), r.get('traffic'))"
done
