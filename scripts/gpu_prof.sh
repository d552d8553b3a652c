#!/bin/bash
# rocprofv3 --kernel-trace --stats of one bench workload (the per-kernel summary the roofline cites)
# usage: bash scripts/gpu_prof.sh TAG workload [bench options ...]
TAG=${1:-p}; WL=${2:-c3}; shift 2
R=$(pwd)
OUT=$R/gpurun_out/${TAG}_prof_$WL
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 ${T:-500} rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT -o run -- \
    python3 $R/bench.py --workload $WL --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -5 $OUT/bench.err; exit 1; }
f=$(find $OUT -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $R/gpurun_out/${TAG}_${WL}_kernel_stats.csv
head -12 $R/gpurun_out/${TAG}_${WL}_kernel_stats.csv | cut -d, -f1-4
