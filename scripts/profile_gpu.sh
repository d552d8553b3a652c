#!/bin/bash
# rocprofv3 passes for bench.py (run on the GPU box from the repo root):
#   1. --kernel-trace --stats  (per-kernel durations)
#   2. --pmc FETCH_SIZE        (own pass; gfx950: reads 1/2 of wide streaming bytes, doubled later)
#   3. --pmc WRITE_SIZE        (own pass)
# Each step is time-limited and chained with &&: a failure ends the script.
# usage: WL=c3 KERN=k_fielddiff NUNITS=100000000 bash scripts/profile_gpu.sh TAG
set -e
R=$(pwd)
TAG=${1:-r02}
WL=${WL:-c3}
KERN=${KERN:-k_fielddiff}
ARGS=${BENCH_ARGS:-"--workload $WL --steps 5 --warmup 1 --no-cpu-baseline --no-host-timing"}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace_bench.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $OUT/fetch -o run -- \
    python3 $R/bench.py $ARGS > $OUT/fetch_bench.json 2> $OUT/fetch_bench.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $OUT/write -o run -- \
    python3 $R/bench.py $ARGS > $OUT/write_bench.json 2> $OUT/write_bench.err
echo "profile done"
cd $R && python3 scripts/pmc_summary.py $OUT --n ${NUNITS:-100000000} --kernel $KERN --write-traffic $OUT/traffic_$WL.json
