#!/bin/bash
# rocprofv3 passes over scripts/sort_bench.py (one C3 side, 3 sorts): kernel trace, FETCH_SIZE,
# WRITE_SIZE and two SQ counter sets, one run per pass (counters are never combined with tracing
# domains).  usage: bash scripts/pmc_sort.sh TAG [sort_bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-sort}
shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
ARGS="--steps 3 --no-check $*"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- \
    python3 $R/scripts/sort_bench.py $ARGS > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; exit 1; }
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -T --output-format csv -d $OUT/p$i -o run -- \
      python3 $R/scripts/sort_bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -3 $OUT/p$i.err; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
