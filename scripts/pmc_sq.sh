#!/bin/bash
# SQ counter passes (issue / wait breakdown) of one bench workload, one rocprofv3 run per pass.
# usage: WL=c3 N=20000000 LIB=kart_amd/probe/libkartdiff_x.so bash scripts/pmc_sq.sh TAG
R=$(pwd)
TAG=${1:-sq}
WL=${WL:-c3}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
[ -n "$LIB" ] && export KART_AMD_LIB=$R/$LIB
ARGS="--workload $WL ${N:+--n $N} --steps 3 --warmup 1 --no-cpu-baseline --no-host-timing --no-sort $BENCH_EXTRA"
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py $ARGS > $OUT/trace.json 2> $OUT/trace.err || exit 1
i=0
P3="TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"
for P in "$P1" "$P2" ${SQ_P3:+"$P3"}; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace -T --output-format csv -d $OUT/p$i -o run -- \
      python3 $R/bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -3 $OUT/p$i.err; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py $OUT
