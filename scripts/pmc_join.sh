#!/bin/bash
# SQ / TA / TCP counter passes over a short bench (run from the repo root on the GPU box)
R=$(pwd); mkdir -p gpurun_out/pmc; export TMPDIR=/tmp; cd /tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-events"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS" \
           "TA_BUSY TA_TA_BUSY TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -T --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- \
     python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.json 2> $R/gpurun_out/pmc/p$i.err || { echo "pass $i failed"; tail -3 $R/gpurun_out/pmc/p$i.err; }
done
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc 2>&1 | grep -E "k_join2|k_fielddiff|k_partition2|k_place2" || true
