#!/bin/bash
# counter list + SQ counter passes over a short bench (run from the repo root on the GPU box)
R=$(pwd); mkdir -p gpurun_out/pmc; export TMPDIR=/tmp; cd /tmp
timeout -k 10 60 rocprofv3 --list-avail > $R/gpurun_out/pmc/avail.txt 2>&1 || true
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-events"
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -T --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- \
     python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.json 2> $R/gpurun_out/pmc/p$i.err || { echo "pass $i failed"; tail -3 $R/gpurun_out/pmc/p$i.err; }
done
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc 2>&1 | grep -E "k_join2|k_fielddiff|k_partition2|k_place2" || true
