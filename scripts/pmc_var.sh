#!/bin/bash
# SQ counter passes of k_join2 for the libs named in $LIBS (paths relative to the repo root)
R=$(pwd); export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-events --no-check"
for lib in $LIBS; do
  name=$(basename $lib .so); mkdir -p gpurun_out/pmcv/$name
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    (cd /tmp && KART_AMD_LIB=$R/$lib timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -T --output-format csv \
       -d $R/gpurun_out/pmcv/$name/p$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcv/$name/p$i.json \
       2> $R/gpurun_out/pmcv/$name/p$i.err) || { echo "$name pass $i failed"; tail -3 gpurun_out/pmcv/$name/p$i.err; exit 1; }
  done
  echo "== $name"; python3 scripts/pmc_summary.py gpurun_out/pmcv/$name 2>&1 | grep -E "k_join2|k_place2" || true
done
