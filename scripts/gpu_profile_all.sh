#!/bin/bash
# rocprofv3 evidence for the committed profiles (one workload after another; each step under its own
# time limit, a failure ends the script):  per workload the --kernel-trace --stats summary and the
# FETCH_SIZE / WRITE_SIZE traffic of its dominant kernel (scripts/profile_gpu.sh), and for c3 / c3v
# the SQ counter passes (scripts/pmc_sq.sh).  Results are collected under gpurun_out/<TAG>/.
# usage: bash scripts/gpu_profile_all.sh TAG workload [workload ...]   (c5arena = c5 through the arenas)
set -o pipefail
TAG=${1:-r06}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
COMMON="--steps 5 --warmup 1 --no-cpu-baseline --no-host-timing --no-sort --no-radix"
for W in "$@"; do
  case $W in
    c3|c3v) K=k_fielddiff; N=100000000; A="--workload $W $COMMON" ;;
    c2) K=k_join2; N=10000000; A="--workload c2 $COMMON" ;;
    c4) K=k_join3; N=50000000; A="--workload c4 $COMMON" ;;
    c5) K=k_gf_dense; N=100000000; A="--workload c5 $COMMON --no-arena-timing" ;;
    c5arena) K=k_gf_match; N=100000000; A="--workload c5 $COMMON --arena" ;;
    c5env) K=k_envelopes; N=20000000; A="--workload c5env $COMMON --no-heads-path" ;;
    c6) K=k_hex; N=20000000; A="--workload c6 $COMMON" ;;
    *) echo "unknown workload $W"; exit 1 ;;
  esac
  WL=$W KERN=$K NUNITS=$N BENCH_ARGS="$A" bash scripts/profile_gpu.sh ${TAG}_$W > $OUT/prof_$W.log 2>&1 || { tail -20 $OUT/prof_$W.log; exit 1; }
  cp gpurun_out/prof_${TAG}_$W/trace/run_kernel_stats.csv $OUT/${W}_kernel_stats.csv
  cp gpurun_out/prof_${TAG}_$W/traffic_$W.json $OUT/traffic_$W.json
  grep -E "^$K|^k_fielddiff|^k_join|^k_gf|^k_env|^k_hex" $OUT/prof_$W.log | cut -c1-200 | head -8 > $OUT/pmc_$W.txt
  echo "$W: $(cat $OUT/traffic_$W.json | tr -d '\n ' | cut -c1-200)"
  if [ $W = c3 ] || [ $W = c3v ]; then
    WL=$W N=100000000 bash scripts/pmc_sq.sh ${TAG}_$W > $OUT/sq_$W.log 2>&1 || { tail -20 $OUT/sq_$W.log; exit 1; }
    grep -E "^k_fielddiff|^k_join2" $OUT/sq_$W.log > $OUT/sq_$W.txt
    echo "$W sq: $(cut -c1-160 $OUT/sq_$W.txt | head -2)"
  fi
done
