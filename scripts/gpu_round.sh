#!/bin/bash
# one GPU round: parity tests, bench (both compaction modes), rocprofv3 kernel traces
TAG=${1:-x}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || { tail gpurun_out/bench_$TAG.err; exit $rc; }
export TMPDIR=/tmp
for mode in unord ord; do
  extra=""; [ $mode = unord ] && extra="--unordered"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof_${TAG}_$mode -o run -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline $extra > $R/gpurun_out/prof_${TAG}_$mode.json 2>$R/gpurun_out/prof_${TAG}_$mode.err)
  rc=$?; echo "prof $mode exit $rc"; [ $rc -eq 0 ] || exit $rc
  cut -d, -f1-4 $R/gpurun_out/prof_${TAG}_$mode/run_kernel_stats.csv
done
