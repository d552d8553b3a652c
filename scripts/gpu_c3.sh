#!/bin/bash
# C3: 100M-polygon layer, 10 % edits, one GPU: bench line + rocprof kernel stats
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --workload c3 --steps 10 --warmup 2 --cpu-seconds 10 --time-all > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
R=$(pwd); export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof_c3 -o run -- \
    python3 $R/bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_c3.json 2> $R/gpurun_out/prof_c3.err
rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
cut -d, -f1-6 $R/gpurun_out/prof_c3/run_kernel_stats.csv
