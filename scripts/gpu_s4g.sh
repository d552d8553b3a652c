#!/bin/bash
# round-end profiles: C2 (trace + FETCH/WRITE/SQ passes), C3 trace, smoke, default bench line
mkdir -p gpurun_out
WL=c2 KERN=k_join2 NPTS=10000000 timeout -k 10 900 bash scripts/profile_gpu.sh r01s4_c2 || exit 1
cut -d, -f1-6 gpurun_out/prof_r01s4_c2/trace/run_kernel_stats.csv
R=$(pwd); export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof_r01s4_c3 -o run -- \
    python3 $R/bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_r01s4_c3.json 2> $R/gpurun_out/prof_r01s4_c3.err) || exit 1
cut -d, -f1-6 gpurun_out/prof_r01s4_c3/run_kernel_stats.csv
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s4g.log 2>&1 || { tail gpurun_out/smoke_s4g.log; exit 1; }
tail -1 gpurun_out/smoke_s4g.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_s4g_default.json 2> gpurun_out/bench_s4g_default.err || { tail gpurun_out/bench_s4g_default.err; exit 1; }
cat gpurun_out/bench_s4g_default.json
