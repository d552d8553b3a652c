#!/bin/bash
# fielddiff phase clocks (probe build) + C4 rocprof kernel stats and HBM traffic passes
mkdir -p gpurun_out
bash scripts/gpu_fdclk.sh || exit 1
WL=c4 KERN=k_join2 NPTS=50000000 timeout -k 10 1000 bash scripts/profile_gpu.sh r01s4_c4 || exit 1
cut -d, -f1-6 gpurun_out/prof_r01s4_c4/trace/run_kernel_stats.csv
