#!/bin/bash
# round 4 evidence, part 1: C3 rocprofv3 (kernel stats + FETCH/WRITE passes; the bench run includes the
# fallback-sort steps) and the C2 / C6 / C5-envelopes bench lines
set -e
WL=c3 KERN=k_fielddiff NUNITS=100000000 bash scripts/profile_gpu.sh r4_c3
for wl in c2 c6 c5env; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 20 > gpurun_out/r4p_bench_$wl.json 2> gpurun_out/r4p_bench_$wl.err
done
echo "prof1 done"
