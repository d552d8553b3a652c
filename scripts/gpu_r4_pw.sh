#!/bin/bash
# round 4: does an untimed burst right before the timed bracket change the step (GPU idle while the
# host checks results between warmup and timing)?  C5-envelopes and C3, with and without
set -e
mkdir -p gpurun_out
for pw in 0 0.1; do
  BENCH_PREWARM_S=$pw timeout -k 10 300 python -u bench.py --workload c5env --steps 20 --no-cpu-baseline --no-heads-path > gpurun_out/r4pw_c5env_$pw.json 2> gpurun_out/r4pw_c5env_$pw.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4pw_c5env_$pw.json'));print('c5env prewarm $pw', d['ms_per_step'], d['kernels_avg_ms'])"
done
for pw in 0 0.1; do
  BENCH_PREWARM_S=$pw timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-timing --no-sort > gpurun_out/r4pw_c3_$pw.json 2> gpurun_out/r4pw_c3_$pw.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4pw_c3_$pw.json'));print('c3 prewarm $pw', d['value'], d['ms_per_step'], d['kernels_avg_ms'])"
done
