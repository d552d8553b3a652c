#!/bin/bash
# timing events without the system-scope fence: step time with events vs without
mkdir -p gpurun_out
for a in "" "--no-events" "--time-all"; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline $a > gpurun_out/bench_ev.json 2> gpurun_out/bench_ev.err || { tail -3 gpurun_out/bench_ev.err; exit 1; }
  echo "[$a] $(python3 -c "import json;d=json.load(open('gpurun_out/bench_ev.json'));print(d['ms_per_step'], d['value'], d['kernels_avg_ms'])")"
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ev5.json 2> gpurun_out/bench_ev5.err && python3 -c "import json;d=json.load(open('gpurun_out/bench_ev5.json'));print('c5', d['ms_per_step'], d['value'], d['kernels_avg_ms'])"
