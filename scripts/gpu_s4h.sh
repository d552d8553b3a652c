#!/bin/bash
# filename compare with 16-B loads: hash/merge parity, whole suite, C4 + C2 bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_s4h.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_s4h.log; [ $rc -eq 0 ] || exit $rc
for wl in c4 c2; do
  timeout -k 10 600 python -u bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --time-all > gpurun_out/bench_s4h_$wl.json 2> gpurun_out/bench_s4h_$wl.err || { tail -3 gpurun_out/bench_s4h_$wl.err; exit 1; }
  echo "$wl $(python3 -c "import json;d=json.load(open('gpurun_out/bench_s4h_$wl.json'));print(d['ms_per_step'], d['value'], d['kernels_avg_ms'])")"
done
