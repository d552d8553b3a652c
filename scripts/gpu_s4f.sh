#!/bin/bash
# parity suite, then C2 / C4 / C3 bench lines (product build)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_s4f.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_s4f.log; [ $rc -eq 0 ] || exit $rc
for wl in c2 c4 c3; do
  timeout -k 10 900 python -u bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --time-all > gpurun_out/bench_s4f_$wl.json 2> gpurun_out/bench_s4f_$wl.err || { tail -3 gpurun_out/bench_s4f_$wl.err; exit 1; }
  echo "$wl $(python3 -c "import json;d=json.load(open('gpurun_out/bench_s4f_$wl.json'));print(d['ms_per_step'], d['value'], d['kernels_avg_ms'])")"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_s4f_c2_plain.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/bench_s4f_c2_plain.json'));print('c2 plain', d['ms_per_step'], d['value'], d['kernels_avg_ms'])"
