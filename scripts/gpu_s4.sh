#!/bin/bash
# session-4 GPU round: full parity suite, smoke, one bench line per workload
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_s4.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_s4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s4.log 2>&1 || { tail gpurun_out/smoke_s4.log; exit 1; }
tail -1 gpurun_out/smoke_s4.log
for wl in c2 c4 c5; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench_s4_$wl.json 2> gpurun_out/bench_s4_$wl.err || { tail gpurun_out/bench_s4_$wl.err; exit 1; }
  cat gpurun_out/bench_s4_$wl.json
done
