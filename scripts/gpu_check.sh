#!/bin/bash
# GPU check: the -m gpu suite, smoke(), then bench lines for the workloads given (default: c3 c2).
# usage: bash scripts/gpu_check.sh TAG [workload ...]
TAG=${1:-chk}; shift
WLS=${@:-c3 c2}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
for W in $WLS; do
  timeout -k 10 500 python -u bench.py --workload $W --time-all > gpurun_out/${TAG}_bench_$W.json 2> gpurun_out/${TAG}_bench_$W.err || { tail gpurun_out/${TAG}_bench_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$W.json'));print('$W', d['value'], d['unit'], d['ms_per_step'], d['kernels_avg_ms'], (d['roofline'] or {}).get('frac'))"
done
