#!/bin/bash
# round-end check of the committed tree: the full GPU suite, smoke(), the default bench line, C6
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3fin_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/r3fin_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3fin_smoke.log 2>&1 || { tail gpurun_out/r3fin_smoke.log; exit 1; }
tail -1 gpurun_out/r3fin_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3fin_bench.json 2> gpurun_out/r3fin_bench.err || { tail gpurun_out/r3fin_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r3fin_bench.json'));print('c3', d['value'], d['ms_per_step'], d.get('value_with_sort'), d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --workload c6 > gpurun_out/r3fin_c6.json 2> gpurun_out/r3fin_c6.err || { tail gpurun_out/r3fin_c6.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r3fin_c6.json'));print('c6', d['value'], {k:v['value'] for k,v in d['cpu_baseline']['end_to_end'].items()})"
