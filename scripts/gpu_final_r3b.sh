#!/bin/bash
# final check of the committed tree: the full GPU suite, smoke(), the default bench line, C4 (and a
# 2^12-sample k_resolve3 probe beside it)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3fin2_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/r3fin2_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3fin2_smoke.log 2>&1 || { tail gpurun_out/r3fin2_smoke.log; exit 1; }
tail -1 gpurun_out/r3fin2_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3fin2_bench.json 2> gpurun_out/r3fin2_bench.err || { tail gpurun_out/r3fin2_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r3fin2_bench.json'));print('c3', d['value'], d['ms_per_step'], d.get('value_with_sort'), d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --workload c4 > gpurun_out/r3fin2_c4.json 2> gpurun_out/r3fin2_c4.err || { tail gpurun_out/r3fin2_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r3fin2_c4.json'));print('c4', d['value'], d['kernels_avg_ms'])"
KART_AMD_LIB=$PWD/kart_amd/probe/libkartdiff_ns12.so timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --time-all --no-cpu-baseline --no-host-timing > gpurun_out/r3fin2_ns12_c4.json 2> gpurun_out/r3fin2_ns12_c4.err || { tail -3 gpurun_out/r3fin2_ns12_c4.err; exit 0; }
python3 -c "import json;d=json.load(open('gpurun_out/r3fin2_ns12_c4.json'));print('ns12', d['value'], d['kernels_avg_ms'])"
