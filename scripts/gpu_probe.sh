#!/bin/bash
# parity tests on the product build, then bench every probe variant (build/probe/*.so)
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-events > gpurun_out/probe_noev.json 2> gpurun_out/probe_noev.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/probe_noev.json')); print('no-events', d['ms_per_step'])"
bash scripts/probe_variants.sh
