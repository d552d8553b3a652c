#!/bin/bash
# parity of the run-merge variant (pytest -m gpu through build/probe/libkartdiff_${PARITY_LIB:-run}.so), then bench all
mkdir -p gpurun_out
KART_AMD_LIB=$(pwd)/build/probe/libkartdiff_${PARITY_LIB:-run}.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_run3.log 2>&1
rc=$?; echo "pytest(run) exit $rc"; tail -3 gpurun_out/pytest_run3.log; [ $rc -eq 0 ] || exit $rc
bash scripts/probe_variants.sh 2>&1 | grep -v "Traceback\|File \|raise\|obj, end\|JSONDecodeError\|json.load\|return \|^ *\^"
