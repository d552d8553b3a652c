#!/bin/bash
# round-end check of the committed tree: the full GPU suite, smoke(), the default bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
