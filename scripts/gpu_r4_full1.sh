#!/bin/bash
# round 4: the whole -m gpu suite except the full-size (100M / 50M) cases, then smoke
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "not 100000000 and not 100_000_000 and not c4_layer and not 50_000_000" > gpurun_out/r4f1_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r4f1_pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/r4f1_pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r4f1_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r4f1_smoke.log; exit $rc
