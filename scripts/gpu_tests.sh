#!/bin/bash
# the -m gpu suite (per-test timeouts; the full-size C3/C4/C5 cases carry their own) + smoke()
TAG=${1:-t}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
