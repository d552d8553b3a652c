#!/bin/bash
# a selection of the GPU tests (pytest arguments after the tag), one process, per-test timeouts
# usage: bash scripts/gpu_pytest.sh TAG [pytest args ...]   (T = whole-run limit in s, default 900)
TAG=${1:-sel}; shift
mkdir -p gpurun_out
timeout -k 10 ${T:-900} python -u -m pytest -x -v --timeout ${PT:-200} --timeout-method thread "$@" \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; exit $rc
