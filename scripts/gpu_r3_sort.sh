#!/bin/bash
# round 3: onesweep sort parity + walk-mode pipelines + perm join + C3 bench with value_with_sort
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r3a}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "sort_side or perm" > "$out/pytest_sort.log" 2>&1 || { echo "sort tests failed"; tail -30 "$out/pytest_sort.log"; exit 1; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py \
    -k "device_pipeline" > "$out/pytest_pipe.log" 2>&1 || { echo "pipeline tests failed"; tail -30 "$out/pytest_pipe.log"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-timing \
    > "$out/bench_c3.json" 2> "$out/bench_c3.err" || { echo "bench failed"; tail -20 "$out/bench_c3.err"; exit 1; }
cat "$out/bench_c3.json"
