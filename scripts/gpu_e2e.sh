#!/bin/bash
# end-to-end repository diffs on the GPU box (the repos are built there, in /tmp):
# usage: [EDITS=0.08,0.01,0.01] bash scripts/gpu_e2e.sh TAG N [N ...]
set -o pipefail
TAG=${1:-e2e}; shift
mkdir -p gpurun_out
for N in "${@:-3000000}"; do
  timeout -k 10 ${T:-900} python -u scripts/e2e_repo_bench.py --n $N --edits ${EDITS:-0.01,0.01,0.01} --out gpurun_out/${TAG}_e2e_$N.json \
      > gpurun_out/${TAG}_e2e_$N.log 2>&1 || { tail -30 gpurun_out/${TAG}_e2e_$N.log; exit 1; }
  tail -5 gpurun_out/${TAG}_e2e_$N.log
done
