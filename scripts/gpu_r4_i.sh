#!/bin/bash
# round 4: end-to-end `kart diff` of a 10M-feature repository (native delta construction)
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/e2e_repo_bench.py --n 10000000 --out gpurun_out/r4i_e2e_10m.json > gpurun_out/r4i_e2e_10m.log 2>&1
rc=$?; tail -40 gpurun_out/r4i_e2e_10m.log; exit $rc
