#!/bin/bash
# r02 first check: GPU suite after pruning + k_fielddiff updates-per-round sweep (C3 shape, 20M)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2a_pytest.log; [ $rc -eq 0 ] || exit $rc
for U in 64 32 16; do
  KD_FD_UPR=$U timeout -k 10 300 python -u bench.py --workload c3 --n 20000000 --steps 10 --warmup 2 --no-cpu-baseline --time-all \
     > gpurun_out/r2a_c3_u$U.json 2> gpurun_out/r2a_c3_u$U.err || { tail gpurun_out/r2a_c3_u$U.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r2a_c3_u$U.json'));print($U, d['ms_per_step'], d['kernels_avg_ms'])"
done
