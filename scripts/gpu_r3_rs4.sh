#!/bin/bash
# k_resolve3 4-ary sub-bracket search: parity, then C4 A/B (probe rs3bin = binary)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "hash or merge3" > gpurun_out/r3ac_pytest.log 2>&1 || { tail -30 gpurun_out/r3ac_pytest.log; exit 1; }
tail -2 gpurun_out/r3ac_pytest.log
for V in default rs3bin default; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --time-all --no-cpu-baseline --no-host-timing \
      > gpurun_out/r3ac_${V}_c4.json 2> gpurun_out/r3ac_${V}_c4.err || { tail -5 gpurun_out/r3ac_${V}_c4.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3ac_${V}_c4.json'));print('$V', d['value'], d['ms_per_step'], d['kernels_avg_ms'])"
done
