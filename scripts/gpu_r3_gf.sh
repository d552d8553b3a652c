#!/bin/bash
# k_gf_heads without per-round barriers, two rounds of loads in flight: parity, then C5 A/B against
# the previous kernel (probe gfold)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spatial_diff.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r3l_pytest.log 2>&1 || { tail -30 gpurun_out/r3l_pytest.log; exit 1; }
tail -2 gpurun_out/r3l_pytest.log
for V in default gfold default; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline --no-host-timing --no-arena-timing \
      > gpurun_out/r3l_${V}_c5.json 2> gpurun_out/r3l_${V}_c5.err || { tail -5 gpurun_out/r3l_${V}_c5.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3l_${V}_c5.json'));print('$V', d['value'], d['ms_per_step'], d['kernels_avg_ms'], d['heads_delta_order']['ms_per_call'], d['heads_delta_order']['roofline']['avg_launch_ms'], d['heads_delta_order']['roofline']['frac'])"
done
