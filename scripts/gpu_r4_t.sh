#!/bin/bash
# round 4: streamed k_fielddiff with full 64-lane tiles (T = 64 / 48: every lane parses), 20M A/B
mkdir -p gpurun_out
KART_AMD_LIB=kart_amd/probe/libkartdiff_s64b.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
    --timeout 200 --timeout-method thread -k "fielddiff_contiguous" > gpurun_out/r4t_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r4t_parity.log; [ $rc -eq 0 ] || exit $rc
for wl in c3 c3v; do
  for v in base s64b s48 s64bnp; do
    if [ $v = base ]; then lib=kart_amd/libkartdiff.so; else lib=kart_amd/probe/libkartdiff_$v.so; fi
    KART_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --n 20000000 --steps 10 --no-cpu-baseline \
        --no-host-timing --no-sort --no-check > gpurun_out/r4t_${wl}_$v.json 2> gpurun_out/r4t_${wl}_$v.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4t_${wl}_$v.err; exit $rc; }
    python3 -c "import json;d=json.load(open('gpurun_out/r4t_${wl}_$v.json'));print('$wl $v', d['ms_per_step'], d['kernels_avg_ms'])"
  done
done
