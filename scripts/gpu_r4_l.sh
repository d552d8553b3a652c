#!/bin/bash
# round 4: register-prefetched streamed k_fielddiff (parity, then a 20M A/B against the windowed
# kernel, C3 / C3v); then persistent k_gf_heads (spatial parity + C5) and the 10M end-to-end diff
mkdir -p gpurun_out
for v in p16 p8; do
  KART_AMD_LIB=kart_amd/probe/libkartdiff_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 200 --timeout-method thread -k "fielddiff_contiguous" > gpurun_out/r4l_parity_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/r4l_parity_$v.log; [ $rc -eq 0 ] || exit $rc
done
for wl in c3 c3v; do
  for v in base s16 p16 p16np p8; do
    if [ $v = base ]; then lib=kart_amd/libkartdiff.so; else lib=kart_amd/probe/libkartdiff_$v.so; fi
    KART_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --n 20000000 --steps 10 --no-cpu-baseline \
        --no-host-timing --no-sort --no-check > gpurun_out/r4l_${wl}_$v.json 2> gpurun_out/r4l_${wl}_$v.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4l_${wl}_$v.err; exit $rc; }
    python3 -c "import json;d=json.load(open('gpurun_out/r4l_${wl}_$v.json'));print('$wl $v', d['ms_per_step'], d['kernels_avg_ms'])"
  done
done
bash scripts/gpu_r4_k.sh
