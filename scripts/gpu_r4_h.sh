#!/bin/bash
# round 4: streamed k_fielddiff phase probes at 20M (C3 / C3v; probe builds give invalid results, only
# their times are read), then the end-to-end 10M-feature repository diff (native delta construction)
mkdir -p gpurun_out
# the double-buffered streamed kernel must be bit-exact before it is timed
for v in s16db s32db; do
  KART_AMD_LIB=kart_amd/probe/libkartdiff_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 200 --timeout-method thread -k "fielddiff_contiguous" > gpurun_out/r4h_parity_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/r4h_parity_$v.log; [ $rc -eq 0 ] || exit $rc
done
for wl in c3 c3v; do
  for v in base s32 s32np s16np s16db s32db s16dbnp; do
    if [ $v = base ]; then lib=kart_amd/libkartdiff.so; else lib=kart_amd/probe/libkartdiff_$v.so; fi
    KART_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --n 20000000 --steps 10 --no-cpu-baseline \
        --no-host-timing --no-sort --no-check > gpurun_out/r4h_${wl}_$v.json 2> gpurun_out/r4h_${wl}_$v.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4h_${wl}_$v.err; exit $rc; }
    python3 -c "import json;d=json.load(open('gpurun_out/r4h_${wl}_$v.json'));print('$wl $v', d['ms_per_step'], d['kernels_avg_ms'])"
  done
done
echo probes done
