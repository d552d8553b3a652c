#!/bin/bash
# round 4: streamed k_fielddiff phase probes at 20M (C3 / C3v; probe builds give invalid results, only
# their times are read), then the end-to-end 10M-feature repository diff (native delta construction)
mkdir -p gpurun_out
for wl in c3 c3v; do
  for v in base s32 s32np s32nc s16np s64np; do
    if [ $v = base ]; then lib=kart_amd/libkartdiff.so; else lib=kart_amd/probe/libkartdiff_$v.so; fi
    KART_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --n 20000000 --steps 10 --no-cpu-baseline \
        --no-host-timing --no-sort --no-check > gpurun_out/r4h_${wl}_$v.json 2> gpurun_out/r4h_${wl}_$v.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4h_${wl}_$v.err; exit $rc; }
    python3 -c "import json;d=json.load(open('gpurun_out/r4h_${wl}_$v.json'));print('$wl $v', d['ms_per_step'], d['kernels_avg_ms'])"
  done
done
timeout -k 10 900 python -u scripts/e2e_repo_bench.py --n 10000000 --out gpurun_out/r4h_e2e_10m.json > gpurun_out/r4h_e2e_10m.log 2>&1
rc=$?; tail -30 gpurun_out/r4h_e2e_10m.log; exit $rc
