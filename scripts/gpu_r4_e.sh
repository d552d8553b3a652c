#!/bin/bash
# round 4: streamed k_fielddiff — parity (contiguous arenas, both kernels; C3/C3v pipeline streamed),
# then a 20M-polygon A/B of the stream tile shapes against the windowed kernel (C3 and C3v)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "fielddiff_contiguous" > gpurun_out/r4e_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r4e_parity.log; [ $rc -eq 0 ] || exit $rc
KD_FD_STREAM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "pipeline and 2000000 and polygons" > gpurun_out/r4e_pipe.log 2>&1
rc=$?; tail -3 gpurun_out/r4e_pipe.log; [ $rc -eq 0 ] || exit $rc
for wl in c3 c3v; do
  for v in base s16 s32 s32b s64; do
    if [ $v = base ]; then lib=kart_amd/libkartdiff.so; else lib=kart_amd/probe/libkartdiff_$v.so; fi
    KART_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --n 20000000 --steps 10 --no-cpu-baseline \
        --no-host-timing --no-sort > gpurun_out/r4e_${wl}_$v.json 2> gpurun_out/r4e_${wl}_$v.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4e_${wl}_$v.err; exit $rc; }
    python3 -c "import json;d=json.load(open('gpurun_out/r4e_${wl}_$v.json'));print('$wl $v', d['ms_per_step'], d['kernels_avg_ms'], d['roofline']['frac'])"
  done
done
timeout -k 10 500 python -u bench.py --workload c5 --steps 20 --no-cpu-baseline > gpurun_out/r4e_bench_c5.json 2> gpurun_out/r4e_bench_c5.err
rc=$?; tail -1 gpurun_out/r4e_bench_c5.err; exit $rc
