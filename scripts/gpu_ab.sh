#!/bin/bash
# A/B of probe builds (kart_amd/probe/libkartdiff_<V>.so, `make probe V=... PFLAGS=...`) on one workload,
# same box: the in-tree library first, then each probe
# usage: bash scripts/gpu_ab.sh TAG workload V1 [V2 ...]      (bench options in BENCH_ARGS)
TAG=${1:-ab}; WL=$2; shift 2
mkdir -p gpurun_out
for V in base "$@"; do
  if [ "$V" = base ]; then unset KART_AMD_LIB; else export KART_AMD_LIB="$(pwd)/kart_amd/probe/libkartdiff_$V.so"; fi
  timeout -k 10 ${T:-500} python -u bench.py --workload $WL $BENCH_ARGS > gpurun_out/${TAG}_${WL}_$V.json \
      2> gpurun_out/${TAG}_${WL}_$V.err || { tail -5 gpurun_out/${TAG}_${WL}_$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${WL}_$V.json'));print('$V', d['value'], d['ms_per_step'], d.get('step_kernels_avg_ms') or d.get('kernels_avg_ms'))"
done
