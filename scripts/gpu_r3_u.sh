#!/bin/bash
# k_fielddiff phase timing (probes with the payload compare or the parse removed; results invalid)
set -o pipefail
mkdir -p gpurun_out
for WL in c3 c3v; do
for V in default fdnocmp fdnoparse; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 400 python -u bench.py --workload $WL --steps 20 --no-check --no-cpu-baseline --no-host-timing --no-sort \
      > gpurun_out/r3u_${V}_$WL.json 2> gpurun_out/r3u_${V}_$WL.err || { tail -5 gpurun_out/r3u_${V}_$WL.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3u_${V}_$WL.json'));print('$V $WL', d['value'], d['ms_per_step'], d['kernels_avg_ms'])"
done
done
