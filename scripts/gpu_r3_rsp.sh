#!/bin/bash
# k_resolve3 phase probes (results invalid): C4 timing without the ancestor search, OID loads or name checks
set -o pipefail
mkdir -p gpurun_out
for V in default rsnosearch rsnooid rsnonames; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --time-all --no-check --no-cpu-baseline --no-host-timing \
      > gpurun_out/r3ad_${V}_c4.json 2> gpurun_out/r3ad_${V}_c4.err || { tail -5 gpurun_out/r3ad_${V}_c4.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3ad_${V}_c4.json'));print('$V', d['kernels_avg_ms'])"
done
