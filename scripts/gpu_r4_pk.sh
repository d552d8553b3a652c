#!/bin/bash
# round 4: k_pkm_* (deltas into pk order) A/B on the C3 layer: masks per scan thread 2 / 4 / 8 / 16
set -e
mkdir -p gpurun_out
for v in base pk2 pk4 pk16; do
  if [ $v = base ]; then lib=kart_amd/libkartdiff.so; else lib=kart_amd/probe/libkartdiff_$v.so; fi
  KART_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-host-timing --no-sort --time-all \
      > gpurun_out/r4pk_$v.json 2> gpurun_out/r4pk_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4pk_$v.json'));k=d['step_kernels_avg_ms'];print('$v', d['ms_per_step'], d['pk_order']['ms_per_step_events'], {x:k[x] for x in k if 'pkm' in x})"
done
