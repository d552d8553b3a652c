#!/bin/bash
# round 4: k_gf_dense with and without the decode (the load/store skeleton alone) on the C5 mix
set -e
mkdir -p gpurun_out
for v in base gfdnd; do
  if [ $v = base ]; then lib=kart_amd/libkartdiff.so; X=""; else lib=kart_amd/probe/libkartdiff_$v.so; X=--no-check; fi
  KART_AMD_LIB=$lib timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --no-cpu-baseline --no-arena-timing $X \
      > gpurun_out/r4gfd_$v.json 2> gpurun_out/r4gfd_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/r4gfd_$v.json'));print('$v', d['ms_per_step'], d['kernels_avg_ms'], d['roofline']['frac'])"
done
