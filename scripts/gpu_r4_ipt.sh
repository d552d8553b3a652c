#!/bin/bash
# round 4: classify2 tile size A/B on C3 (items per thread 4 = default, 3, 6, 8)
set -e
mkdir -p gpurun_out
for v in base ipt3 ipt6 ipt8; do
  if [ $v = base ]; then lib=kart_amd/libkartdiff.so; else lib=kart_amd/probe/libkartdiff_$v.so; fi
  KART_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-host-timing --no-sort --time-all \
      > gpurun_out/r4ipt_$v.json 2> gpurun_out/r4ipt_$v.err || { tail -5 gpurun_out/r4ipt_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4ipt_$v.json'));k=d['step_kernels_avg_ms'];print('$v', d['ms_per_step'], {x:k[x] for x in ('k_partition2','k_join2','k_gscan2','k_place2')})"
done
