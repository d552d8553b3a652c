#!/bin/bash
# round 4: k_gf_heads A/B on the C5 mix (delta-order heads): rounds per tile, persistent vs one block
# per tile, the load/store skeleton alone; then the C5-envelopes step with every kernel timed
mkdir -p gpurun_out
run() {  # tag lib env...
  local tag=$1 lib=$2; shift 2
  env "$@" KART_AMD_LIB=$lib timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --no-cpu-baseline \
      --no-arena-timing --time-all $X > gpurun_out/r4v_c5_$tag.json 2> gpurun_out/r4v_c5_$tag.err
  local rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4v_c5_$tag.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4v_c5_$tag.json'));print('$tag', d['ms_per_step'], d['kernels_avg_ms'], d['roofline']['frac'])"
}
run base kart_amd/libkartdiff.so A=0
run nopersist kart_amd/libkartdiff.so KD_GF_NOPERSIST=1
run r8 kart_amd/probe/libkartdiff_gfr8.so A=0
X=--no-check run nodecode kart_amd/probe/libkartdiff_gfnd.so A=0
timeout -k 10 300 python -u bench.py --workload c5env --steps 20 --no-cpu-baseline --time-all > gpurun_out/r4v_c5env.json 2> gpurun_out/r4v_c5env.err
python3 -c "import json;d=json.load(open('gpurun_out/r4v_c5env.json'));print('c5env', d['ms_per_step'], d['kernels_avg_ms'])"
