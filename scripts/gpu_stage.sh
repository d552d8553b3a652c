#!/bin/bash
# staging ablations (build/probe) + the k_join2r wall-clock timeline (build/clk)
mkdir -p gpurun_out
bash scripts/probe_variants.sh 2>&1 | grep -v "Traceback\|File \|raise\|obj, end\|JSONDecodeError\|json.load\|return \|^ *\^" || exit 1
KART_AMD_LIB=$(pwd)/build/clk/libkartdiff_clk.so timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline \
  --no-check > gpurun_out/clk.txt 2> gpurun_out/clk.err || exit 1
grep -c "^JT" gpurun_out/clk.txt
