#!/bin/bash
# k_join2r phase clocks (build/clk variants): one JCLK line per launch
mkdir -p gpurun_out
for lib in build/clk/*.so; do
  name=$(basename $lib .so)
  KART_AMD_LIB=$(pwd)/$lib timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-check --time-all \
    > gpurun_out/$name.txt 2> gpurun_out/$name.err || { echo "$name failed"; tail -3 gpurun_out/$name.err; exit 1; }
  echo "$name"; grep "^JCLK" gpurun_out/$name.txt | tail -2
done
