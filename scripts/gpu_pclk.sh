#!/bin/bash
mkdir -p gpurun_out
KART_AMD_LIB=$(pwd)/build/clk/libkartdiff_pclk.so timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check \
  > gpurun_out/pclk.txt 2> gpurun_out/pclk.err || { tail -3 gpurun_out/pclk.err; exit 1; }
grep -c PCLK gpurun_out/pclk.txt; grep PCLK gpurun_out/pclk.txt | head -20
