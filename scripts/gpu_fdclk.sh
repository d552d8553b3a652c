#!/bin/bash
mkdir -p gpurun_out
KART_AMD_LIB=$(pwd)/build/clk/libkartdiff_fdclk.so timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check \
  > gpurun_out/fdclk.txt 2> gpurun_out/fdclk.err || { tail -3 gpurun_out/fdclk.err; exit 1; }
grep "^FD " gpurun_out/fdclk.txt | tail -12
