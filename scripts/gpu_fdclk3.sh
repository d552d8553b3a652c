#!/bin/bash
mkdir -p gpurun_out
KART_AMD_LIB=$(pwd)/build/clk/libkartdiff_fdclk.so timeout -k 10 300 python bench.py --workload c3 --n 20000000 --steps 1 --warmup 0 --no-cpu-baseline --no-check \
  > gpurun_out/fdclk3.txt 2> gpurun_out/fdclk3.err || { tail -3 gpurun_out/fdclk3.err; exit 1; }
grep "^FD " gpurun_out/fdclk3.txt | tail -6
KART_AMD_LIB=$(pwd)/build/clk/libkartdiff_fdclk.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check \
  > gpurun_out/fdclk2.txt 2> gpurun_out/fdclk2.err || { tail -3 gpurun_out/fdclk2.err; exit 1; }
grep "^FD " gpurun_out/fdclk2.txt | tail -4
