#!/bin/bash
# rocprofv3 kernel stats of a short bench run (lib: $LIB or the product build)
R=$(pwd); mkdir -p gpurun_out/kst; export TMPDIR=/tmp
[ -n "$LIB" ] && export KART_AMD_LIB=$R/$LIB
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kst -o run -- \
  python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-check > $R/gpurun_out/kst/bench.json 2> $R/gpurun_out/kst/bench.err \
  || { echo "rocprof failed"; tail -5 $R/gpurun_out/kst/bench.err; exit 1; }
cd $R && f=$(find gpurun_out/kst -name "*kernel_stats.csv" | head -1) && cut -d, -f1-8 $f | head -20
