#!/bin/bash
# FETCH_SIZE calibration of k_fielddiff's access widths (scripts/fetch_calib.hip): build, one
# uninstrumented run, then one --pmc FETCH_SIZE pass; summary in gpurun_out/<tag>_calib.json
set -e
TAG=${1:-calib}
R=$(pwd)
OUT=$R/gpurun_out/${TAG}_calib
mkdir -p $OUT
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 -o $OUT/fetch_calib scripts/fetch_calib.hip
timeout -k 10 120 $OUT/fetch_calib > $OUT/patterns.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $OUT/pmc -o run -- \
    $OUT/fetch_calib > $OUT/pmc_stdout.txt 2> $OUT/pmc_stderr.txt
cd $R
python3 scripts/fetch_calib.py $OUT/patterns.jsonl $OUT/pmc --out gpurun_out/${TAG}_calib.json
rm -f $OUT/fetch_calib
