#!/bin/bash
# session-5 round-end check: GPU suite, smoke(), default bench line, then the C2 rocprof passes
bash scripts/gpu_final.sh || exit $?
cp gpurun_out/bench_final.json gpurun_out/r01s5_bench_default.json
bash scripts/profile_gpu.sh r01s5_c2
