#!/bin/bash
# round 4: drop-in GPU tests + 10M end-to-end diff, then C3 rocprof evidence + C2/C6/C5env lines
mkdir -p gpurun_out
bash scripts/gpu_r4_q.sh || exit $?
bash scripts/gpu_r4_prof1.sh
