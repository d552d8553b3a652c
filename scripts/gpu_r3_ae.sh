#!/bin/bash
# k_resolve3 phase probes, then the end-to-end diffs (GC promotion after bulk construction)
set -o pipefail
bash scripts/gpu_r3_rsp.sh && bash scripts/gpu_e2e.sh r3ae 3000000 10000000
