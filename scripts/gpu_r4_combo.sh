#!/bin/bash
# round 4: GPU suite (minus full-size) + smoke on the final tree, then the k_gf_dense skeleton probe
bash scripts/gpu_r4_full1.sh || exit 1
bash scripts/gpu_r4_gfd.sh
