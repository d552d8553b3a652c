#!/bin/bash
# round 4: spatial parity + C5 (persistent heads, deferred fallbacks), merge parity + C4 A/B (split join3)
bash scripts/gpu_r4_k.sh || exit $?
bash scripts/gpu_r4_m.sh
