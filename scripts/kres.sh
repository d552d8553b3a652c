#!/bin/bash
# per-kernel VGPR / LDS / scratch / occupancy of one .hip file (gfx950)
f=$1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -c kart_amd/csrc/$f -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|ScratchSize|Occupancy|LDS Size" \
  | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' | paste -sd' ' | sed 's/Function Name/\nFunction Name/g'
echo
