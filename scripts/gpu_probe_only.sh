#!/bin/bash
# bench every probe variant (build/probe/*.so) and the product build (no tests)
mkdir -p gpurun_out
bash scripts/probe_variants.sh
