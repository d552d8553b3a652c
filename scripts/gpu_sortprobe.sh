#!/bin/bash
# A/B of kd_sort probe builds on a C3-shaped 100M side + rocprof stats of the default build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r3b}
mkdir -p "$out"
libs=kart_amd/libkartdiff.so
for v in ${2:-}; do libs="$libs,kart_amd/probe/libkartdiff_$v.so"; done
timeout -k 10 400 python -u scripts/sort_bench.py --libs "$libs" ${3:-} > "$out/sort_ab.jsonl" 2> "$out/sort_ab.err" \
    || { echo "sort_bench failed"; tail -20 "$out/sort_ab.err"; exit 1; }
cat "$out/sort_ab.jsonl"
if [ -n "${4:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof" -o sort -- \
      python3 "$GRAFT_REPO_ROOT/scripts/sort_bench.py" --steps 3 > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1 \
      || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/$out/prof.log"; exit 1; }
  find "$GRAFT_REPO_ROOT/$out/prof" -name "*kernel_stats.csv" | head -3
fi
