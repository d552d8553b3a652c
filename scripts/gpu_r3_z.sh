#!/bin/bash
# late-materialised join with the tile's order ranges staged in LDS: parity, then value_with_sort A/B (probe permold)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "perm or late or gather or hash" > gpurun_out/r3z_pytest.log 2>&1 || { tail -30 gpurun_out/r3z_pytest.log; exit 1; }
tail -2 gpurun_out/r3z_pytest.log
for V in default permold default; do
  if [ $V = default ]; then L=kart_amd/libkartdiff.so; else L=kart_amd/probe/libkartdiff_$V.so; fi
  KART_AMD_LIB=$PWD/$L timeout -k 10 400 python -u bench.py --workload c3 --no-cpu-baseline --no-host-timing \
      > gpurun_out/r3z_${V}_c3.json 2> gpurun_out/r3z_${V}_c3.err || { tail -5 gpurun_out/r3z_${V}_c3.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3z_${V}_c3.json'));print('$V', d['value'], d['value_with_sort'], d['ms_per_step_with_sort'], d['sort']['k_join2_perm_avg_ms'] if 'sort' in d else None)"
done
