cd $GRAFT_REPO_ROOT
for lib in kart_amd/libkartdiff.so build/probe/libkartdiff_staged.so; do
echo "== $lib"
KART_AMD_LIB=$(pwd)/$lib timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 60 --timeout-method thread -k "edges" 2>&1 | tail -3
done
