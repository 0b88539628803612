# A/B of a copy-emit kernel change: smoltcp_amd/libsmolcsum_base.so (before) against the in-tree build,
# interleaved 3 times, then the copy-emit parity tests on the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/copy_ab; mkdir -p $O
for i in 1 2 3; do
    SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_base.so timeout -k 10 120 python tools/exp_copy.py ${SHAPES:-8} 17 > $O/base$i.log 2>&1 || { tail -20 $O/base$i.log; exit 1; }
    timeout -k 10 120 python tools/exp_copy.py ${SHAPES:-8} 17 > $O/new$i.log 2>&1 || { tail -20 $O/new$i.log; exit 1; }
    echo "base $(grep '"round": 2' $O/base$i.log)"; echo "new  $(grep '"round": 2' $O/new$i.log)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_copy_emit.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; exit $rc
