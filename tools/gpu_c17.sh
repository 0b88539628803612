set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/c17; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_copy_emit.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|differ" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python tools/exp_copy.py ${SHAPES:-0,1,2,3,8} ${VARS:-16,17,18} > $O/exp.log 2>&1 || { tail -20 $O/exp.log; exit 1; }
grep '"round": 2' $O/exp.log
