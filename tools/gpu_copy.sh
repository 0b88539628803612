set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/copy1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_copy_emit.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/exp_copy.py 0,1 8,11,12,1 > $O/exp.log 2>&1 || { tail -20 $O/exp.log; exit 1; }
cat $O/exp.log
