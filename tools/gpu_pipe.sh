# Copy-emit variant A/B (default: 18, whole-line hand-over, against 17): copy parity tests,
# interleaved timing per shape, FETCH / WRITE per variant.
# Usage: gpurun -- 'bash tools/gpu_pipe.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pipe; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_copy_emit.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/exp_copy.py ${SHAPES:-8,2,1,3} ${VARS:-17,18} > $O/time.log 2>&1 || { tail -20 $O/time.log; exit 1; }
grep -v '"round": 0' $O/time.log
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- python3 tools/exp_copy.py 8 ${VARS:-17,18} > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
    python3 tools/pmc_kernels.py $O/$c copy
done
