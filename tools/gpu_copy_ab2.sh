# Copy-emit read-amplification experiment: variant 17 (default) against 18
# (no destination load for all-payload chunks), 19 (field-free window chunks stored in round 1),
# 20 (both), interleaved, then FETCH_SIZE / WRITE_SIZE per variant, then the copy parity tests.
# Usage: gpurun -- 'bash tools/gpu_copy_ab2.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/cab; mkdir -p $O
timeout -k 10 300 python tools/exp_copy.py 8 17,18,19,20 > $O/time.log 2>&1 || { tail -20 $O/time.log; exit 1; }
grep -v '"round": 0' $O/time.log
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- python3 tools/exp_copy.py 8 17,18,19,20 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
    python3 tools/pmc_kernels.py $O/$c copy_kernel
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_copy_emit.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
