# Emit with whole 64-B field segments (variant 19) against variant 5: the parity tests, timing,
# then FETCH / WRITE per variant.  Usage: gpurun -- 'bash tools/gpu_emit_seg.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/seg; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
VARS=${VARS:-5,19} timeout -k 10 300 python tools/exp_emit_seg.py c2,c4 > $O/time.log 2>&1 || { tail -20 $O/time.log; exit 1; }
grep -v amdgpu.ids $O/time.log
for c in FETCH_SIZE WRITE_SIZE; do
    K=5 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- python3 tools/exp_emit_seg.py c2 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
    python3 tools/pmc_kernels.py $O/$c csum_kernel
done
