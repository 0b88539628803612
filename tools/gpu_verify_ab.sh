# Verify over-fetch experiment: variants 5 (default), 10 (each step's first
# chunk cached: the record's first line stays in L2 for the neighbour's last step) and 14 (shared
# boundary lines, shared_from) on C2 / C4, timed interleaved, then FETCH_SIZE per variant, then the
# verify parity tests for the new variants.
# Usage: gpurun -- 'bash tools/gpu_verify_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/vab; mkdir -p $O
for c in ${CFGS:-c2 c4}; do
    sh=$([ $c = c2 ] && echo 7 || echo 0)
    timeout -k 10 300 python tools/sweep.py --config $c --shapes $sh --var 5,15,10 --reps 20 --rounds 3 > $O/sweep_$c.log 2>&1 || { tail -20 $O/sweep_$c.log; exit 1; }
    grep -v '"round": 0' $O/sweep_$c.log
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$c -o run -- python3 tools/sweep.py --config $c --shapes $sh --var 5,15 --reps 3 --rounds 1 > $O/fetch_$c.log 2>&1 || { tail -20 $O/fetch_$c.log; exit 1; }
    python3 tools/pmc_kernels.py $O/fetch_$c csum_kernel
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "variants_fixed" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
