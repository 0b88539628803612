# Verify over-fetch experiments: verify variants timed interleaved per config,
# then FETCH_SIZE per variant, then the parity tests of the variants.
#   round 3 measured here (profiles/r03_experiments/) and then removed: 10 / 15 (the
#   record's first line loaded cached), 14 (shared_from in verify), 21 / 22 (REV chunk order)
# Usage: gpurun -- 'VARS_c2=5,<new> bash tools/gpu_verify_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/vab; mkdir -p $O
for c in ${CFGS:-c2 c4 c3}; do
    case $c in c2) sh=7; v=${VARS_c2:-5};; c4) sh=0; v=${VARS_c4:-5};; *) sh=8; v=${VARS_c3:-13};; esac
    timeout -k 10 300 python tools/sweep.py --config $c --shapes $sh --var $v --reps 20 --rounds 3 > $O/sweep_$c.log 2>&1 || { tail -20 $O/sweep_$c.log; exit 1; }
    grep -v '"round": 0' $O/sweep_$c.log | grep round
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$c -o run -- python3 tools/sweep.py --config $c --shapes $sh --var $v --reps 3 --rounds 1 > $O/fetch_$c.log 2>&1 || { tail -20 $O/fetch_$c.log; exit 1; }
    python3 tools/pmc_kernels.py $O/fetch_$c csum_kernel
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "variants_fixed or packed_mixed_lengths_descriptors" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
