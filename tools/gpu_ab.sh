# A/B of a compile-time kernel change: smoltcp_amd/libsmolcsum_base.so (before) against the in-tree
# build (after), per config; then the -m gpu suite on the in-tree build.
# Usage: gpurun -- 'bash tools/gpu_ab.sh'  (env: AB_CONFIGS, AB_SHAPES, AB_VARS, AB_TESTS=0 to skip tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
for c in ${AB_CONFIGS:-c2 c4 c3}; do
    SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_base.so timeout -k 10 300 python tools/sweep.py --config $c --shapes ${AB_BASE_SHAPES:-0,7,1} --var ${AB_BASE_VARS:-5} --reps 20 > $O/base_$c.log 2>&1 || { tail -20 $O/base_$c.log; exit 1; }
    timeout -k 10 300 python tools/sweep.py --config $c --shapes ${AB_SHAPES:-0,7,1,2,8} --var ${AB_VARS:-5,13} --reps 20 > $O/new_$c.log 2>&1 || { tail -20 $O/new_$c.log; exit 1; }
    echo "== $c base"; grep '"round": 1' $O/base_$c.log
    echo "== $c new"; grep '"round": 1' $O/new_$c.log
done
if [ "${AB_TESTS:-1}" = 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
    tail -2 $O/tests.log
fi
