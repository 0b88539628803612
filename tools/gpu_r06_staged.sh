# Round 6: the staged emit (variants 80 / 81) — its parity tests, then bench lines interleaved with the
# in-place defaults.  Usage: gpurun -- 'OUT=gpurun_out/r6e bash tools/gpu_r06_staged.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6e}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
    tail -${TAILN:-1} "$O/$name.log" | cut -c1-300
}
if [ -z "$SKIP_TESTS" ]; then
TAILN=3 step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK:-staged or wide_record or kernel_for or forced_copy}"
fi
for rnd in 1 2; do
    for c in ${AB:-c2 c4}; do
        for v in ${EMITV:-80 81 57 -1}; do
            SMOLCSUM_LIB=$GRAFT_REPO_ROOT/smoltcp_amd/libsmolcsum_exp.so step ab_${c}_${v}_$rnd 300 python bench.py --config $c --steps 30 --warmup 5 --cpu-seconds 0 --emit-variant $v
        done
    done
done
echo "== done ($(date +%T))"
