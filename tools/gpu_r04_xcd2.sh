# Round 4: the XCD-contiguous block order per kernel and per batch size (tools/exp_inplace.py, emit
# alone / verify alone / the C2 step / the in-place step, 2^20 .. 2^26 records).
# Usage: gpurun --timeout 1200 -- 'bash tools/gpu_r04_xcd2.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4xcd2}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -40 "$O/$name.log"; exit $rc; fi
}
for x in 0 1; do
    XCD_EMIT=$x XCD_VERIFY=$x SIZES=20,22,24,26 ROUNDS=3 step sizes_x$x 500 python tools/exp_inplace.py 0 c2,inplace,emit,verify
done
echo "== done ($(date +%T))"
