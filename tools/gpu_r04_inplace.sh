# Round 4: the in-place step (C5) against C2's two-buffer step, per kernel (tools/exp_inplace.py),
# and the bench lines with the fixed list / seg64 floor probes.
# Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_inplace.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4inplace}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -40 "$O/$name.log"; exit $rc; fi
    tail -${TAILN:-1} "$O/$name.log" | cut -c1-400
}
TAILN=40 step inplace_n20 300 python tools/exp_inplace.py 1048576
TAILN=40 step inplace_n24 300 python tools/exp_inplace.py 16777216
for c in c2 c3 c4; do step bench_$c 300 python bench.py --config $c --steps 20 --cpu-seconds 0; done
echo "== done ($(date +%T))"
