# Round 4: emit / verify per record against the buffer size (2^17 .. 2^24 records of 1500 B), C2's
# two-buffer step against the in-place step; then C2 / C5 bench lines with the fixed floor probes.
# Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_sizes.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4sizes}
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
[[ ${SKIP_SIZES:-0} == 1 ]] || SIZES=17,18,19,20,21,22,23,24 ROUNDS=3 TAILN=200 step sizes 600 python tools/exp_inplace.py 0 c2,inplace,emit,verify
for c in c2 c4 c3; do step bench_$c 300 python bench.py --config $c --steps 20 --cpu-seconds 0; done
step bench_c5 400 python bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 0
echo "== done ($(date +%T))"
