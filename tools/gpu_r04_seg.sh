# Round 4: whole-segment emit for descriptor batches and across wavefronts (variants 23-27).
# Parity tests of the new variants, then interleaved emit timing on C2 / C4 / C3, then the C5
# investigation (tools/gpu_r04_c5.sh stages).  Usage: gpurun --timeout 1200 -- 'bash tools/gpu_r04_seg.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4seg}
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
S=${STAGES:-tests time}
if [[ $S == *tests* ]]; then
    TAILN=3 step tests_seg 600 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_nhc.py -m gpu -x -v --timeout 300 --timeout-method thread
    TAILN=3 step tests_par 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "emit or variants or packed"
fi
if [[ $S == *time* ]]; then
    VARS=${VARS:-19,5,23,24,25,26,27} VARS_c3=${VARS_c3:-7,13,26,27,23,24} TAILN=200 step time 600 python tools/exp_emit_seg.py c2,c4,c3
fi
echo "== done ($(date +%T))"
