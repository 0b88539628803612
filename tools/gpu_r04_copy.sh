# Round 4: copy-emit tile kernel (variant 20) against variant 17: parity tests, interleaved timing,
# FETCH / WRITE per variant.  Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_copy.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4copy}
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
S=${STAGES:-tests time pmc}
if [[ $S == *tests* ]]; then
    TAILN=3 step tests_copy 600 python -u -m pytest tests/test_gpu_copy_emit.py tests/test_gpu_status.py -m gpu -x -q --timeout 300 --timeout-method thread
fi
if [[ $S == *time* ]]; then
    TAILN=100 step time 400 python tools/exp_copy.py ${COPY_SHAPES:-8,1} ${COPY_VARS:-17,20}
fi
if [[ $S == *pmc* ]]; then
    for c in FETCH_SIZE WRITE_SIZE; do
        K=3 ROUNDS=1 step pmc_$c 200 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- python3 tools/exp_copy.py ${COPY_SHAPES:-8,1} ${COPY_VARS:-17,20}
        python3 tools/pmc_kernels.py $O/$c copy
    done
fi
echo "== done ($(date +%T))"
