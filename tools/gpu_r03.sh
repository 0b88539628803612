# Round-3 GPU pass: parity tests, smoke, benches at the driver's flags, kernel traces.
# Usage: gpurun --timeout 1200 -- 'bash tools/gpu_r03.sh'   (STAGES="tests bench kt" to pick)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>: stop on the first failure
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
    tail -${TAILN:-1} "$O/$name.log" | cut -c1-600
}
S=${STAGES:-tests bench kt}
if [[ $S == *tests* ]]; then
    TAILN=3 step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $S == *bench* ]]; then
    step bench_c2 300 python bench.py --gpus 1 --steps 20 --warmup 5
    for c in ${CONFIGS:-c3 c4 c2copy}; do
        step bench_$c 300 python bench.py --config $c --cpu-seconds 0
    done
fi
if [[ $S == *kt* ]]; then
    for c in ${KT:-c2}; do
        step kt_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 0
    done
fi
echo "== done ($(date +%T))"
