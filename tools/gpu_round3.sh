# Round-3 full GPU pass: parity tests, smoke, benches (C2 at the driver's flags with the CPU
# baseline, C3 / C4 / C2copy, C5 at full size), the PCIe end-to-end rates, the C1 loopback analogue,
# kernel traces and FETCH / WRITE counter passes.  Outputs under gpurun_out/r3f/.
# Usage: gpurun --timeout 1800 -- 'bash tools/gpu_round3.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r3f}
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>: stop on the first failure
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
    tail -${TAILN:-1} "$O/$name.log" | cut -c1-300
}
S=${STAGES:-tests bench e2e kt pmc}
if [[ $S == *tests* ]]; then
    TAILN=2 step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $S == *bench* ]]; then
    step bench_c2 300 python bench.py --gpus 1 --steps 20 --warmup 5
    for c in c3 c4 c2copy; do step bench_$c 300 python bench.py --config $c --cpu-seconds 0; done
    step bench_c5 600 python bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 10
fi
if [[ $S == *e2e* ]]; then
    step e2e 400 python tools/e2e.py
    step loopback 400 tools/loopback_ring 262144 5
fi
for c in ${KT:-c2 c3 c4 c2copy}; do
    [[ $S == *kt* ]] || break
    step kt_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/$c/kt -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 0
done
for c in ${PMC:-c2 c3 c4 c2copy}; do
    [[ $S == *pmc* ]] || break
    step fetch_$c 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/$c/fetch -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0
    step write_$c 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/$c/write -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0
done
echo "== done ($(date +%T))"
