# One GPU-box pass: parity tests, benches (C2/C3/C4), end-to-end PCIe rate, rocprofv3 profiles.
# Usage: gpurun --timeout 1800 -- 'bash tools/gpu_round.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>: stop the whole script on the first failure
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
}
step tests 900 python -m pytest tests -m gpu -x -q
tail -3 $O/tests.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for c in ${BENCH_CONFIGS:-c2 c3 c4}; do
    step bench_$c 400 python bench.py --config $c --probe
    tail -1 $O/bench_$c.log
done
step e2e 400 python tools/e2e.py
tail -1 $O/e2e.log
step loopback 400 tools/loopback_ring 262144 5
tail -1 $O/loopback.log
for c in ${PROF_CONFIGS:-c2 c3 c4}; do
    step kt_$c 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/$c/kt -o run -- python3 bench.py --config $c --steps 20 --cpu-seconds 0
    step fetch_$c 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/$c/fetch -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --cpu-seconds 0
    step write_$c 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/$c/write -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --cpu-seconds 0
done
echo "== done ($(date +%T))"
