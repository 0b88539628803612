# Quick GPU check: parity tests, smoke, then C2/C3/C4 benches without the CPU baseline.
# Usage: gpurun -- 'bash tools/gpu_check.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/check
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>: stop on the first failure
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
    tail -${TAILN:-1} "$O/$name.log"
}
TAILN=2 step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for c in ${CONFIGS:-c2 c3 c4}; do
    step bench_$c 300 python bench.py --config $c --cpu-seconds 0
    python3 -c "import json,sys; d=json.loads(open('$O/bench_$c.log').read().strip().splitlines()[-1]); print('   ', '$c', d['value'], d['unit'], d['kernels_ms'])"
done
echo "== done"
