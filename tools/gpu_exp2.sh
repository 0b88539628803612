# Round-2 experiment pass: parity tests, smoke, the default bench (with the CPU baseline), then
# the emit variants A/B (5 = default, 9 / 10 = cached field lines) on C2 / C4 with kernel traces.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/exp2
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
if [ -z "$SKIP_TESTS" ]; then
TAILN=2 step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_default 300 python bench.py --probe
for c in ${CONFIGS:-c2 c4}; do
  for v in 5 9 10; do
    step ab_${c}_v$v 300 python bench.py --config $c --variant $v --cpu-seconds 0
    python3 -c "import json; d=json.loads(open('$O/ab_${c}_v$v.log').read().strip().splitlines()[-1]); print('   $c v$v', d['value'], d['kernels_ms'])"
  done
done
for v in 5 9; do
  step kt_c2_v$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/c2_v$v/kt -o run -- python3 bench.py --config c2 --variant $v --steps 20 --cpu-seconds 0
  step write_c2_v$v 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/c2_v$v/write -o run -- python3 bench.py --config c2 --variant $v --steps 5 --warmup 1 --cpu-seconds 0
  step fetch_c2_v$v 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/c2_v$v/fetch -o run -- python3 bench.py --config c2 --variant $v --steps 5 --warmup 1 --cpu-seconds 0
done
echo "== done ($(date +%T))"
