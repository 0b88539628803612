# Ad-hoc GPU-box pass: parity tests, smoke, and the c2copy bench + profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/exp
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
for v in -1 1; do
    timeout -k 10 300 python bench.py --config c2copy --variant $v > $O/c2copy_$v.json 2> $O/c2copy_$v.err || { echo "rc=$?"; tail -20 $O/c2copy_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2copy_$v.json').read().strip().splitlines()[-1]); print('var $v', d['value'], d['kernels_ms'])"
done
P=$O/prof/c2copy
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o run -- python3 bench.py --config c2copy --steps 20 > $O/kt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 bench.py --config c2copy --steps 5 --warmup 1 > $O/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 bench.py --config c2copy --steps 5 --warmup 1 > $O/write.log 2>&1 || exit 1
echo "== done"
