# GPU-box pass: the -m gpu suite, smoke, and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/tests
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --cpu-seconds 4 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['kernels_ms'], d['roofline']['frac'], d['parity_sample'])"
