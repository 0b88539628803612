set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; cat gpurun_out/smoke.log | tail -5; echo "smoke rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== bench"; timeout -k 10 300 python bench.py --probe > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?; cat gpurun_out/bench1.json; tail -3 gpurun_out/bench1.err; echo "bench rc=$rc"
