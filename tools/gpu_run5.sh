set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu"; timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== sweep c2"; timeout -k 10 600 python tools/sweep.py --config c2 --blocks 0,4 --nt 1 --shapes 0,1,2 --defer 1,0 > gpurun_out/sweep_c2.log 2>&1; rc=$?; grep '"round": 1' gpurun_out/sweep_c2.log; echo "sweep rc=$rc"
echo "== bench"; timeout -k 10 300 python bench.py --cpu-seconds 2 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; echo "bench rc=$rc"
