set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu"; timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -30 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== sweep c2"; timeout -k 10 600 python tools/sweep.py --config c2 --blocks 0 --var 3,4 --shapes 0,2 --defer 0 --tile 32,64 --blocks 0,4,8,16,32 > gpurun_out/sweep_c2.log 2>&1; rc=$?; grep '"round": 1' gpurun_out/sweep_c2.log | cut -c1-200; echo "sweep rc=$rc"
