set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== probe"; timeout -k 10 300 ./tools/probe_bw > gpurun_out/probe_bw.log 2>&1; rc=$?; cat gpurun_out/probe_bw.log; echo "probe rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
