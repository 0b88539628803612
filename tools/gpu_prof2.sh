set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2/kt -o run -- python3 bench.py --steps 20 --cpu-seconds 0 > gpurun_out/prof2/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
cat gpurun_out/prof2/kt/run_kernel_stats.csv | cut -d, -f1-4
