set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== sweep c2 walk big grids"; timeout -k 10 600 python tools/sweep.py --config c2 --blocks 32,64,128,256 --var 0,1 --shapes 0,1,2 --defer 0 > gpurun_out/sweep_c2w.log 2>&1; rc=$?; grep '"round": 1' gpurun_out/sweep_c2w.log | cut -c1-190; echo "sweep rc=$rc"
