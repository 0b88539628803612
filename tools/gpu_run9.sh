set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== sweep c2 tile"; timeout -k 10 600 python tools/sweep.py --config c2 --blocks 0 --var 3,4 --shapes 0,1,2,3,4,5 --defer 0 --tile 32 > gpurun_out/sweep_c2t.log 2>&1; rc=$?; grep '"round": 1' gpurun_out/sweep_c2t.log | cut -c1-190; echo "sweep rc=$rc"
echo "== sweep c2 walk"; timeout -k 10 600 python tools/sweep.py --config c2 --blocks 4,8,16,32 --var 0,1 --shapes 0,2 --defer 0 > gpurun_out/sweep_c2w.log 2>&1; rc=$?; grep '"round": 1' gpurun_out/sweep_c2w.log | cut -c1-190; echo "sweep rc=$rc"
