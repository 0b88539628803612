# Ad-hoc experiment pass on the GPU box.  Usage: gpurun -- 'bash tools/gpu_exp.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/exp
mkdir -p $O
echo "== sweep c3"
timeout -k 10 600 python tools/sweep.py --config c3 --shapes 0,1,2,4,6,8 --var 1,7 --tile 32 --defer 0 > $O/sweep_c3.log 2>&1 || { echo "rc=$?"; tail -20 $O/sweep_c3.log; exit 1; }
grep '"round": 1' $O/sweep_c3.log | cut -c1-160
echo "== done"
