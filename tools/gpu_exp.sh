# Ad-hoc experiment pass on the GPU box.  Usage: gpurun -- 'bash tools/gpu_exp.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/exp
mkdir -p $O
for c in c3 c3; do
    timeout -k 10 600 python tools/sweep.py --config $c --shapes 1,8 --var 5,8 --defer 0 --reps 10 > $O/sweep_$c.log 2>&1 || { echo "rc=$?"; tail -20 $O/sweep_$c.log; exit 1; }
    grep '"round": 1' $O/sweep_$c.log | cut -c1-170
done
echo "== fetch"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc8 -o run -- python3 bench.py --config c2 --steps 5 --warmup 1 --cpu-seconds 0 --variant 8 > $O/pmc8.log 2>&1 || { echo "rc=$?"; tail -20 $O/pmc8.log; exit 1; }
echo "== done"
