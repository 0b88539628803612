# Round 4: the driver's exact command twice, then its kernel trace (per-step anatomy with
# tools/step_trace.py).  Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_steps.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4steps}
mkdir -p $O
for i in 1 2; do
    echo "== drv_$i"; timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { tail -20 $O/drv_$i.log; exit 1; }
    grep '^{' $O/drv_$i.log | cut -c1-200
done
echo "== kt_drv"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_drv -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/kt_drv.log 2>&1 || { tail -20 $O/kt_drv.log; exit 1; }
python3 tools/step_trace.py $O/kt_drv --steps 20 --warmup 5 --out $O/step_trace_c2.json > $O/step_trace.log 2>&1 || { tail -20 $O/step_trace.log; exit 1; }
tail -5 $O/step_trace.log
echo "== done ($(date +%T))"
