# Timed-region anatomy at the driver's flags (--steps 20 --warmup 5) and the C5 refresh.
# Usage: gpurun --timeout 900 -- 'bash tools/gpu_steps.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/steps
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>: stop on the first failure
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
    tail -${TAILN:-1} "$O/$name.log" | cut -c1-400
}
for i in 1 2 3; do
    step drv_$i 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0
done
step w100 200 python bench.py --gpus 1 --steps 20 --warmup 100 --cpu-seconds 0
step s200 200 python bench.py --gpus 1 --steps 200 --warmup 5 --cpu-seconds 0
step kt_drv 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_drv -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0
step kt_w100 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_w100 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 100 --cpu-seconds 0
if [ -n "$C5" ]; then
    step c5 600 python bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 10
    step kt_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c5 -o run -- python3 bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 0
fi
echo "== done ($(date +%T))"
