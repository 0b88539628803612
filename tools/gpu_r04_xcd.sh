# Round 4: XCD-contiguous block order for the walk kernel (smol_csum_tool_set_xcd_remap) and split
# launches (smol_csum_tool_set_launch_records): parity, then bench lines with and without them,
# interleaved (C2, C4, C3, then C5 at full size).
# Usage: gpurun --timeout 1200 -- 'bash tools/gpu_r04_xcd.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4xcd}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -40 "$O/$name.log"; exit $rc; fi
    tail -${TAILN:-1} "$O/$name.log" | cut -c1-300
}
TAILN=3 step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py -m gpu -x -q --timeout 300 --timeout-method thread -k "xcd or loopback or cpp or launch_records"
for rnd in ${ROUNDS:-1 2}; do
    for c in c2 c4 c3; do
        for x in 0 1; do step bench_${c}_x${x}_r$rnd 300 python bench.py --config $c --steps 20 --cpu-seconds 0 --xcd-remap $x; done
    done
done
for x in 0 1; do
    for lr in 0 2097152; do
        step bench_c5_x${x}_lr$lr 400 python bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 0 --xcd-remap $x --launch-records $lr
    done
done
echo "== done ($(date +%T))"
