# Round 4: the XCD block order for copy-emit (copy_kernel, C2copy) and for emit / verify over
# descriptor batches (tile kernel, walk kernel; C3), on / off interleaved; then the parity test.
# Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_xcd4.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4xcd4}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -40 "$O/$name.log"; exit $rc; fi
}
step tests 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "xcd"
for rnd in 1 2; do
    for x in 0 1 64; do
        XCD=$x step copy_x${x}_r$rnd 300 python tools/exp_copy.py 8 17
        XCD=$x VARS_c3=7,13 K=20 step c3_x${x}_r$rnd 300 python tools/exp_emit_seg.py c3
    done
done
for x in 0 1; do step bench_c3_x$x 300 python bench.py --config c3 --steps 20 --cpu-seconds 0 --xcd-remap $x; done
echo "== done ($(date +%T))"
