# Round 4 counters: C3 emit (tile kernel 7, walk 13, whole-segment 27) and copy-emit (17 vs the
# tile split 20): FETCH / WRITE and SQ instruction counters per kernel, one rocprofv3 pass each.
# Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_pmc.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4pmc}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -40 "$O/$name.log"; exit $rc; fi
}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for c in FETCH_SIZE WRITE_SIZE "$SQ"; do
    n=$(echo $c | cut -d' ' -f1)
    K=3 VARS_c3=${VARS_c3:-7,13,27} step c3_$n 240 rocprofv3 --pmc $c --output-format csv -d $O/c3_$n -o run -- python3 tools/exp_emit_seg.py c3
    python3 tools/pmc_kernels.py $O/c3_$n csum
    K=3 ROUNDS=1 step copy_$n 240 rocprofv3 --pmc $c --output-format csv -d $O/copy_$n -o run -- python3 tools/exp_copy.py 8 17,20
    python3 tools/pmc_kernels.py $O/copy_$n copy
done
echo "== done ($(date +%T))"
