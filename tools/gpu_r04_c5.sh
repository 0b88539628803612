# Round 4: where does C5's per-record emit penalty come from?
# - bench lines of the in-place C5 workload at 2^20 .. 2^27 records (is it the buffer size?)
# - C2 beside it on the same box
# - C5 kernel trace, FETCH / WRITE passes and an address-translation (UTCL1 / UTCL2) pass, and the
#   same translation pass on C2
# Usage: gpurun --timeout 1200 -- 'bash tools/gpu_r04_c5.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4c5}
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
S=${STAGES:-sizes kt pmc}
TLB="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
if [[ $S == *sizes* ]]; then
    for c in c2 c3 c4; do step bench_$c 300 python bench.py --config $c --steps 20 --cpu-seconds 0; done
    for e in 20 22 24 26 27; do
        step bench_c5_n$e 300 python bench.py --config c5 --n $((1 << e)) --steps 10 --warmup 2 --cpu-seconds 0
    done
fi
if [[ $S == *kt* ]]; then
    step kt_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/c5/kt -o run -- python3 bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 0
fi
if [[ $S == *pmc* ]]; then
    step fetch_c5 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/c5/fetch -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --ramp-ms 0 --cpu-seconds 0
    step write_c5 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/c5/write -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --ramp-ms 0 --cpu-seconds 0
    step tlb_c5 240 rocprofv3 --pmc $TLB --output-format csv -d $O/prof/c5/tlb -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --ramp-ms 0 --cpu-seconds 0
    step tlb_c2 120 rocprofv3 --pmc $TLB --output-format csv -d $O/prof/c2/tlb -o run -- python3 bench.py --config c2 --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0
    step tlb_c5_n20 120 rocprofv3 --pmc $TLB --output-format csv -d $O/prof/c5n20/tlb -o run -- python3 bench.py --config c5 --n 1048576 --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0
fi
echo "== done ($(date +%T))"
