# Round-6 GPU pass.  Stages (STAGES, space-separated):
#   tests   the -m gpu suite and smoke()
#   bench   bench lines for BENCH (default: c2 at the driver's flags, then c3 c4 c2copy)
#   c5      the C5 bench line (201 GB, ~2 min)
#   kt      kernel traces (rocprofv3 --kernel-trace --stats) for KT configs
#   pmc     FETCH_SIZE / WRITE_SIZE passes for PMC configs
#   sq      SQ instruction counters for SQ configs
#   e2e     PCIe end-to-end rates and the C1 loopback analogue
#   wtax    tools/probe_wtax (inline / deferred / pipelined / staged field-segment writes, C2 geometry)
#   ab      bench lines per EMITV (emit variants, experiments build) for AB configs, interleaved
# Outputs under $OUT (default gpurun_out/r5).  Usage: gpurun --timeout 1200 -- 'STAGES="tests bench" bash tools/gpu_r06.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6}
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
S=${STAGES:-tests bench}
if [[ $S == *tests* ]]; then
    TAILN=2 step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $S == *bench* ]]; then
    for c in ${BENCH:-c2 c3 c4 c2copy}; do
        if [ $c = c2 ]; then step bench_c2 300 python bench.py --gpus 1 --steps 20 --warmup 5
        else step bench_$c 300 python bench.py --config $c --cpu-seconds 0; fi
    done
fi
if [[ $S == *c5* ]]; then
    step bench_c5 600 python bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 10
fi
if [[ $S == *e2e* ]]; then
    step e2e 400 python tools/e2e.py
    step loopback 400 tools/loopback_ring 262144 5
fi
if [[ $S == *kt* ]]; then
    for c in ${KT:-c2 c3 c4 c2copy}; do
        step kt_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/$c/kt -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 0
    done
fi
if [[ $S == *pmc* ]]; then
    for c in ${PMC:-c2 c3 c4 c2copy}; do
        step fetch_$c 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/$c/fetch -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0
        step write_$c 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/$c/write -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0
    done
fi
if [[ $S == *sq* ]]; then
    for c in ${SQ:-c2 c2copy}; do
        step sq_$c 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $O/prof/$c/sq -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0
    done
fi
if [[ $S == *wtax* ]]; then
    step wtax 400 tools/probe_wtax ${WTAX_N:-1048576} ${WTAX_L:-1500} ${WTAX_ROUNDS:-3}
    cp $O/wtax.log $O/wtax.jsonl
fi
if [[ $S == *ab* ]]; then
    for rnd in 1 2; do
        for c in ${AB:-c2}; do
            for v in ${EMITV:--1}; do
                SMOLCSUM_LIB=$GRAFT_REPO_ROOT/smoltcp_amd/libsmolcsum_exp.so step ab_${c}_${v}_$rnd 300 python bench.py --config $c --steps 30 --warmup 5 --cpu-seconds 0 --emit-variant $v
            done
        done
    done
fi
echo "== done ($(date +%T))"
