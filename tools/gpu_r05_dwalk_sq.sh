# Round 5: SQ counters of C3 verify / emit, the walk / tile kernels (default) against the transposed
# walk over descriptor batches (variant 56, experiments build).  Usage: gpurun -- 'bash tools/gpu_r05_dwalk_sq.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_exp.so
O=gpurun_out/dwsq; mkdir -p $O
for v in -1 56; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $O/v$v -o run -- python3 bench.py --config c3 --variant $v --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0 > $O/v$v.log 2>&1 || { tail -5 $O/v$v.log; exit 1; }
done
