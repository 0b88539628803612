# Round 5: SQ instruction / wait counters of emit variants (experiments build), one rocprofv3 pass per
# counter set over tools/exp_r05_emit.py (C2, one round).  VARS (default 69,101,103 = 5 / 37 / 39
# without stores).  Usage: gpurun -- 'bash tools/gpu_r05_sq.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5sq}; mkdir -p $O
export SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_exp.so
V=${VARS:-69,101,103}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
i=0
for set in "$P1" "$P2"; do
    i=$((i+1))
    VARS=$V ROUNDS=2 K=8 timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/exp_r05_emit.py c2 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
    python3 tools/pmc_kernels.py $O/p$i csum_kernel > $O/p$i.txt
done
cat $O/p1.txt $O/p2.txt | cut -c1-600
