# Counters per kernel of tools/exp_copy.py for one copy variant (VAR), one rocprofv3 pass per set.
# Usage: gpurun -- 'VAR=16 bash tools/gpu_pmc_exp.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmc_exp; mkdir -p $O
V=${VAR:-16}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/$V/$i -o run -- python3 tools/exp_copy.py ${SHAPE:-0} $V > $O/$V.$i.log 2>&1 || { tail -20 $O/$V.$i.log; exit 1; }
    python3 tools/pmc_kernels.py $O/$V/$i _kernel
done
