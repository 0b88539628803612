# SQ instruction / cycle counters per kernel of one bench config (one rocprofv3 pass).
# Usage: gpurun -- 'CFG=c2copy KF=smolcsum bash tools/gpu_pmc_sq.sh'  (KF: kernel-name filter of the summary, default csum_)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmc_sq; mkdir -p $O
CFG=${CFG:-c2copy}
SQ=${SQ:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY}
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/$CFG -o run -- python3 bench.py --config $CFG --steps 5 --warmup 1 --cpu-seconds 0 > $O/$CFG.log 2>&1 || { tail -20 $O/$CFG.log; exit 1; }
python3 tools/pmc_kernels.py $O/$CFG ${KF:-csum_}
