set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM --output-format csv -d gpurun_out/pmc2/a -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc2/a.log 2>&1; echo "rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc2/b -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc2/b.log 2>&1; echo "rc=$?"
