set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc1
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc1/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" gpurun_out/pmc1/counters.txt | sort -u > gpurun_out/pmc1/sq_counters.txt || true
wc -l gpurun_out/pmc1/sq_counters.txt
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d gpurun_out/pmc1/a -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc1/a.log 2>&1; echo "rc=$?"
