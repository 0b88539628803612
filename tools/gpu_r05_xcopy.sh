# Round 5: copy-emit on the transposed layout (variants 49 / 50, experiments build): its tests, C2copy timing
# against variant 21, SQ counters.  Usage: gpurun -- 'bash tools/gpu_r05_xcopy.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_exp.so
mkdir -p gpurun_out/xc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_copy_emit.py -k "xcopy or fixed_stride" > gpurun_out/xc/t.log 2>&1 || { tail -30 gpurun_out/xc/t.log; exit 1; }
tail -1 gpurun_out/xc/t.log
ROUNDS=3 timeout -k 10 200 python -u tools/exp_copy.py 8 21,49,50 > gpurun_out/xc/e.jsonl 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d gpurun_out/xc/sq -o run -- python3 tools/exp_copy.py 8 21,49 > gpurun_out/xc/sq.log 2>&1 || exit 1
