# Round 5: FETCH_SIZE / WRITE_SIZE of copy-emit variant 21 against the transposed layout (49, 52 = 49
# without body stores, 55 = walk-shaped stores) on C2copy, one pass per counter.
# Usage: gpurun -- 'bash tools/gpu_r05_xcopy_pmc.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_exp.so NOCHECK=52 ROUNDS=1 K=4
mkdir -p gpurun_out/xcp
for k in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $k --output-format csv -d gpurun_out/xcp/$k -o run -- python3 tools/exp_copy.py 8 21,49,55,52 > gpurun_out/xcp/$k.log 2>&1 || { tail -5 gpurun_out/xcp/$k.log; exit 1; }
done
