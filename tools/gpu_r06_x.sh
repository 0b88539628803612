set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6x
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6x/tests.log 2>&1; rc=$?
tail -4 gpurun_out/r6x/tests.log
[ $rc -eq 0 ] || exit $rc
SMOLCSUM_LIB=$GRAFT_REPO_ROOT/smoltcp_amd/libsmolcsum_exp.so VARS=41,94 timeout -k 10 400 python tools/exp_r06_desc_step.py > gpurun_out/r6x/desc_step.jsonl && cat gpurun_out/r6x/desc_step.jsonl
