# Round-3 pass for the whole-segment emit default (variant 19): emit A/B (5 vs 19, parity tests of
# test_gpu_parity.py first), then the full GPU suite, smoke and the bench lines.
# Usage: gpurun --timeout 1500 -- 'bash tools/gpu_r03g.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_emit_seg.sh && OUT=gpurun_out/r3g STAGES="tests bench" bash tools/gpu_round3.sh
