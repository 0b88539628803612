# Round 6: full GPU suite + bench lines on the current tree, then C4 emit / verify variant A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/r7d} STAGES="tests bench" bash tools/gpu_r06.sh || exit 1
OUT=${OUT:-gpurun_out/r7d} AB="c4" ROUNDS=2 VARIANTS="--variant -1;--emit-variant 39;--emit-variant 81;--emit-variant 80;--verify-variant 47;--verify-variant 89" bash tools/gpu_ab_args.sh
