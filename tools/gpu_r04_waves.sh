# Round 4: C2 verify held to 5 waves per SIMD (variant 31, 96 VGPRs + 32 B of spills, against
# variant 5's 109 VGPRs, 4 waves) and emit held to 5 waves (variant 32 against 29), interleaved;
# the fixed-stride variant parity tests first.  Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_waves.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4waves}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "variants_fixed_stride and (31 or 32)" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/sweep.py --config c2 --shapes 7 --var 29,32,5,31 --rounds 4 > $O/sweep_c2.log 2>&1 || { tail -20 $O/sweep_c2.log; exit 1; }
grep '"round"' $O/sweep_c2.log
echo "== done ($(date +%T))"
