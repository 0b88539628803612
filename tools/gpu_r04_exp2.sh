# Round 4: emit variant 30 (nt segment stores) against 29 / 19 / 5, the emit launch shapes of
# variant 29 on C2 / C4, and the XCD-order grain sweep (tools/gpu_r04_xcd3.sh).
# Usage: gpurun --timeout 1200 -- 'bash tools/gpu_r04_exp2.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4exp2}
mkdir -p $O
echo "== variants ($(date +%T))"
VARS=29,30,19,5 timeout -k 10 300 python tools/exp_emit_seg.py c2,c4 > $O/variants.log 2>&1 || { tail -20 $O/variants.log; exit 1; }
echo "== shapes ($(date +%T))"
for c in c2 c4; do timeout -k 10 300 python tools/sweep.py --config $c --shapes 0,7,1,8,2 --var 29 --rounds 3 > $O/shapes_$c.log 2>&1 || { tail -20 $O/shapes_$c.log; exit 1; }; done
echo "== xcd grain ($(date +%T))"
OUT=$O/xcd3 bash tools/gpu_r04_xcd3.sh
echo "== done ($(date +%T))"
