# Round 4: C3 emit (tile kernel, variant 7) launch shapes and tile sizes, and C3 verify (variant 13)
# shapes, at steady clocks (tools/sweep.py).  Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_c3sweep.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4c3sweep}
mkdir -p $O
timeout -k 10 400 python tools/sweep.py --config c3 --shapes 0,1,2,3,4 --var 7 --tile 32,64 --rounds 2 > $O/tile.log 2>&1 || { tail -20 $O/tile.log; exit 1; }
timeout -k 10 400 python tools/sweep.py --config c3 --shapes 1,8,2,3,4 --var 13 --rounds 2 > $O/walk13.log 2>&1 || { tail -20 $O/walk13.log; exit 1; }
grep '"round": 1' $O/tile.log $O/walk13.log | cut -d: -f2- | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['var'], d['shape'], d['tile'], d['emit_ms'], d['verify_ms'])"
echo "== done ($(date +%T))"
