# Launch-shape / variant sweep at steady clocks (tools/sweep.py ramps first): are the defaults,
# chosen by round-1/2 sweeps without a clock ramp, still the fastest?
# Usage: gpurun -- 'bash tools/gpu_sweep3.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sweep3; mkdir -p $O
timeout -k 10 400 python tools/sweep.py --config c2 --shapes 0,7,1,8,2 --var 5,0,6 --reps 15 --rounds 2 > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
timeout -k 10 400 python tools/sweep.py --config c4 --shapes 0,7,1,8 --var 5,0,6 --reps 15 --rounds 2 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
timeout -k 10 400 python tools/sweep.py --config c3 --shapes 1,8,2 --var 13,5,7 --reps 10 --rounds 2 > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
for c in c2 c4 c3; do
    echo "== $c"
    python3 - "$O/$c.log" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{") and '"round": 1' in l]
for k in ("emit_ms", "verify_ms"):
    best = sorted(rows, key=lambda r: r[k])[:4]
    print(k, [(r["shape"], r["var"], r[k]) for r in best])
PY
done
