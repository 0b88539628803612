# Round 4: C5-sized in-place step (2^27 records, one 201-GB buffer) with emit in the XCD order and
# verify at several grains of it (0 dispatch order, K = 64 / 256 / 1024 workgroups per XCD turn).
# Usage: gpurun --timeout 900 -- 'bash tools/gpu_r04_c5verify.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4c5v}
mkdir -p $O
for k in 0 64 256 1024; do
    echo "== verify K=$k ($(date +%T))"
    XCD_EMIT=1 XCD_VERIFY=$k SIZES=27 ROUNDS=3 K=5 timeout -k 10 400 python tools/exp_inplace.py 0 inplace > $O/k$k.log 2>&1 || { tail -20 $O/k$k.log; exit 1; }
    grep '"round": 2' $O/k$k.log
done
echo "== done ($(date +%T))"
