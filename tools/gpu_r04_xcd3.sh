# Round 4: the XCD block order at several grains (xcd_chunk: runs of K workgroups per XCD turn;
# 0 dispatch order, 1 contiguous) for emit alone and verify alone at 2^20, 2^24 and 2^26 records.
# Usage: gpurun --timeout 1200 -- 'bash tools/gpu_r04_xcd3.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4xcd3}
mkdir -p $O
for k in ${KS:-0 1 4 16 64 256}; do
    echo "== K=$k ($(date +%T))"
    XCD_EMIT=$k XCD_VERIFY=$k SIZES=${SZ:-20,24,26} ROUNDS=3 timeout -k 10 400 python tools/exp_inplace.py 0 emit,verify > $O/k$k.log 2>&1 || { tail -20 $O/k$k.log; exit 1; }
done
echo "== done ($(date +%T))"
