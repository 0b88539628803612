# Round 5: A/B of two product builds (smoltcp_amd/libsmolcsum_base.so = before, the in-tree library =
# after) with tools/exp_r05_emit.py (default variants: emit and verify as the library picks them),
# libraries in turn, REPS times.  Usage: gpurun -- 'bash tools/gpu_r05_libab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5libab}; mkdir -p $O
for i in $(seq 1 ${REPS:-2}); do
    for L in base new; do
        if [ $L = base ]; then lib=$PWD/smoltcp_amd/libsmolcsum_base.so; else lib=$PWD/smoltcp_amd/libsmolcsum.so; fi
        SMOLCSUM_LIB=$lib VARS=${VARS:--1} ROUNDS=3 timeout -k 10 200 python tools/exp_r05_emit.py ${CFGS:-c2,c4} > $O/${L}_$i.jsonl 2>&1 || { tail -20 $O/${L}_$i.jsonl; exit 1; }
        echo "== $L $i"; python tools/summ_emit.py $O/${L}_$i.jsonl
    done
done
