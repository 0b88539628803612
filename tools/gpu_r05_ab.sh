# Round 5: bench lines (rotating batches) with forced emit variants from the experiments build,
# interleaved.  VARS (default 29 37 38), CFGS (default c2 c4), REPS (default 3).
# Usage: gpurun -- 'bash tools/gpu_r05_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5ab}; mkdir -p $O
export SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_exp.so
for i in $(seq 1 ${REPS:-3}); do
    for c in ${CFGS:-c2 c4}; do
        for v in ${VARS:-29 38 39}; do
            timeout -k 10 120 python bench.py --config $c --variant $v --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_${c}_${v}_$i.json 2> $O/b_${c}_${v}_$i.err || { tail -5 $O/b_${c}_${v}_$i.err; exit 1; }
            python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['kernels_ms'], (d.get('emit_same_batch') or {}).get('emit_ms'))" $O/b_${c}_${v}_$i.json $c $v
        done
    done
done
