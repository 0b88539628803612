# Round 5: the walk kernel at wider group shapes (one load step per record) against the defaults,
# bench lines over rotating batches, interleaved.  PAIRS: "variant shape" pairs.
# Usage: gpurun -- 'bash tools/gpu_r05_shapes.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5shapes}; mkdir -p $O
[ -n "$EXP" ] && export SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_exp.so
for i in $(seq 1 ${REPS:-2}); do
    for c in ${CFGS:-c2 c4}; do
        for vs in ${PAIRS:-"-1,-1" "13,4" "5,4" "13,2" "5,2" "13,8" "5,8"}; do
            v=${vs%,*}; sh=${vs#*,}
            timeout -k 10 120 python bench.py --config $c --variant $v --shape $sh --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_${c}_${v}_${sh}_$i.json 2> $O/b_${c}_${v}_${sh}_$i.err || { tail -5 $O/b_${c}_${v}_${sh}_$i.err; exit 1; }
            python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], 'var', sys.argv[3], 'shape', sys.argv[4], d['value'], d['kernels_ms'])" $O/b_${c}_${v}_${sh}_$i.json $c $v $sh
        done
    done
done
