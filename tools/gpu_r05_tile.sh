# Round 5: the tile kernel (variant 7) on fixed-stride batches at the wide group shapes (a whole
# wavefront streams one record at a time: 1 KiB per load instruction), against the defaults;
# bench lines over rotating batches, interleaved.  Usage: gpurun -- 'bash tools/gpu_r05_tile.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5tile}; mkdir -p $O
for i in $(seq 1 ${REPS:-2}); do
    for c in ${CFGS:-c2 c4}; do
        for vs in "-1 -1" "7 5" "7 6" "7 4" "7 8"; do
            set -- $vs
            timeout -k 10 120 python bench.py --config $c --variant $1 --shape $2 --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_${c}_$1_$2_$i.json 2> $O/b_${c}_$1_$2_$i.err || { tail -5 $O/b_${c}_$1_$2_$i.err; exit 1; }
            python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], 'var', sys.argv[3], 'shape', sys.argv[4], d['value'], d['kernels_ms'])" $O/b_${c}_$1_$2_$i.json $c $1 $2
        done
    done
done
