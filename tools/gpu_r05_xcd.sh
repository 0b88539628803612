# Round 5: the XCD-contiguous block order (--xcd-remap 1) against the dispatch order for copy-emit
# (C2copy) and the C2 step, bench lines over rotating batches, interleaved.  REPS (default 3).
# Usage: gpurun -- 'bash tools/gpu_r05_xcd.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5xcd}; mkdir -p $O
for i in $(seq 1 ${REPS:-3}); do
    for c in ${CFGS:-c2copy c2}; do
        for x in 0 1; do
            timeout -k 10 120 python bench.py --config $c --xcd-remap $x --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_${c}_x${x}_$i.json 2> $O/b_${c}_x${x}_$i.err || { tail -5 $O/b_${c}_x${x}_$i.err; exit 1; }
            python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], 'xcd', sys.argv[3], d['value'], d['kernels_ms'])" $O/b_${c}_x${x}_$i.json $c $x
        done
    done
done
