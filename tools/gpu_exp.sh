# Ad-hoc experiment pass on the GPU box.  Usage: gpurun -- 'bash tools/gpu_exp.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/exp
mkdir -p $O
for rep in 1 2 3; do
for c in c2 c4; do
    for lib in new alt; do
        if [ $lib = alt ]; then export SMOLCSUM_LIB=$PWD/build_alt/libsmolcsum.so; else unset SMOLCSUM_LIB; fi
        timeout -k 10 300 python bench.py --config $c --cpu-seconds 0 > $O/ab_${c}_${lib}.log 2>&1 || { echo "rc=$?"; tail -20 $O/ab_${c}_${lib}.log; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/ab_${c}_${lib}.log').read().strip().splitlines()[-1]); print('$rep $c $lib', d['value'], d['kernels_ms'])"
    done
done
done
echo "== done"
