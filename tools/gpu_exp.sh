# Ad-hoc experiment pass on the GPU box.  Usage: gpurun -- 'bash tools/gpu_exp.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/exp
mkdir -p $O
for v in 1 9 10 11 12 1 9; do
    timeout -k 10 300 python bench.py --config c2copy --cpu-seconds 0 --variant $v > $O/c2copy_$v.log 2>&1 || { echo "rc=$?"; tail -20 $O/c2copy_$v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2copy_$v.log').read().strip().splitlines()[-1]); print('var $v', d['value'], d['kernels_ms'])"
done
echo "== done"
