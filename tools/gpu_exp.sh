# Ad-hoc experiment pass on the GPU box.  Usage: gpurun -- 'bash tools/gpu_exp.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/exp
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>: stop on the first failure
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
    tail -${TAILN:-1} "$O/$name.log"
}
for lib in default w5 w6; do
L=smoltcp_amd/libsmolcsum.so; [ $lib != default ] && L=build_alt/lib_$lib.so
for c in c2 c4 c3; do
    SMOLCSUM_LIB=$L step bench_${c}_$lib 300 python bench.py --config $c --cpu-seconds 0
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${c}_$lib.log').read().strip().splitlines()[-1]); print('   ', '$lib', '$c', d['value'], d['unit'], d['kernels_ms'])"
done
done
echo "== done"
