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
TAILN=3 step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for lib in default NOSHARE; do
L=smoltcp_amd/libsmolcsum.so; [ $lib != default ] && L=build_alt/lib_$lib.so
for c in c2 c4; do
    SMOLCSUM_LIB=$L TAILN=0 step sweep_${c}_$lib 600 python tools/sweep.py --config $c --shapes 0,7 --var 1,5 --defer 0
    grep '"round": 1' $O/sweep_${c}_$lib.log | cut -c1-140
done
done
echo "== done"
