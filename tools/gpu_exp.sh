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
kstats() {
    python3 - $1 <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "csum" in r["Name"] or "scatter" in r["Name"]:
        print("   ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
}
for lib in default NOSLOT SLOT64; do
    L=smoltcp_amd/libsmolcsum.so; [ $lib != default ] && L=build_alt/lib_$lib.so
    SMOLCSUM_LIB=$L step kt_$lib 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$lib -o run -- python3 bench.py --config c2 --steps 20 --cpu-seconds 0 --variant 5 --defer 1 --shape 7
    kstats $O/kt_$lib
done
echo "== done"
