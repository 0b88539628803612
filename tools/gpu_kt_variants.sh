# Kernel traces of bench.py lines per emit variant (experiments build): rocprofv3 --kernel-trace --stats.
# Usage: gpurun -- 'OUT=gpurun_out/x CFGS="c2" EMITV="80 57" bash tools/gpu_kt_variants.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/ktv}
mkdir -p $O
for c in ${CFGS:-c2}; do
    for v in ${EMITV:-80}; do
        echo "== $c $v ($(date +%T))"
        SMOLCSUM_LIB=$GRAFT_REPO_ROOT/smoltcp_amd/libsmolcsum_exp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c/$v -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 0 --emit-variant $v > $O/${c}_$v.log 2>&1 || { tail -20 $O/${c}_$v.log; exit 1; }
        f=$(find $O/$c/$v -name "*kernel_stats.csv" | head -1)
        python3 - "$f" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    n = row.get("Name") or row.get("KernelName")
    print(f"   {n[:90]:90s} calls={row['Calls']:>6s} avg_us={float(row['AverageNs'])/1000:9.2f}")
PY
    done
done
echo "== done ($(date +%T))"
