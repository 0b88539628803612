# Kernel trace of tools/probe_wtax (per-kernel split of its multi-launch forms).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/ktp}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- tools/probe_wtax ${WTAX_N:-1048576} ${WTAX_L:-1500} 1 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    n = row.get("Name") or row.get("KernelName")
    print(f"   {n[:110]:110s} calls={row['Calls']:>6s} avg_us={float(row['AverageNs'])/1000:9.2f}")
PY
