# CPU-baseline stability: two back-to-back C2 benches at the driver's flags (the baseline leg on).
# Usage: gpurun -- 'bash tools/gpu_cpub.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cpub; mkdir -p $O
for i in 1 2; do
    timeout -k 10 250 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_$i.json 2> $O/c2_$i.err || { tail -20 $O/c2_$i.err; exit 1; }
done
python3 - <<'PY'
import json
for i in (1, 2):
    d = json.loads(open(f"gpurun_out/cpub/c2_{i}.json").read().strip().splitlines()[-1])
    c = d["cpu_baseline"]
    keys = ("value", "single_core_value", "spread_p10_p90", "pass_rate_p10_p50_p90",
            "single_core_pass_rate_p10_p50_p90", "pinned_cpus", "numa_nodes")
    print(d["value"], {k: c[k] for k in keys}, d["parity_sample"])
PY
