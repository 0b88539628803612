# Interleaved A/B of bench.py lines (experiments build): VARIANTS is a ';'-separated list of extra
# bench.py arguments, each run ROUNDS times in turn for every config in AB.
# Usage: gpurun -- 'OUT=gpurun_out/x AB="c2" VARIANTS="--emit-variant 57;--emit-variant 83" bash tools/gpu_ab_args.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/ab}
mkdir -p $O
IFS=';' read -r -a VS <<< "${VARIANTS:---variant -1}"
for rnd in $(seq 1 ${ROUNDS:-2}); do
    for c in ${AB:-c2}; do
        for i in "${!VS[@]}"; do
            v=${VS[$i]}
            echo "== $c [$v] round $rnd ($(date +%T))"
            SMOLCSUM_LIB=$GRAFT_REPO_ROOT/smoltcp_amd/libsmolcsum_exp.so timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --cpu-seconds 0 $v > $O/${c}_${i}_$rnd.log 2>&1 || { tail -20 $O/${c}_${i}_$rnd.log; exit 1; }
            python3 - $O/${c}_${i}_$rnd.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"   {d['value']:8.1f} GiB/s  step {d['ms_per_step']:.4f}  kernels {d['kernels_ms']}  {d['kernels_launched']}")
PY
        done
    done
done
echo "== done ($(date +%T))"
