set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmcvar
mkdir -p $O
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/v$v -o run -- python3 bench.py --variant $v --steps 5 --warmup 1 --cpu-seconds 0 > $O/v$v.log 2>&1 || exit 1
  tail -1 $O/v$v.log | cut -c1-300
done
