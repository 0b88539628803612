# C5 (2^27 x 1500 B = 201 GB in one HBM buffer) bench at full size, and the c2copy profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c5
mkdir -p $O
echo "== c5 ($(date +%T))"
timeout -k 10 500 python bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 10 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
echo "== c2copy bench ($(date +%T))"
timeout -k 10 300 python bench.py --config c2copy > $O/bench_c2copy.json 2> $O/bench_c2copy.err || { tail -20 $O/bench_c2copy.err; exit 1; }
cat $O/bench_c2copy.json
echo "== c2copy kernel trace ($(date +%T))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/c2copy/kt -o run -- python3 bench.py --config c2copy --steps 20 > $O/kt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/c2copy/fetch -o run -- python3 bench.py --config c2copy --steps 5 --warmup 1 > $O/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/c2copy/write -o run -- python3 bench.py --config c2copy --steps 5 --warmup 1 > $O/write.log 2>&1 || exit 1
echo "== done ($(date +%T))"
