set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
echo "== bench"; timeout -k 10 300 python bench.py --probe > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err; rc=$?; cat gpurun_out/bench_r01.json; echo "bench rc=$rc"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_r01.err; exit $rc; fi
echo "== rocprof kernel trace"; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o run -- python3 bench.py --steps 20 --cpu-seconds 0 > gpurun_out/prof/kt.log 2>&1; rc=$?; echo "kt rc=$rc"; tail -3 gpurun_out/prof/kt.log
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== rocprof FETCH_SIZE"; timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/prof/fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"; tail -3 gpurun_out/prof/fetch.log
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== rocprof WRITE_SIZE"; timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/prof/write.log 2>&1; rc=$?; echo "write rc=$rc"; tail -3 gpurun_out/prof/write.log
find gpurun_out/prof -name "*.csv" | head -20
