set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu"; timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
for c in c2 c3 c4; do
echo "== bench $c"; timeout -k 10 300 python bench.py --config $c --cpu-seconds 3 --probe > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err; rc=$?; cat gpurun_out/bench_$c.json; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_$c.err; exit $rc; fi
done
echo "== sweep c3"; timeout -k 10 600 python tools/sweep.py --config c3 --blocks 0 --var 0,1 --shapes 2,4,5,6 --defer 0 > gpurun_out/sweep_c3.log 2>&1; rc=$?; grep '"round": 1' gpurun_out/sweep_c3.log | cut -c1-200; echo "sweep rc=$rc"
echo "== sweep c4"; timeout -k 10 600 python tools/sweep.py --config c4 --blocks 0 --var 0,1 --shapes 0,2,4 --defer 0 > gpurun_out/sweep_c4.log 2>&1; rc=$?; grep '"round": 1' gpurun_out/sweep_c4.log | cut -c1-200; echo "sweep rc=$rc"
