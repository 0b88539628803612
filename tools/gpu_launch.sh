# The bench launcher's GPU tests (plain --gpus 1 and a one-rank torch.distributed.run over RCCL),
# then the C2 bench line at the driver's flags with the CPU baseline (cgroup throttling counters).
# Usage: gpurun -- 'bash tools/gpu_launch.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/launch; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -4 $O/tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-400
timeout -k 10 300 python tools/exp_tail.py > $O/tail.log 2>&1 || { tail -20 $O/tail.log; exit 1; }
grep round $O/tail.log
