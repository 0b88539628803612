# Round 5: cached header lines on fixed-stride batches: the transposed walk with each record's first
# KiB loaded cached (variant 45) and the descriptor walk over fixed strides (62 / 63), against the
# defaults; parity first.  Usage: gpurun -- 'bash tools/gpu_r05_cached_fixed.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/cf}; mkdir -p $O
EXP=$PWD/smoltcp_amd/libsmolcsum_exp.so
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "wide or variants_fixed or dwalk" -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
fi
for i in 1 2; do
for cv in ${BENCH:-c2:-1 c2:45 c2:63 c2:62 c4:-1 c4:45 c4:63}; do
    c=${cv%%:*}; v=${cv##*:}
    SMOLCSUM_LIB=$EXP timeout -k 10 200 python -u bench.py --config $c --variant $v --steps 30 --warmup 5 --cpu-seconds 0 > $O/b_${c}_${v}_$i.json 2> $O/b_${c}_$v.err || { tail -5 $O/b_${c}_$v.err; exit 1; }
done
done
