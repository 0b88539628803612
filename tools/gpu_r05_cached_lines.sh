# Round 5: header lines loaded cached so that emit's field stores hit lines the L2 holds.
# Parity of the new variants (walk 12 / 14, descriptor walk 61-63), then descriptor-batch emit
# timing (tools/exp_r05_desc.py) and bench lines of C3 / C2 / C4 with the variants forced.
# Usage: gpurun -- 'bash tools/gpu_r05_cached_lines.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/cl}; mkdir -p $O
EXP=$PWD/smoltcp_amd/libsmolcsum_exp.so
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segments.py -k "dwalk or variants_fixed or write_set or field_stores" -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
fi
SMOLCSUM_LIB=$EXP VARS=${DVARS:--1,62,63} CASES=${DCASES:-c3_packed,c3_gapped,c3_shuffled,short_packed,fixed1500} timeout -k 10 400 python -u tools/exp_r05_desc.py > $O/desc.jsonl 2>&1 || { tail -5 $O/desc.jsonl; exit 1; }
for cv in ${BENCH:-c3:-1 c3:62 c3:63 c2:-1 c2:12 c2:14 c4:-1 c4:12}; do
    c=${cv%%:*}; v=${cv##*:}
    SMOLCSUM_LIB=$EXP timeout -k 10 200 python -u bench.py --config $c --variant $v --steps 30 --warmup 5 --cpu-seconds 0 > $O/b_${c}_$v.json 2> $O/b_${c}_$v.err || { tail -5 $O/b_${c}_$v.err; exit 1; }
done
