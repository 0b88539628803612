# Round 5: bench lines with emit and verify variants forced separately (bench.py --emit-variant /
# --verify-variant), two interleaved rounds.  BENCH: config:emit_variant:verify_variant ...
# Usage: gpurun -- 'BENCH="c2:-1:-1 c2:45:-1" bash tools/gpu_r05_split.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/sp}; mkdir -p $O
EXP=$PWD/smoltcp_amd/libsmolcsum_exp.so
for i in 1 2; do
for cv in $BENCH; do
    IFS=: read c e v <<< "$cv"
    SMOLCSUM_LIB=$EXP timeout -k 10 200 python -u bench.py --config $c --emit-variant $e --verify-variant $v --steps 30 --warmup 5 --cpu-seconds 0 > $O/b_${c}_${e}_${v}_$i.json 2> $O/err || { tail -5 $O/err; exit 1; }
done
done
