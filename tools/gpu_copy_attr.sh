# Where copy-emit's time goes: the default build against builds with one part of the per-record work
# removed (build_alt/libsmolcsum_expN.so: 1 = fixed geometry instead of the parse, 2 = no gates /
# field writes, 3 = window chunks stored whole without byte masks).  Outputs are NOT correct in the
# experiment builds; timing only.  Usage: gpurun -- 'bash tools/gpu_copy_attr.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/copy_attr; mkdir -p $O
for L in base 1 2 3; do
    if [ $L = base ]; then lib=$PWD/smoltcp_amd/libsmolcsum.so; else lib=$PWD/build_alt/libsmolcsum_exp$L.so; fi
    SMOLCSUM_LIB=$lib timeout -k 10 120 python tools/exp_copy.py ${SHAPES:-8} 17 > $O/$L.log 2>&1 || { tail -20 $O/$L.log; exit 1; }
    echo "== $L"; grep '"round": 2' $O/$L.log
done
