# FETCH_SIZE / WRITE_SIZE per copy-emit variant (tools/exp_copy.py, C2copy), one rocprofv3 pass each.
# Usage: gpurun -- 'VARS="11 14" bash tools/gpu_pmc_copy.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmc_copy; mkdir -p $O
for v in ${VARS:-11 14}; do
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/$v/$c -o run -- python3 tools/exp_copy.py ${SHAPE:-0} $v > $O/$v.$c.log 2>&1 || { tail -20 $O/$v.$c.log; exit 1; }
        echo "== variant $v $c"; python3 tools/pmc_kernels.py $O/$v/$c csum_kernel
    done
done
