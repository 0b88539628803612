# Where copy-emit's extra reads come from: the L2's memory-side read requests by size, hit / miss,
# for copy_kernel (variant 17) and, as the calibration of a known byte count, the C2 verify kernel
# (16-B aligned streaming loads: FETCH_SIZE x 2 = the bytes, MI355X_MICROARCH.md).
# Usage: gpurun -- 'bash tools/gpu_copy_pmc.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/cpmc; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -oE "TCC_EA0_RD[A-Z0-9_]*|TCC_EA0_WR[A-Z0-9_]*|TCC_(HIT|MISS)[A-Z0-9_]*|TCP_TCC_[A-Z_]*REQ[A-Z0-9_]*" $O/avail.txt | sort -u > $O/tcc_names.txt || true
cat $O/tcc_names.txt | tr '\n' ' '; echo
i=0
for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/exp_copy.py 8 17 > $O/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $O/p$i.log; continue; }
    python3 tools/pmc_kernels.py $O/p$i copy_kernel
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/v$i -o run -- python3 tools/sweep.py --config c2 --shapes 7 --var 5 --reps 3 --rounds 1 > $O/v$i.log 2>&1 || { echo "verify pass $i failed"; continue; }
    python3 tools/pmc_kernels.py $O/v$i "csum_kernel<8, 7, 2"
done
