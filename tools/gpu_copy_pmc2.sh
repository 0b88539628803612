# Read requests by size and by destination (DRAM vs the rest) for copy_kernel and C2 verify.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/cpmc2; mkdir -p $O
i=0
for set in "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum" "TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/exp_copy.py 8 17 > $O/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $O/p$i.log; continue; }
    python3 tools/pmc_kernels.py $O/p$i copy_kernel
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/v$i -o run -- python3 tools/sweep.py --config c2 --shapes 7 --var 5 --reps 3 --rounds 1 > $O/v$i.log 2>&1 || { echo "verify pass $i failed"; continue; }
    python3 tools/pmc_kernels.py $O/v$i "csum_kernel<8, 7"
done
