# Round 6: copy-emit's L2 <-> memory requests: per launch of copy_kernel (and the
# C2 emit / verify kernels for reference), in separate rocprofv3 --pmc passes of at most 4 TCC
# counters: read requests by size, write requests by size, L2 hits / misses; and FETCH_SIZE /
# WRITE_SIZE with the payload source packed (1472-B stride) and line-aligned (1536).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/copypmc}
mkdir -p $O
pass() {  # pass <name> <extra bench args> -- <counters...>
    local name=$1 extra=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 bench.py --config c2copy --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0 $extra > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
}
pass rd "" TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum
pass wr "" TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
pass hit "" TCC_HIT_sum TCC_MISS_sum
pass fetch "" FETCH_SIZE
pass write "" WRITE_SIZE
pass fetch1536 "--src-stride 1536" FETCH_SIZE
pass write1536 "--src-stride 1536" WRITE_SIZE
pass rd1536 "--src-stride 1536" TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum
for d in rd wr hit fetch write fetch1536 write1536 rd1536; do
    echo "-- $d"; python3 tools/pmc_kernels.py $O/$d copy_kernel || true; python3 tools/pmc_kernels.py $O/$d xwalk || true
done > $O/summary.txt 2>&1
cat $O/summary.txt
echo "== done ($(date +%T))"
