# Round 5: L2 counters of C2 emit, the walk kernel (variant 39) against the transposed walk (47):
# hits / misses and memory-side write and read requests, one rocprofv3 --pmc pass per counter set.
# Usage: gpurun -- 'bash tools/gpu_r05_emit_pmc.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_exp.so
O=gpurun_out/epmc; mkdir -p $O
for v in 39 47; do
    i=0
    for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
        i=$((i+1))
        timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/v$v/p$i -o run -- python3 bench.py --config c2 --variant $v --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0 > $O/v${v}_p$i.log 2>&1 || { tail -5 $O/v${v}_p$i.log; exit 1; }
        echo "v$v p$i done"
    done
done
