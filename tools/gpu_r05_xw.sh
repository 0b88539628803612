# Round 5: HBM traffic of the transposed walk's emit / verify against the walk kernel's (C2 / C4 bench
# lines with a forced variant from the experiments build): one FETCH_SIZE and one WRITE_SIZE pass each.
# VARS (default 39 44 47), CFGS (default c2 c4).  Usage: gpurun -- 'bash tools/gpu_r05_xw.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5xw}; mkdir -p $O
export SMOLCSUM_LIB=$PWD/smoltcp_amd/libsmolcsum_exp.so
for c in ${CFGS:-c2 c4}; do
    for v in ${VARS:-39 44 47}; do
        for k in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 120 rocprofv3 --pmc $k --output-format csv -d $O/$c/$v/$k -o run -- python3 bench.py --config $c --variant $v --steps 8 --warmup 2 --ramp-ms 0 --cpu-seconds 0 > $O/${c}_${v}_$k.log 2>&1 || { tail -5 $O/${c}_${v}_$k.log; exit 1; }
            echo "$c $v $k done"
        done
    done
done
