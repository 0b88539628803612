# Round 6: descriptor-emit choice tests, copy-emit variant 98's L2 requests and timing, C3 default line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6b2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-descriptor_emit_choice or dwalk_descriptor or staged or last_launch or kernel_for or dispatch_table or forced_copy or copy_emit}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 21 98; do
  SMOLCSUM_LIB=$GRAFT_REPO_ROOT/smoltcp_amd/libsmolcsum_exp.so timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum --output-format csv -d $O/rd$v -o run -- python3 bench.py --config c2copy --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0 --variant $v > $O/rd$v.log 2>&1 || { tail -20 $O/rd$v.log; exit 1; }
  python3 tools/pmc_kernels.py $O/rd$v copy_kernel
done
for r in 1 2; do for v in 21 98; do
  SMOLCSUM_LIB=$GRAFT_REPO_ROOT/smoltcp_amd/libsmolcsum_exp.so timeout -k 10 200 python bench.py --config c2copy --steps 30 --warmup 5 --cpu-seconds 0 --variant $v > $O/ab$v_$r.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/ab$v_$r.log').read().strip().splitlines()[-1]); print($v, d['value'], d['kernels_ms'], d['kernels_launched'])"
done; done
timeout -k 10 200 python bench.py --config c3 --cpu-seconds 0 > $O/c3.log 2>&1 && python3 -c "import json; d=json.loads(open('$O/c3.log').read().strip().splitlines()[-1]); print('c3', d['value'], d['kernels_ms'], d['kernels_launched'])"
