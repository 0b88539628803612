# Round 4: what C2 / C4 emit costs without its field stores.  smoltcp_amd/libsmolcsum_nostore.so is
# the library with csum_walk_emit_fixed.hip built with -DSMOL_EXP_NOSTORE (field values computed,
# nothing stored; wrong bytes, timing only).  Both libraries run in turn: emit and verify of one C2 /
# C4 buffer (tools/exp_inplace.py "emit" / "verify" sequences, tools/exp_emit_seg.py for C4).
# Build first (CPU): bash tools/gpu_r04_nostore.sh build.  Usage: gpurun -- 'bash tools/gpu_r04_nostore.sh'
set -o pipefail
if [ "$1" = build ]; then
    cd "$(dirname "$0")/../smoltcp_amd/csrc" || exit 1
    mkdir -p build_nostore
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSMOL_EXP_NOSTORE -c csum_walk_emit_fixed.hip \
        -o build_nostore/csum_walk_emit_fixed.hip.o || exit 1
    objs=$(ls build/*.o | grep -v csum_walk_emit_fixed)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../libsmolcsum_nostore.so $objs build_nostore/csum_walk_emit_fixed.hip.o
    exit $?
fi
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4nostore}; mkdir -p $O
for i in 1 2; do
    for L in base nostore; do
        if [ $L = base ]; then lib=$PWD/smoltcp_amd/libsmolcsum.so; else lib=$PWD/smoltcp_amd/libsmolcsum_nostore.so; fi
        SMOLCSUM_LIB=$lib ROUNDS=3 timeout -k 10 200 python tools/exp_inplace.py 1048576 emit,verify > $O/c2_${L}_$i.log 2>&1 || { tail -20 $O/c2_${L}_$i.log; exit 1; }
        SMOLCSUM_LIB=$lib NOCHECK=29 VARS_c4=29 timeout -k 10 200 python tools/exp_emit_seg.py c4 > $O/c4_${L}_$i.log 2>&1 || { tail -20 $O/c4_${L}_$i.log; exit 1; }
    done
done
grep -H '"round": [12]' $O/*.log
