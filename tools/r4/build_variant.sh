#!/bin/bash
# build_variant.sh NAME "-DFLAG=.. ..." [UNIT ...] -> qwen3-asr.cpp_amd/var_NAME.so: libqasr.so with the given
# csrc units (default attention) rebuilt under extra defines (A/B runs through QASR_LIB_OVERRIDE; build container only)
set -e
N=$1; F=$2; shift 2
UNITS=${@:-attention}
D=/root/repo/qwen3-asr.cpp_amd
mkdir -p /tmp/var_$N
OBJS=$(ls $D/build/*.o)
for u in $UNITS; do
    X=""; [ "$u" = fa_exact ] && X="-fno-slp-vectorize"; [ "$u" = gemm_q8 ] && X="-mllvm -amdgpu-mfma-vgpr-form=1"
    /opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -I/root/repo/include -I$D/host -I$D/csrc $X $F -c $D/csrc/$u.hip -o /tmp/var_$N/$u.o
    OBJS=$(echo "$OBJS" | grep -v "/$u.o$")
    OBJS="$OBJS /tmp/var_$N/$u.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/var_$N.so $OBJS -lgomp -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libqasr.so
echo built $D/var_$N.so
