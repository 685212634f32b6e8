#!/bin/bash
# build_variant.sh NAME "-DFLAG=.. ..." -> qwen3-asr.cpp_amd/var_NAME.so: libqasr.so with attention.hip rebuilt
# under extra defines (A/B runs through QASR_LIB_OVERRIDE; build container only)
set -e
N=$1; F=$2
D=/root/repo/qwen3-asr.cpp_amd
mkdir -p /tmp/var_$N
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -I/root/repo/include -I$D/host -I$D/csrc $F -c $D/csrc/attention.hip -o /tmp/var_$N/attention.o
OBJS=$(ls $D/build/*.o | grep -v '/attention.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/var_$N.so /tmp/var_$N/attention.o $OBJS -lgomp -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libqasr.so
echo built $D/var_$N.so
