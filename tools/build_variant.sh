#!/bin/bash
# Build an experimental variant of the kernels into mpc_fatigue_amd/libmf_<name>.so (selected at
# run time with MF_LIB=libmf_<name>.so).  usage: tools/build_variant.sh NAME path/to/ipm_kernels.hip [extra hipcc flags]
set -e
NAME=$1; SRCF=$(readlink -f $2); shift 2
cd "$(dirname "$0")/../mpc_fatigue_amd"
make -s build/capi.hip.o build/urdf.cpp.o build/gipm.hip.o
mkdir -p build_var
cp "$SRCF" csrc/_variant_$NAME.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable "$@" \
  -c csrc/_variant_$NAME.hip -o build_var/$NAME.o
rm -f csrc/_variant_$NAME.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o libmf_$NAME.so build/capi.hip.o build_var/$NAME.o build/gipm.hip.o build/urdf.cpp.o
echo built libmf_$NAME.so
