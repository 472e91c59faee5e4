#!/usr/bin/env bash
# Link a CLI variant whose SWAR kernels are compiled with extra defines:
#   tools/r03/build_variant.sh NAME -DPCONV_SWAR_ORDER=1 ...
# -> parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv_NAME
# (the other objects come from the regular in-tree build; run make first).
set -euo pipefail
name=$1; shift
C=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/csrc
T=$(mktemp -d)
for k in stencil_swar stencil_resident; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -I$C/include \
    --offload-arch=gfx950 -ffp-contract=off "$@" -c $C/kernels/$k.hip -o $T/$k.o &
done
wait
objs=$(ls $C/build/*.o | grep -v -e py_module -e stencil_swar.o -e stencil_resident.o)
g++ -o $C/../bin/conv_$name $objs $T/stencil_swar.o $T/stencil_resident.o -L/opt/rocm/lib -lamdhip64 -fopenmp -ldl \
  -Wl,--disable-new-dtags,-rpath,/opt/rocm/lib
rm -rf $T
echo "built bin/conv_$name"
