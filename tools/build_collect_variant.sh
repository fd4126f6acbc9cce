#!/bin/bash
# A variant build of the library with svgd_collect.hip compiled under extra
# -D flags (compile-time A/B switches of k_pair_mcol, e.g. SVGD_MCOL_CODE=1),
# the other objects as built by make.  Output tools/ablibs/<name>.so
# (git-ignored, travels with gpurun).  Usage: build_collect_variant.sh name -DX=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
S=svgdcpp_amd/csrc
make -s
mkdir -p tools/ablibs /tmp/colvar
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm -amdgpu-mfma-vgpr-form \
  "$@" -c $S/svgd_collect.hip -o /tmp/colvar/$name.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/ablibs/$name.so $S/svgd_kernels.o /tmp/colvar/$name.o \
  $S/svgd_capi.o $S/plan.o $S/host_models.o $S/hostcomm.o -L/opt/rocm/lib -lrccl -fopenmp -Wl,-rpath,/opt/rocm/lib
