#!/bin/bash
# Variant builds of the library for same-box A/B of the fp64 tile phi
# (k_phi<double>): base = the committed kernel source (git HEAD), then
# -D SVGD_PHI_PRE / SVGD_PHI_WPE variants of the working tree.  Outputs
# tools/ablibs/<name>.so (git-ignored, travel with gpurun).
set -e
cd "$(dirname "$0")/.."
S=svgdcpp_amd/csrc
T=/tmp/phivar
mkdir -p $T tools/ablibs
OTHER="$S/svgd_collect.o $S/svgd_capi.o $S/plan.o $S/host_models.o $S/hostcomm.o"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I$S"
link() { /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/ablibs/$1.so $2 $OTHER -L/opt/rocm/lib -lrccl -fopenmp -Wl,-rpath,/opt/rocm/lib; }
pids=()
if false; then
  git show $BASE_REV:$S/svgd_kernels.hip > $S/.base_kernels.hip
  ( /opt/rocm/bin/hipcc $F -c $S/.base_kernels.hip -o $T/base.o && link base $T/base.o ) & pids+=($!)
fi
for v in "$@"; do  # name:PRE:WPE:NW
  IFS=: read name pre wpe nw <<< "$v"
  ( /opt/rocm/bin/hipcc $F -DSVGD_PHI_PRE=$pre -DSVGD_PHI_WPE=$wpe -DSVGD_PHI_NW=$nw -c $S/svgd_kernels.hip -o $T/$name.o && link $name $T/$name.o ) & pids+=($!)
done
rc=0; for p in "${pids[@]}"; do wait $p || rc=1; done
rm -f $S/.base_kernels.hip
exit $rc
