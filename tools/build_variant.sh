#!/bin/bash
# Build an A/B variant of the HIP library: tools/build_variant.sh NAME [extra hipcc flags...]
# -> 3d-renderer_amd/lib/variants/NAME.so (select it with TRI_RASTER_LIB=... on the GPU box).
# raster_plain.hip is compiled without SLP vectorisation and with the max-ILP scheduler, as in the Makefile.
set -e
cd "$(dirname "$0")/../3d-renderer_amd"
name=$1; shift
mkdir -p lib/variants/obj_$name
for s in raster_kernels raster_plain vertex_stage tri_raster_capi tri_group band_codec tri_xfer; do
  extra=""; [ $s = raster_plain ] && extra="-fno-slp-vectorize -mllvm --amdgpu-sched-strategy=max-ilp"
  [ $s = vertex_stage ] && extra="${VERTEX_SCHED-}"  # (the Makefile default: the default scheduler)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function -mllvm -amdgpu-kernarg-preload-count=2 $extra "$@" \
    -c csrc/$s.hip -o lib/variants/obj_$name/$s.o &
done
wait
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o lib/variants/$name.so lib/variants/obj_$name/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built lib/variants/$name.so"
