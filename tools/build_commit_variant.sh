#!/bin/bash
# Build the HIP library of another commit as an A/B variant: tools/build_commit_variant.sh NAME COMMIT
# -> 3d-renderer_amd/lib/variants/NAME.so (select with TRI_RASTER_LIB=... on the GPU box). Same units and flags as
# the Makefile (kernarg preload; raster_plain without SLP under max-ILP; vertex_stage under max-ILP).
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2
src=$(mktemp -d)
out=$PWD/3d-renderer_amd/lib/variants
rm -rf $out/obj_$name
mkdir -p $src/pkg/csrc $src/include $out/obj_$name
units=""
for f in raster_kernels.hip raster_plain.hip vertex_stage.hip tri_raster_capi.hip tri_group.hip band_codec.hip tri_xfer.hip \
         raster_common.h raster_launch.h; do
  if git cat-file -e $rev:3d-renderer_amd/csrc/$f 2>/dev/null; then
    git show $rev:3d-renderer_amd/csrc/$f > $src/pkg/csrc/$f
    case $f in *.hip) units="$units ${f%.hip}";; esac
  fi
done
git show $rev:include/tri_raster.h > $src/include/tri_raster.h
for s in $units; do
  extra=""
  [ $s = raster_plain ] && extra="-fno-slp-vectorize -mllvm --amdgpu-sched-strategy=max-ilp"
  [ $s = vertex_stage ] && extra="-mllvm --amdgpu-sched-strategy=max-ilp"
  (cd $src/pkg && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function \
     -mllvm -amdgpu-kernarg-preload-count=2 $extra -c csrc/$s.hip -o $out/obj_$name/$s.o) &
done
wait
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o $out/$name.so $out/obj_$name/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf $src
echo "built 3d-renderer_amd/lib/variants/$name.so ($rev)"
