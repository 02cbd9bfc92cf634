#!/bin/bash
# Build libraries whose k_dbp_unpack skips one part (DBP_ABLATE bits: 1 plane decode, 2 scans, 4 stores), linked with
# the Makefile's objects of the other translation units -> 3d-renderer_amd/lib/variants/dbp_a$k.so
set -e
cd "$(dirname "$0")/../3d-renderer_amd"
mkdir -p lib/variants
for k in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function \
    -mllvm -amdgpu-kernarg-preload-count=2 -DDBP_ABLATE=$k -c csrc/band_codec.hip -o lib/variants/band_codec_a$k.o
  objs=$(ls lib/obj/*.o | grep -v host_ | grep -v band_codec)
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o lib/variants/dbp_a$k.so $objs lib/variants/band_codec_a$k.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built lib/variants/dbp_a$k.so"
done
