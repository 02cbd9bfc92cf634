#!/bin/bash
# Round-6 A/B of front-end register/occupancy variants on C3 (tools/ab.sh, 200 steps, no secondaries), two rounds in
# alternation; variants are lib/variants/NAME.so built by tools/build_variant.sh. usage: bash tools/gpu_ab6.sh NAME...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
V=3d-renderer_amd/lib/variants
set=("")
for n in "$@"; do set+=("TRI_RASTER_LIB=$V/$n.so"); done
EXTRA="--no-secondary ${AB_EXTRA}" bash tools/ab.sh "${set[@]}" "${set[@]}"
