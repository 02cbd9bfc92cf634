#!/bin/bash
# Round 4 (i): C5 fragment-stage cost split by ablation builds (diagnostics only: 2048 no shadow lookup,
# 128 no texture sample, 64 no lights), the bench line's C5 raster stage per build, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=3d-renderer_amd/lib/variants
bash tools/ab.sh "TRI_RASTER_LIB=$V/ab2048.so" "TRI_RASTER_LIB=$V/ab128.so" "TRI_RASTER_LIB=$V/ab64.so" "" "TRI_RASTER_LIB=$V/ab2048.so" "TRI_RASTER_LIB=$V/ab128.so" "TRI_RASTER_LIB=$V/ab64.so" ""
