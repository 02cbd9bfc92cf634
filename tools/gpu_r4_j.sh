#!/bin/bash
# Round 4 (j): C5 shadow lookup A/B: deferred ambiguous lookups x light-space positions from world vs gathered.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=3d-renderer_amd/lib/variants
bash tools/ab.sh "TRI_RASTER_LIB=$V/dnolposw.so" "TRI_RASTER_LIB=$V/nodefer.so" "TRI_RASTER_LIB=$V/nodefer_nolposw.so" "" "TRI_RASTER_LIB=$V/dnolposw.so" "TRI_RASTER_LIB=$V/nodefer.so" "TRI_RASTER_LIB=$V/nodefer_nolposw.so" ""
