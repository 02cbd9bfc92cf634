set -o pipefail
for v in "" dbp_a1 dbp_a2 dbp_a4 dbp_a7; do
  if [ -n "$v" ]; then export TRI_RASTER_LIB=3d-renderer_amd/lib/variants/$v.so; else unset TRI_RASTER_LIB; fi
  echo "== ${v:-base}"
  DBP_SIZES=8 timeout -k 10 120 python -u tools/dbp_scaling.py 2>&1 | grep -v amdgpu.ids || exit 1
done
