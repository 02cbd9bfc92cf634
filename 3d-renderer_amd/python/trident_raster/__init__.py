"""Trident HIP software rasterizer — Python plumbing over the C-ABI (include/tri_raster.h)."""
from . import abi  # noqa: F401
