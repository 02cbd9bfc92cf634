// vertex_stage.hip — the frame's first kernels (k_vertex, k_vertex_band, k_reset) in a translation unit of their
// own, compiled with LLVM's max-ILP scheduling strategy (Makefile). raster_kernels.hip holds the code; here only
// those kernels and their accessor tri_vertex_stage_kernel are instantiated.
#define TRI_VERTEX_TU 1
#include "raster_kernels.hip"
