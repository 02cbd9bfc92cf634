// raster_plain.hip — k_raster for frames without the shadow pre-pass, in a translation unit of its own so
// that it is compiled without SLP vectorisation (Makefile: -fno-slp-vectorize). raster_kernels.hip holds
// the code; here only k_raster_plain and its launcher tri_launch_raster_plain are instantiated.
#define TRI_RASTER_PLAIN_TU 1
#include "raster_kernels.hip"
