// gol_band_pipe.hip -- band_pipe_kernel (gol_kernels.hip) in a translation unit of its own, so
// that the Makefile can compile it with the max-ILP machine scheduler (the byte pipeline is
// faster with the default one); see the GOL_TU_BAND_PIPE section of gol_kernels.hip.
#define GOL_TU_BAND_PIPE 1
#include "gol_kernels.hip"
