// gol_bytes_pipe.hip -- bytes_pipe_kernel (gol_kernels.hip) in a translation unit of its own, so
// that the Makefile can compile it with the max-memory-clause machine scheduler (the band
// pipeline runs best under max-ILP, the rest under the default); see the GOL_TU_BYTES_PIPE
// section of gol_kernels.hip.
#define GOL_TU_BYTES_PIPE 1
#include "gol_kernels.hip"
