// Microbenchmark: issue cost of v_bitop3_b32 vs the VGPR banks of its three sources
// (VGPR n is in bank n % 4), in-kernel s_memtime timing, 1/2/4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 valu_banks.hip -o valu_banks && ./valu_banks
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// 8 independent instructions (destinations v40..v47, sources never written)
#define OPS8(S0, S1, S2)                                                                    \
    asm volatile("v_bitop3_b32 v40, " S0 ", " S1 ", " S2 " bitop3:0x96\n\t"                 \
                 "v_bitop3_b32 v41, " S0 ", " S1 ", " S2 " bitop3:0x96\n\t"                 \
                 "v_bitop3_b32 v42, " S0 ", " S1 ", " S2 " bitop3:0x96\n\t"                 \
                 "v_bitop3_b32 v43, " S0 ", " S1 ", " S2 " bitop3:0x96\n\t"                 \
                 "v_bitop3_b32 v44, " S0 ", " S1 ", " S2 " bitop3:0x96\n\t"                 \
                 "v_bitop3_b32 v45, " S0 ", " S1 ", " S2 " bitop3:0x96\n\t"                 \
                 "v_bitop3_b32 v46, " S0 ", " S1 ", " S2 " bitop3:0x96\n\t"                 \
                 "v_bitop3_b32 v47, " S0 ", " S1 ", " S2 " bitop3:0x96" ::                   \
                     : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v20", "v21", \
                       "v22", "v23", "v24", "v28", "v32")

template <int MODE>
__global__ void __launch_bounds__(256) k(uint64_t *cyc, int iters)
{
    asm volatile("v_mov_b32 v20, 1\n\tv_mov_b32 v21, 2\n\tv_mov_b32 v22, 3\n\tv_mov_b32 v23, 4\n\t"
                 "v_mov_b32 v24, 5\n\tv_mov_b32 v28, 6\n\tv_mov_b32 v32, 7" ::
                     : "v20", "v21", "v22", "v23", "v24", "v28", "v32");
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (MODE == 0) OPS8("v20", "v21", "v22");  // banks 0, 1, 2
            if (MODE == 1) OPS8("v20", "v24", "v21");  // banks 0, 0, 1
            if (MODE == 2) OPS8("v20", "v24", "v28");  // banks 0, 0, 0
            if (MODE == 3) OPS8("v20", "v20", "v20");  // one register three times
            if (MODE == 4) OPS8("v20", "v21", "s0");   // two VGPRs (banks 0, 1) + SGPR
            if (MODE == 5) OPS8("v20", "v21", "v21");  // banks 0, 1, 1 (one register twice)
            if (MODE == 6) OPS8("v20", "v21", "v20");  // banks 0, 1, 0 (one register twice)
            if (MODE == 7) OPS8("v21", "v20", "v24");  // banks 1, 0, 0
            if (MODE == 8) OPS8("v22", "v23", "v21");  // banks 2, 3, 1
            if (MODE == 9) OPS8("v20", "v28", "v21");  // banks 0, 0, 1 (other pair)
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
void run(int wps, const char *name)
{
    const int blocks = 256 * wps, iters = 4000;
    uint64_t *cyc;
    (void)hipMalloc(&cyc, (size_t)blocks * 4 * 8);
    hipLaunchKernelGGL((k<MODE>), dim3(blocks), dim3(256), 0, 0, cyc, 10);
    hipLaunchKernelGGL((k<MODE>), dim3(blocks), dim3(256), 0, 0, cyc, iters);
    (void)hipDeviceSynchronize();
    uint64_t *h = (uint64_t *)malloc((size_t)blocks * 4 * 8);
    (void)hipMemcpy(h, cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i];
    mean /= blocks * 4;
    const double ninst = (double)iters * 8 * 8;
    printf("%-34s waves/SIMD=%d  wave-cyc/inst=%6.2f  SIMD-cyc/inst=%5.2f\n", name, wps, mean / ninst,
           mean / ninst / wps);
    free(h);
    (void)hipFree(cyc);
}

int main()
{
    for (int rep = 0; rep < 2; ++rep)
        for (int w : {2, 4}) {
            run<2>(w, "bitop3 srcs banks 0,0,0");
            run<0>(w, "bitop3 srcs banks 0,1,2");
            run<4>(w, "bitop3 vgpr banks 0,1 + sgpr");
            run<1>(w, "bitop3 srcs banks 0,0,1");
            run<3>(w, "bitop3 same vgpr x3");
            run<5>(w, "bitop3 srcs v20,v21,v21");
            run<6>(w, "bitop3 srcs v20,v21,v20");
            run<7>(w, "bitop3 srcs banks 1,0,0");
            run<8>(w, "bitop3 srcs banks 2,3,1");
            run<9>(w, "bitop3 srcs v20,v28,v21");
        }
    return 0;
}
