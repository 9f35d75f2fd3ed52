// Microbenchmark: VALU issue rate of v_bitop3_b32 (3 VGPR sources) vs waves per SIMD and
// independent chains per wave, timed in-kernel with s_memtime (shader clock cycles).
// Prints SIMD cycles per wave64 instruction = wave cycles / (instructions x waves per SIMD).
//   hipcc --offload-arch=gfx950 -O3 valu_occ.hip -o valu_occ && ./valu_occ
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int CH, int MODE>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint64_t *cyc, int iters)
{
    uint32_t x[CH], y[CH], z[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) { x[c] = threadIdx.x * 7 + c; y[c] = threadIdx.x * 13 + 3 * c; z[c] = blockIdx.x + c; }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if (MODE == 0) x[c] = __builtin_amdgcn_bitop3_b32(x[c], y[c], z[c], 0x96);
                if (MODE == 1) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(x[c]) : "v"(y[c]));  // VOP2, 4 bytes
                if (MODE == 3) asm volatile("v_xor_b32_e64 %0, %1, %0" : "+v"(x[c]) : "v"(y[c]));  // VOP3, 8 bytes
                if (MODE == 4) asm volatile("v_not_b32_e32 %0, %0" : "+v"(x[c]));                  // VOP1
                if (MODE == 2) {                   // one DPP move per 4 bitop3
                    x[c] = __builtin_amdgcn_bitop3_b32(x[c], y[c], z[c], 0x96);
                    if ((r & 3) == 0) y[c] = __builtin_amdgcn_mov_dpp(x[c], 0x138, 0xf, 0xf, true);
                }
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s ^= x[c] ^ y[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int CH, int MODE>
void run(int wps, const char *name)
{
    const int cus = 256, blocks = cus * wps, iters = 4000;
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&cyc, (size_t)blocks * 4 * 8);
    hipLaunchKernelGGL((k<CH, MODE>), dim3(blocks), dim3(256), 0, 0, out, cyc, 10);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<CH, MODE>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint64_t *h = (uint64_t *)malloc((size_t)blocks * 4 * 8);
    (void)hipMemcpy(h, cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i];
    mean /= blocks * 4;
    const double ninst = (double)iters * 16 * CH * (MODE == 2 ? 1.25 : 1.0);
    // wave cycles / instructions = cycles per instruction for one wave; x waves per SIMD
    // sharing the SIMD = SIMD cycles per instruction
    printf("%-28s waves/SIMD=%d chains=%2d  wave-cyc/inst=%6.2f  SIMD-cyc/inst=%5.2f  clock=%.2f GHz\n", name, wps,
           CH, mean / ninst, mean / ninst / wps, mean / (ms * 1e-3) / 1e9);
    free(h);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main()
{
    for (int w : {1, 2, 4}) {
        run<4, 0>(w, "bitop3 (3 vgpr)");
        run<8, 0>(w, "bitop3 (3 vgpr)");
        run<8, 1>(w, "v_xor_b32_e32 (vop2, 4 B)");
        run<8, 3>(w, "v_xor_b32_e64 (vop3, 8 B)");
        run<8, 4>(w, "v_not_b32_e32 (vop1)");
        run<8, 2>(w, "bitop3 + dpp/4");
    }
    return 0;
}
