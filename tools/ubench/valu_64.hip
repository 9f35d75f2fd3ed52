// Throughput of 64-bit shift-class ops on gfx950 (cycles per wave64 instruction per SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define R8(S) S S S S S S S S
#define OUT8 "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5]), "=v"(o[6]), "=v"(o[7])
template <int OP>
__global__ void __launch_bounds__(256) kern(uint64_t *out, int iters)
{
    uint64_t x = threadIdx.x * 0x9E3779B97F4A7C15ull, y = blockIdx.x, o[8];
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) asm volatile(R8("v_lshlrev_b64 %0, 1, %8\n v_lshlrev_b64 %1, 1, %8\n v_lshlrev_b64 %2, 1, %8\n v_lshlrev_b64 %3, 1, %8\n v_lshlrev_b64 %4, 1, %8\n v_lshlrev_b64 %5, 1, %8\n v_lshlrev_b64 %6, 1, %8\n v_lshlrev_b64 %7, 1, %8\n") : OUT8 : "v"(x));
        if (OP == 1) asm volatile(R8("v_lshl_add_u64 %0, %8, 1, %9\n v_lshl_add_u64 %1, %8, 1, %9\n v_lshl_add_u64 %2, %8, 1, %9\n v_lshl_add_u64 %3, %8, 1, %9\n v_lshl_add_u64 %4, %8, 1, %9\n v_lshl_add_u64 %5, %8, 1, %9\n v_lshl_add_u64 %6, %8, 1, %9\n v_lshl_add_u64 %7, %8, 1, %9\n") : OUT8 : "v"(x), "v"(y));
        if (OP == 2) asm volatile(R8("v_lshrrev_b64 %0, 1, %8\n v_lshrrev_b64 %1, 1, %8\n v_lshrrev_b64 %2, 1, %8\n v_lshrrev_b64 %3, 1, %8\n v_lshrrev_b64 %4, 1, %8\n v_lshrrev_b64 %5, 1, %8\n v_lshrrev_b64 %6, 1, %8\n v_lshrrev_b64 %7, 1, %8\n") : OUT8 : "v"(x));
        if (OP == 3) asm volatile(R8("v_pk_mov_b32 %0, %8, %9 op_sel:[0,1]\n v_pk_mov_b32 %1, %8, %9 op_sel:[0,1]\n v_pk_mov_b32 %2, %8, %9 op_sel:[0,1]\n v_pk_mov_b32 %3, %8, %9 op_sel:[0,1]\n v_pk_mov_b32 %4, %8, %9 op_sel:[0,1]\n v_pk_mov_b32 %5, %8, %9 op_sel:[0,1]\n v_pk_mov_b32 %6, %8, %9 op_sel:[0,1]\n v_pk_mov_b32 %7, %8, %9 op_sel:[0,1]\n") : OUT8 : "v"(x), "v"(y));
        x += o[0] ^ o[7];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x + o[3];
}
template <int OP>
void run(const char *name, int wps)
{
    uint64_t *out;
    const int blocks = 256 * wps, iters = 4000;
    (void)hipMalloc(&out, blocks * 256 * 8);
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-18s waves/SIMD=%d cycles/instr/SIMD=%.2f\n", name, wps, ms * 1e-3 * 2.4e9 / ((double)iters * 64 * wps));
    (void)hipFree(out);
}
int main()
{
    for (int w : {2, 4}) {
        run<0>("v_lshlrev_b64", w);
        run<1>("v_lshl_add_u64", w);
        run<2>("v_lshrrev_b64", w);
        run<3>("v_pk_mov_b32", w);
    }
}
