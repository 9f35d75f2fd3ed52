// Throughput of single VALU opcodes on gfx950: 64 independent instructions per loop
// iteration (inline asm, 8 rotating destinations), W waves per SIMD.  Reports cycles
// per wave64 instruction per SIMD (wall time x 2.4 GHz, so a lower clock reads high).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define R8(I) I I I I I I I I
#define BODY(INS)                                                                              \
    asm volatile(R8(INS " %0, %8, %9, %10\n" INS " %1, %8, %9, %10\n" INS " %2, %8, %9, %10\n"  \
                    INS " %3, %8, %9, %10\n" INS " %4, %8, %9, %10\n" INS " %5, %8, %9, %10\n"  \
                    INS " %6, %8, %9, %10\n" INS " %7, %8, %9, %10\n")                           \
                 : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5]), "=v"(o[6]), "=v"(o[7]) \
                 : "v"(x), "v"(y), "v"(z))
#define BODY2(INS)                                                                             \
    asm volatile(R8(INS " %0, %8, %9\n" INS " %1, %8, %9\n" INS " %2, %8, %9\n" INS " %3, %8, %9\n" \
                    INS " %4, %8, %9\n" INS " %5, %8, %9\n" INS " %6, %8, %9\n" INS " %7, %8, %9\n") \
                 : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5]), "=v"(o[6]), "=v"(o[7]) \
                 : "v"(x), "v"(y))
#define BODY1(INS)                                                                             \
    asm volatile(R8(INS " %0, %8\n" INS " %1, %8\n" INS " %2, %8\n" INS " %3, %8\n" INS " %4, %8\n" \
                    INS " %5, %8\n" INS " %6, %8\n" INS " %7, %8\n")                              \
                 : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5]), "=v"(o[6]), "=v"(o[7]) \
                 : "v"(x))

template <int OP>
__global__ void __launch_bounds__(256) kern(uint32_t *out, int iters)
{
    uint32_t x = threadIdx.x, y = blockIdx.x, z = threadIdx.x * 3, o[8];
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) asm volatile(R8("v_bitop3_b32 %0, %8, %9, %10 bitop3:0x96\nv_bitop3_b32 %1, %8, %9, %10 bitop3:0x96\nv_bitop3_b32 %2, %8, %9, %10 bitop3:0x96\nv_bitop3_b32 %3, %8, %9, %10 bitop3:0x96\nv_bitop3_b32 %4, %8, %9, %10 bitop3:0x96\nv_bitop3_b32 %5, %8, %9, %10 bitop3:0x96\nv_bitop3_b32 %6, %8, %9, %10 bitop3:0x96\nv_bitop3_b32 %7, %8, %9, %10 bitop3:0x96\n") : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5]), "=v"(o[6]), "=v"(o[7]) : "v"(x), "v"(y), "v"(z));
        if (OP == 1) BODY2("v_xor_b32");
        if (OP == 2) BODY("v_or3_b32");
        if (OP == 3) BODY("v_alignbit_b32");
        if (OP == 4) BODY2("v_and_b32");
        if (OP == 5) BODY("v_add3_u32");
        if (OP == 6) BODY("v_perm_b32");
        if (OP == 7) BODY("v_lshl_or_b32");
        if (OP == 8) BODY("v_bfi_b32");
        if (OP == 9) asm volatile(R8("v_mov_b32_dpp %0, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %1, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %2, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %3, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %4, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %5, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %6, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %7, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n") : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5]), "=v"(o[6]), "=v"(o[7]) : "v"(x));
        if (OP == 10) BODY2("v_lshlrev_b32");
        if (OP == 11) BODY("v_and_or_b32");

        if (OP == 13) BODY2("v_or_b32");
        if (OP == 14) BODY2("v_pk_add_u16");
        x += o[0] ^ o[7];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x + o[3];
}

template <int OP>
void run(const char *name, int wps)
{
    uint32_t *out;
    const int blocks = 256 * wps, iters = 4000;
    (void)hipMalloc(&out, blocks * 256 * 4);
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
    const double per_simd = (double)iters * 64 * wps;
    printf("%-20s waves/SIMD=%d cycles/instr/SIMD=%.2f\n", name, wps, ms * 1e-3 * 2.4e9 / per_simd);
    (void)hipFree(out);
}

int main()
{
    for (int w : {2, 4}) {
        run<0>("v_bitop3_b32", w);
        run<1>("v_xor_b32", w);
        run<2>("v_or3_b32", w);
        run<3>("v_alignbit_b32", w);
        run<4>("v_and_b32", w);
        run<5>("v_add3_u32", w);
        run<6>("v_perm_b32", w);
        run<7>("v_lshl_or_b32", w);
        run<8>("v_bfi_b32", w);
        run<9>("v_mov_b32_dpp(none)", w);
        run<10>("v_lshlrev_b32", w);
        run<11>("v_and_or_b32", w);
        run<13>("v_or_b32", w);
        run<14>("v_pk_add_u16", w);
    }
    return 0;
}
