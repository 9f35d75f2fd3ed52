// Throughput of carry-based lane shifts on gfx950 (candidates for the bit-board horizontal sum):
//  A: v_mov_b32_dpp + v_alignbit_b32            (current: neighbour word, then funnel shift)
//  B: v_add_co_u32_dpp (carry = neighbour's bit 31) + v_addc_co_u32 (2c + carry)
//  C: v_add_co_u32 + v_addc_co_u32 (same without DPP)
//  D: v_cmp_gt_i32_dpp (vcc = neighbour bit31) + v_addc_co_u32
// 8 independent pairs per asm block, 8 blocks per iteration; reports cycles per PAIR per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define X8(S) S S S S S S S S
#define PAIR_A(D, T) "v_mov_b32_dpp " T ", %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_alignbit_b32 " D ", %16, " T ", 31\n"
#define PAIR_B(D, T) "v_add_co_u32_dpp " T ", vcc, %16, %17 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_addc_co_u32 " D ", vcc, %16, %16, vcc\n"
#define PAIR_C(D, T) "v_add_co_u32 " T ", vcc, %16, %17\n v_addc_co_u32 " D ", vcc, %16, %16, vcc\n"
#define PAIR_D(D, T) "v_cmp_gt_i32_dpp vcc, %17, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_addc_co_u32 " D ", vcc, %16, %16, vcc\n"
#define BLOCK(P) P("%0", "%8") P("%1", "%9") P("%2", "%10") P("%3", "%11") P("%4", "%12") P("%5", "%13") P("%6", "%14") P("%7", "%15")
#define OUTS "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5]), "=v"(o[6]), "=v"(o[7]), \
             "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7])

template <int OP>
__global__ void __launch_bounds__(256) kern(uint32_t *out, int iters)
{
    uint32_t x = threadIdx.x * 0x9E3779B9u, k = 0x80000000u, o[8], t[8];
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) asm volatile(X8(BLOCK(PAIR_A)) : OUTS : "v"(x), "v"(k) : "vcc");
        if (OP == 1) asm volatile(X8(BLOCK(PAIR_B)) : OUTS : "v"(x), "v"(k) : "vcc");
        if (OP == 2) asm volatile(X8(BLOCK(PAIR_C)) : OUTS : "v"(x), "v"(k) : "vcc");
        x += o[0] ^ o[7] ^ t[3];
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
    const double pairs = (double)iters * 64 * wps;
    printf("%-34s waves/SIMD=%d cycles/pair/SIMD=%.2f\n", name, wps, ms * 1e-3 * 2.4e9 / pairs);
    (void)hipFree(out);
}

int main()
{
    for (int w : {2, 4}) {
        run<0>("A mov_dpp + alignbit", w);
        run<1>("B add_co_dpp + addc", w);
        run<2>("C add_co + addc", w);
    }
    return 0;
}
