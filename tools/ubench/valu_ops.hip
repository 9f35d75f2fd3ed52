// Microbenchmark: throughput (cycles per wave64 instruction per SIMD) of the VALU ops the
// bit-board step uses and of candidate replacements, 4 independent chains, 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CH 4
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, int iters)
{
    uint32_t v[CH], w[CH];
    for (int c = 0; c < CH; ++c) { v[c] = threadIdx.x * 7 + c; w[c] = threadIdx.x * 13 + c; }
    const uint32_t a = blockIdx.x, b = threadIdx.x ^ 0x55;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                uint32_t x = v[c];
                if (OP == 0) x = __builtin_amdgcn_bitop3_b32(x, a, w[c], 0x96);
                if (OP == 1) x = x ^ w[c];                       // v_xor_b32 (VOP2)
                if (OP == 2) x = (x & w[c]) ;                     // v_and_b32
                if (OP == 3) x = __builtin_amdgcn_alignbit(x, w[c], 31);
                if (OP == 4) x = __builtin_amdgcn_mov_dpp(x, 0x138, 0xf, 0xf, true);
                if (OP == 5) x = __builtin_amdgcn_mov_dpp(x, 0x111, 0xf, 0xf, true);  // row_shr:1
                if (OP == 6) x = x + w[c];                        // v_add_u32
                if (OP == 7) x = (x << 1);                        // v_lshlrev_b32
                if (OP == 8) x = x ^ w[c] ^ a;                    // v_xor3 or bitop3
                if (OP == 9) { uint64_t y = ((uint64_t)x << 32 | w[c]); y = y ^ (y << 1); x = (uint32_t)(y >> 7); }
                if (OP == 10) x = __builtin_amdgcn_perm(x, w[c], 0x05040100);
                if (OP == 11) x = __builtin_amdgcn_update_dpp(x, w[c], 0x138, 0xf, 0xf, false);
                v[c] = x;
                w[c] = w[c] + 1;
            }
        }
    }
    uint32_t s = 0;
    for (int c = 0; c < CH; ++c) s ^= v[c] ^ w[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
void run(const char *name)
{
    uint32_t *out;
    const int wps = 4, blocks = 256 * wps, iters = 2000;
    (void)hipMalloc(&out, blocks * 256 * 4);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // per inner op: the op + the w[c] add (counted as 1 extra instr)
    const double per_simd = (double)iters * 16 * CH * wps;
    printf("%-22s cycles per (op + v_add) per SIMD at 2.4GHz: %.2f\n", name, ms * 1e-3 * 2.4e9 / per_simd);
    (void)hipFree(out);
}

int main()
{
    run<6>("add (baseline 2 adds)");
    run<0>("bitop3");
    run<1>("xor (VOP2)");
    run<2>("and (VOP2)");
    run<3>("alignbit");
    run<4>("mov_dpp wave_shr");
    run<5>("mov_dpp row_shr");
    run<7>("lshl");
    run<8>("xor3");
    run<9>("64-bit shift mix");
    run<10>("perm");
    run<11>("update_dpp wave_shr");
    return 0;
}
