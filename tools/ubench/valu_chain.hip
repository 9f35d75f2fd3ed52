// Microbenchmark: issue rate of dependent vs independent v_bitop3 chains and of DPP
// wave shifts on gfx950, at 1..8 waves per SIMD.  Prints cycles per instruction per wave
// and per SIMD.  (tools/ubench; informs the bits_step_kernel schedule.)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE, int CHAINS>
__global__ void __launch_bounds__(256) chain(uint32_t *out, int iters, unsigned long long *cyc)
{
    uint32_t v[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) v[c] = threadIdx.x * 7 + c;
    const uint32_t a = blockIdx.x, b = threadIdx.x ^ 0x55;
    unsigned long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) {
                if (MODE == 0) v[c] = __builtin_amdgcn_bitop3_b32(v[c], a, b, 0x96);
                if (MODE == 1) v[c] = __builtin_amdgcn_mov_dpp(v[c], 0x138, 0xf, 0xf, true) ^ a;
                if (MODE == 2) v[c] = __builtin_amdgcn_alignbit(v[c], b, 31) ^ a;
            }
        }
    }
    unsigned long long t1 = clock64();
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE, int CHAINS>
void run(const char *name, int waves_per_simd)
{
    uint32_t *out;
    unsigned long long *cyc;
    const int blocks = 256 * waves_per_simd;  // 4 waves per block -> 1 wave per SIMD per block
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&cyc, 8);
    const int iters = 2000;
    hipLaunchKernelGGL((chain<MODE, CHAINS>), dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((chain<MODE, CHAINS>), dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // each chain-op pair counts as the ops issued per loop body
    const int ops_per_iter = 16 * CHAINS * (MODE == 0 ? 1 : 2);
    const double instr = (double)iters * ops_per_iter;
    const double ghz = 2.4;
    const double wall_cyc = ms * 1e-3 * ghz * 1e9;
    printf("%-12s chains=%d waves/SIMD=%d  clock64 cyc/instr/wave=%.2f  wall cyc/instr/SIMD=%.2f\n", name, CHAINS,
           waves_per_simd, c / instr, wall_cyc / (instr * waves_per_simd));
    hipFree(out);
    hipFree(cyc);
}

int main()
{
    for (int w : {1, 2, 3, 4, 8}) {
        run<0, 1>("bitop3", w);
        run<0, 2>("bitop3", w);
        run<0, 4>("bitop3", w);
        run<1, 1>("dpp+xor", w);
        run<1, 2>("dpp+xor", w);
        run<1, 4>("dpp+xor", w);
        run<2, 1>("alignbit+xor", w);
        run<2, 4>("alignbit+xor", w);
    }
    return 0;
}
