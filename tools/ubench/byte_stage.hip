// Cycles per 3-row block of the byte pipeline's compute (sstage_waves3, one word per lane, KW
// stages), alone (MODE 0) and with the per-block LDS hand-off of a middle wave (MODE 1: three
// ds_read_b32 + wait, three ds_write_b32 + wait, on the wave's own slot), at 1..8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -I../../include -I../../gol-distributed-final_amd/csrc byte_stage.hip -o byte_stage
#include "gol_kernels.hip"

template <int KW, int MODE>
__global__ void __launch_bounds__(256) bs_kernel(uint32_t *out, uint64_t *cyc, int iters)
{
    using namespace golk;
    __shared__ uint32_t slot[4][3][64];
    lds_u32 *const my = (lds_u32 *)&slot[threadIdx.x >> 6][0][0] + (threadIdx.x & 63);
    Pipe<KW, 1> p;
    pipe_init(p);
    uint32_t w3[3] = {threadIdx.x * 2654435761u, blockIdx.x * 40503u + 7u, threadIdx.x ^ 0x5bd1e995u};
    if (MODE) {
        for (int S = 0; S < 3; ++S) lds_wr32(my + S * 64, (int)w3[S]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE) lds_rd32x3(my, w3);
        sstage_waves3<KW, KW>(p, w3, std::make_integer_sequence<int, KW + 2>());
        acc ^= w3[0] ^ w3[1] ^ w3[2];
        if (MODE) {
            for (int S = 0; S < 3; ++S) lds_wr32(my + S * 64, (int)w3[S]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else {
            w3[0] ^= it;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KW, int MODE>
void run(int wps)
{
    const int blocks = 256 * wps, threads = 256, iters = 4000;  // wps workgroups of 4 waves per CU
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    (void)hipMalloc(&cyc, (size_t)blocks * 4 * 8);
    hipLaunchKernelGGL((bs_kernel<KW, MODE>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 10);
    hipLaunchKernelGGL((bs_kernel<KW, MODE>), dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    (void)hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    uint64_t *h = (uint64_t *)malloc((size_t)nw * 8);
    (void)hipMemcpy(h, cyc, (size_t)nw * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < nw; ++i) mean += (double)h[i];
    mean /= nw;
    printf("KW=%d mode=%d waves/SIMD=%d  cycles per block per wave=%.0f  SIMD cycles per block=%.0f\n", KW, MODE, wps,
           mean / iters, mean / iters / wps);
    free(h);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main()
{
    for (int w : {1, 2, 3, 4, 6, 8}) {
        run<4, 0>(w);
        run<4, 1>(w);
    }
    return 0;
}
