// Issue rate of the band pipeline's pair step (pstage, round 5: 8 logic ops per 32 cells) alone,
// KW = 3 stages per 2-row block as in band_pipe_kernel, at 1-4 waves per SIMD: is the kernel's
// ~0.73 VALU issue (of the measured clock) the compute code's own rate or its hand-offs?
// MODE 0: compute only.  MODE 1: + the kernel's LDS hand-off per block on the wave's own slot
// (two ds_write_b128 of the results, two ds_read_b128 of the next block issued at the block's end
// and waited at the next block's start; no cross-wave waits).  MODE 2: + two 16-byte buffer
// stores per block (range 0: dropped), as the last wave.  MODE 3: both.  MODE bit 4: wave 0 of
// each workgroup also stages two 1 KiB rows per block HBM -> LDS with global_load_lds (blocks b+1 ..
// b+3 in flight, the kernel's vmcnt wait), walking its own column group of a 16 GiB board as the
// band loader does.  MODE bit 8: + the kernel's flag traffic per block (one ds_write_b32 flag, one
// ds_read_b32 poll that succeeds at once, readfirstlane).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-sched-strategy=max-ilp -mllvm -disable-post-ra \
//     -I include -I gol-distributed-final_amd/csrc tools/ubench/pair_compute.hip -o tools/variants/pair_compute
#define GOL_TU_BAND_PIPE 1  // only the band pipeline part of the kernels file
#include "gol_kernels.hip"

template <int MODE>
__global__ void __launch_bounds__(256) pc_kernel(uint32_t *out, uint64_t *cyc, int iters, const char *board)
{
    using namespace golk;
    constexpr int DW = 4, KW = 3;
    __shared__ uint32_t ring[4][4][2][256];
    __shared__ uint32_t in_ring[4][2][256];
    __shared__ int flags[8];
    const bool loader = (MODE & 4) && threadIdx.x < 64;
    const int lane = threadIdx.x & 63;
    const int group = blockIdx.x % 142, strip = blockIdx.x / 142;
    const char *src = board + (int64_t)(strip * 1048 % 131000) * 131072 + group * 928 + lane * 16;
    lds_u32 *const in_l = (lds_u32 *)&in_ring[0][0][0];
    if (threadIdx.x < 8) flags[threadIdx.x] = 1 << 20;
    __syncthreads();
    lds_u32 *const fl = (lds_u32 *)&flags[threadIdx.x >> 6];
    auto dma = [&](int b, int u) {
        if (!loader) return;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + (int64_t)(2 * b) * 131072), in_l + u * 512, 16, 0, 0);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + (int64_t)(2 * b + 1) * 131072), in_l + u * 512 + 256, 16, 0, 0);
    };
    if (MODE & 4) { dma(0, 0); dma(1, 1); dma(2, 2); }
    lds_u32 *const slot = (lds_u32 *)&ring[threadIdx.x >> 6][0][0][0] + (threadIdx.x & 63) * 4;
    v4u32 nx0 = v4u32{threadIdx.x, 1u, 2u, 3u}, nx1 = v4u32{blockIdx.x, 5u, 6u, 7u};
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000);  // range 0: dropped
    PairState<DW> st[KW];
#pragma unroll
    for (int g = 0; g < KW; ++g)
#pragma unroll
        for (int j = 0; j < DW; ++j) { st[g].a0[j] = j; st[g].a1[j] = g; st[g].b0[j] = j ^ g; st[g].b1[j] = 7; st[g].cb[j] = 9; }
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint32_t r0[DW], r1[DW];
            if (MODE & 1) lds_settle2(nx0, nx1);
            if (MODE & 8) {
                lds_flag_wr(fl, it * 4 + u);
                const int f = __builtin_amdgcn_readfirstlane(lds_rd32(fl));
                if (f < 0) out[0] = f;  // (never)
            }
#pragma unroll
            for (int j = 0; j < DW; ++j) {
                r0[j] = nx0[j] ^ (uint32_t)(it * 4 + u);
                r1[j] = nx1[j] ^ (uint32_t)(it * 4 + u + j);
            }
#pragma unroll
            for (int g = 0; g < KW; ++g) pstage<DW>(st[g], r0, r1);
            if (MODE & 2) {
                __builtin_amdgcn_raw_buffer_store_b128(v4u32{r0[0], r0[1], r0[2], r0[3]}, rs, threadIdx.x * 16u, 0, 2);
                __builtin_amdgcn_raw_buffer_store_b128(v4u32{r1[0], r1[1], r1[2], r1[3]}, rs, threadIdx.x * 16u + 16u, 0, 2);
            }
            if (MODE & 4) {
                dma(it * 4 + u + 3, (u + 3) % 4);
                if (loader) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            }
            if (MODE & 1) {
                lds_wr128x2_o<0, 1024>(slot + u * 2048, v4u32{r0[0], r0[1], r0[2], r0[3]}, v4u32{r1[0], r1[1], r1[2], r1[3]});
                lds_rd128x2_issue_o<0, 1024>(slot + ((u + 1) % 4) * 2048, nx0, nx1);
            } else {
                nx0 = v4u32{r0[0], r0[1], r0[2], r0[3]};
                nx1 = v4u32{r1[0], r1[1], r1[2], r1[3]};
            }
        }
    }
    if (MODE & 1) lds_settle2(nx0, nx1);
    if (MODE & 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    acc = nx0[0] ^ nx1[3];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

static char *g_board;
template <int MODE>
void run(int wps)
{
    const int blocks = 256 * wps, iters = 500;
    uint64_t *cyc;
    uint32_t *out;
    (void)hipMalloc(&cyc, (size_t)blocks * 4 * 8);
    (void)hipMalloc(&out, 4096);
    hipLaunchKernelGGL((pc_kernel<MODE>), dim3(blocks), dim3(256), 0, 0, out, cyc, 10, (const char *)g_board);
    hipLaunchKernelGGL((pc_kernel<MODE>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters, (const char *)g_board);
    (void)hipDeviceSynchronize();
    uint64_t *h = (uint64_t *)malloc((size_t)blocks * 4 * 8);
    (void)hipMemcpy(h, cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i];
    mean /= blocks * 4;
    const double valu = 3.0 * (16 * 4 + 4) + 8;  // per block: 3 pair steps (64 logic + 4 DPP) + input xors
    const double blk = (double)iters * 4;
    printf("mode=%d waves/SIMD=%d  SIMD cycles per block=%.1f  VALU issue=%.3f of 1 per 2 cycles\n", MODE, wps,
           mean / blk / wps, valu * 2.0 / (mean / blk / wps));
    free(h);
    (void)hipFree(cyc);
    (void)hipFree(out);
}

int main()
{
    (void)hipMalloc(&g_board, (size_t)131072 * 131072);
    (void)hipMemset(g_board, 0x5a, (size_t)131072 * 131072);
    for (int rep = 0; rep < 2; ++rep)
        for (int w : {3, 4}) {
            run<0>(w);
            run<3>(w);
            run<7>(w);
            run<11>(w);
            run<15>(w);
        }
    return 0;
}
