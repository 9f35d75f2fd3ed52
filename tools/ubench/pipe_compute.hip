// Issue rate of the band pipeline's compute alone (bstage_seq, 4 words per lane, KW stages,
// 3 rows per block) with no memory traffic, at a given number of waves per SIMD: is the
// split kernel's 2.86 cycles per VALU op the compute code's own rate or its memory/sync?
//   hipcc --offload-arch=gfx950 -O3 -I../../include -I../../gol-distributed-final_amd/csrc pipe_compute.hip -o pipe_compute
#include "gol_kernels.hip"

// MODE bit 2 (4): the op-by-op stage (bstage) instead of the word-by-word one (bstage_seq).
// MODE 0: compute only.  MODE 1: + the pipe kernel's LDS hand-off per row (ds_write_b128 of
// the row's result, ds_read_b128 of the next row issued one row ahead, waited with
// lgkmcnt(1)), on the wave's own slot so there is no cross-wave waiting.  MODE 2: + one
// 16-byte global store per row (a buffer store, like the last wave).  MODE 3: both.
template <int KW, int MODE = 0>
__global__ void __launch_bounds__(256) pc_kernel(uint32_t *out, uint64_t *cyc, int iters)
{
    using namespace golk;
    constexpr int DW = 4;
    __shared__ uint32_t ring[4][3][3][256];
    lds_u32 *const slot = (lds_u32 *)&ring[threadIdx.x >> 6][0][0][0] + (threadIdx.x & 63) * 4;
    v4u32 nextv = v4u32{threadIdx.x, 1u, 2u, 3u};
    if (MODE & 1) lds_wr128_o<0>(slot, nextv);
    if (MODE & 1) nextv = lds_rd128_issue_o<0>(slot);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000);  // range 0: dropped
    Pipe<KW, DW> p;
    pipe_init(p);
    uint32_t seed = threadIdx.x * 2654435761u + blockIdx.x;
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int S = 0; S < 3; ++S) {
            uint32_t cur[DW];
            if (MODE & 1) {
                lds_wait_n<1>(nextv);
                const v4u32 v = nextv;
                nextv = lds_rd128_issue_o<0>(slot + ((S + 1) % 3) * 256);
#pragma unroll
                for (int j = 0; j < DW; ++j) cur[j] = v[j] ^ (it * 3 + S + j);
            } else {
#pragma unroll
                for (int j = 0; j < DW; ++j) cur[j] = seed ^ (it * 3 + S + j);
            }
#pragma unroll
            for (int g = 0; g < KW; ++g) {
                if (MODE & 4) {
                    if (S == 0) bstage<KW, DW, 0>(p, g, cur);
                    if (S == 1) bstage<KW, DW, 1>(p, g, cur);
                    if (S == 2) bstage<KW, DW, 2>(p, g, cur);
                } else {
                    if (S == 0) bstage_seq<KW, DW, 0>(p, g, cur);
                    if (S == 1) bstage_seq<KW, DW, 1>(p, g, cur);
                    if (S == 2) bstage_seq<KW, DW, 2>(p, g, cur);
                }
            }
#pragma unroll
            for (int j = 0; j < DW; ++j) acc ^= cur[j];
            if (MODE & 1) lds_wr128_o<0>(slot + S * 256, v4u32{cur[0], cur[1], cur[2], cur[3]});
            if (MODE & 2) {
                typedef __attribute__((ext_vector_type(4))) uint32_t v4u;
                __builtin_amdgcn_raw_buffer_store_b128(v4u{cur[0], cur[1], cur[2], cur[3]}, rs, (threadIdx.x & 63) * 16, 0, 0);
            }
        }
    }
    if (MODE & 1) {
        lds_wait_n<0>(nextv);
        acc ^= nextv.x;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KW, int MODE = 0>
void run(int wps)
{
    const int blocks = 256 * wps, iters = 2000;
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&cyc, (size_t)blocks * 4 * 8);
    hipLaunchKernelGGL((pc_kernel<KW, MODE>), dim3(blocks), dim3(256), 0, 0, out, cyc, 10);
    hipLaunchKernelGGL((pc_kernel<KW, MODE>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    (void)hipDeviceSynchronize();
    uint64_t *h = (uint64_t *)malloc((size_t)blocks * 4 * 8);
    (void)hipMemcpy(h, cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i];
    mean /= blocks * 4;
    // VALU per row and stage: 10 logic + 2/4 DPP (approx); report cycles per word-generation
    const double wordgens = (double)iters * 3 * KW * 4;
    printf("KW=%d mode=%d waves/SIMD=%d  SIMD cycles per word-generation=%.2f\n", KW, MODE, wps, mean / wordgens / wps);
    free(h);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main()
{
    for (int rep = 0; rep < 2; ++rep)
        for (int w : {1, 2, 3, 4}) {
            run<3, 0>(w);
            run<3, 4>(w);
            run<3, 1>(w);
            run<3, 3>(w);
            run<3, 7>(w);
        }
    return 0;
}
