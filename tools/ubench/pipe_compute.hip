// Issue rate of the band pipeline's compute alone (bstage_seq, 4 words per lane, KW stages,
// 3 rows per block) with no memory traffic, at a given number of waves per SIMD: is the
// split kernel's 2.86 cycles per VALU op the compute code's own rate or its memory/sync?
//   hipcc --offload-arch=gfx950 -O3 -I../../include -I../../gol-distributed-final_amd/csrc pipe_compute.hip -o pipe_compute
#include "gol_kernels.hip"

template <int KW>
__global__ void __launch_bounds__(256) pc_kernel(uint32_t *out, uint64_t *cyc, int iters)
{
    using namespace golk;
    constexpr int DW = 4;
    Pipe<KW, DW> p;
    PipeSel<KW, DW, 0>::init(p);
    uint32_t seed = threadIdx.x * 2654435761u + blockIdx.x;
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int S = 0; S < 3; ++S) {
            uint32_t cur[DW];
#pragma unroll
            for (int j = 0; j < DW; ++j) cur[j] = seed ^ (it * 3 + S + j);
#pragma unroll
            for (int g = 0; g < KW; ++g) {
                if (S == 0) bstage_seq<KW, DW, 0>(p, g, cur);
                if (S == 1) bstage_seq<KW, DW, 1>(p, g, cur);
                if (S == 2) bstage_seq<KW, DW, 2>(p, g, cur);
            }
#pragma unroll
            for (int j = 0; j < DW; ++j) acc ^= cur[j];
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KW>
void run(int wps)
{
    const int blocks = 256 * wps, iters = 2000;
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&cyc, (size_t)blocks * 4 * 8);
    hipLaunchKernelGGL((pc_kernel<KW>), dim3(blocks), dim3(256), 0, 0, out, cyc, 10);
    hipLaunchKernelGGL((pc_kernel<KW>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    (void)hipDeviceSynchronize();
    uint64_t *h = (uint64_t *)malloc((size_t)blocks * 4 * 8);
    (void)hipMemcpy(h, cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i];
    mean /= blocks * 4;
    // VALU per row and stage: 10 logic + 2/4 DPP (approx); report cycles per word-generation
    const double wordgens = (double)iters * 3 * KW * 4;
    printf("KW=%d waves/SIMD=%d  SIMD cycles per word-generation=%.2f\n", KW, wps, mean / wordgens / wps);
    free(h);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main()
{
    for (int w : {2, 4}) {
        run<3>(w);
        run<8>(w);
    }
    return 0;
}
