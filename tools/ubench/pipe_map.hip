// Which SIMDs should the 4 waves of a band pipeline sit on?  Synthetic pipeline (no HBM): the
// band kernel's stages (bstage_seq, 4 words per lane, 3 stages per wave, 3-row blocks handed on
// through LDS rings with ready / consumed flags), run on every CU in two wave maps:
//   MAP 0 ("spread", the product kernel): workgroups of 4 waves, 4 per CU; a pipeline's waves
//         sit on 4 different SIMDs, each SIMD runs 4 waves of 4 different pipelines;
//   MAP 1 ("same SIMD"): one workgroup of 16 waves per CU; pipeline p = the waves whose SIMD is
//         p (read from HW_ID), stage = rank among them, so a SIMD runs one whole pipeline.
// Also prints the wave -> SIMD map of a 16-wave workgroup.  Reports SIMD cycles per
// word-generation (10.5 VALU ops x 2 cycles = 21 at the issue peak).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../../gol-distributed-final_amd/csrc pipe_map.hip -o pipe_map
#include "gol_kernels.hip"

using namespace golk;
constexpr int DW = 4, KW = 3, P = 4, NS = 3, ROW = 256;

struct PipeLds {
    uint32_t ring[P - 1][NS][3][ROW];
    int ready[P], consumed[P];
    int scratch[P][64];
};

template <int MAP>
__global__ void __launch_bounds__(MAP ? 1024 : 256) pm_kernel(uint32_t *out, uint64_t *cyc, uint32_t *map, int nblk)
{
    __shared__ PipeLds L[MAP ? 4 : 1];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const int simd = (hw >> 4) & 3;
    int pipe = 0, stage = wave;
    if (MAP) {
        // rank of this wave among the workgroup's waves on the same SIMD (via LDS)
        __shared__ int simd_of[16];
        if (lane == 0) simd_of[wave] = simd;
        __syncthreads();
        int r = 0, n = 0;
        for (int i = 0; i < 16; ++i) { r += i < wave && simd_of[i] == simd; n += simd_of[i] == simd; }
        pipe = simd;
        stage = r;
        if (n != 4) { pipe = wave & 3; stage = wave >> 2; r |= 0x80; }  // not 4 waves per SIMD
        if (blockIdx.x == 0 && lane == 0) map[wave] = simd | (r << 8);
    } else {
        stage = (wave + blockIdx.x / 256) % P;  // rotated per workgroup, like the product kernel
    }
    PipeLds &l = L[pipe];
    if (threadIdx.x < 4 * P) {
        L[threadIdx.x / P].ready[threadIdx.x % P] = 0;
        L[threadIdx.x / P].consumed[threadIdx.x % P] = 0;
    }
    __syncthreads();
    lds_u32 *const ring_l = (lds_u32 *)&l.ring[0][0][0][0];
    lds_u32 *const ready_l = (lds_u32 *)&l.ready[0];
    lds_u32 *const consumed_l = (lds_u32 *)&l.consumed[0];
    lds_u32 *const scr = (lds_u32 *)&l.scratch[stage][lane];
    lds_u32 *const rdy_addr = lane == 0 ? ready_l + stage + 1 : scr;
    lds_u32 *const cns_addr = lane == 0 ? consumed_l + stage : scr;
    constexpr int SLOT = 3 * ROW;
    lds_u32 *const rd_base = ring_l + (stage - 1) * NS * SLOT + lane * 4;
    lds_u32 *const wr_base = ring_l + stage * NS * SLOT + lane * 4;

    Pipe<KW, DW> p;
    pipe_init(p);
    uint32_t acc = 0, seed = threadIdx.x * 2654435761u + blockIdx.x;
    int seen_ready = 0, seen_free = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < nblk; ++b) {
        const int slot = b % NS;
        uint32_t cur[3][DW];
        if (stage > 0) {
            if (seen_ready < b + 1) seen_ready = spin_until_ge(ready_l + stage, b + 1);
            for (int S = 0; S < 3; ++S) {
                v4u32 v = lds_rd128(rd_base + slot * SLOT + S * ROW);
                cur[S][0] = v.x; cur[S][1] = v.y; cur[S][2] = v.z; cur[S][3] = v.w;
            }
            lds_flag_wr(cns_addr, b + 1);
        } else {
            for (int S = 0; S < 3; ++S)
                for (int j = 0; j < DW; ++j) cur[S][j] = seed ^ (b * 3 + S + j * 7);
        }
#pragma unroll
        for (int g = 0; g < KW; ++g) {
            bstage_seq<KW, DW, 0>(p, g, cur[0]);
            bstage_seq<KW, DW, 1>(p, g, cur[1]);
            bstage_seq<KW, DW, 2>(p, g, cur[2]);
        }
        if (stage < P - 1) {
            if (seen_free < b + 1 - NS) seen_free = spin_until_ge(consumed_l + stage + 1, b + 1 - NS);
            for (int S = 0; S < 3; ++S)
                lds_wr128_o<0>(wr_base + slot * SLOT + S * ROW, v4u32{cur[S][0], cur[S][1], cur[S][2], cur[S][3]});
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lds_flag_wr(rdy_addr, b + 1);
        } else {
            for (int S = 0; S < 3; ++S) acc ^= cur[S][0] ^ cur[S][1] ^ cur[S][2] ^ cur[S][3];
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + wave] = t1 - t0;
}

template <int MAP>
void run(int nblk)
{
    const int threads = MAP ? 1024 : 256, blocks = MAP ? 256 : 1024;
    const int waves = blocks * threads / 64;
    uint32_t *out, *map;
    uint64_t *cyc;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    (void)hipMalloc(&cyc, (size_t)waves * 8);
    (void)hipMalloc(&map, 64 * 4);
    hipLaunchKernelGGL((pm_kernel<MAP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, map, 10);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((pm_kernel<MAP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, map, nblk);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint64_t *h = (uint64_t *)malloc((size_t)waves * 8);
    (void)hipMemcpy(h, cyc, (size_t)waves * 8, hipMemcpyDeviceToHost);
    double mean = 0, mx = 0;
    for (int i = 0; i < waves; ++i) { mean += (double)h[i]; mx = h[i] > mx ? h[i] : mx; }
    mean /= waves;
    const double wordgens_per_simd = (double)nblk * 3 * DW * KW * P;  // 4 waves x 3 stages per SIMD
    const double ghz = mx / (ms * 1e6);
    printf("MAP=%d nblk=%d  %.3f ms  clock %.2f GHz  SIMD cycles per word-gen: mean %.2f  max %.2f\n", MAP, nblk, ms, ghz,
           mean / wordgens_per_simd, mx / wordgens_per_simd);
    if (MAP) {
        uint32_t hm[16];
        (void)hipMemcpy(hm, map, 64, hipMemcpyDeviceToHost);
        printf("  wave -> simd/rank:");
        for (int i = 0; i < 16; ++i) printf(" %u/%u", hm[i] & 0xff, hm[i] >> 8);
        printf("\n");
    }
    free(h);
    (void)hipFree(out);
    (void)hipFree(cyc);
    (void)hipFree(map);
}

int main()
{
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(3000);
        run<1>(3000);
    }
    return 0;
}
