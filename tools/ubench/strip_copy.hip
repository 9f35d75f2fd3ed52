// HBM rate of the band kernels' access pattern without the compute: every wave copies a
// 1 KiB column chunk (64 lanes x 16 B) of a 2^17 x 128 KiB board, walking a strip of rows,
// with a workgroup of WPB waves on adjacent chunks.  Is ~4-4.7 TB/s (what the k = 4 and
// k = 8 kernels reach) the pattern's ceiling, and does a wider workgroup raise it?
//   hipcc --offload-arch=gfx950 -O3 strip_copy.hip -o strip_copy
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// TILED: the board stored chunk-major (all rows of a 1 KiB column chunk contiguous), so a
// wave's strip is one sequential stream.
template <int WPB, bool TILED>
__global__ void __launch_bounds__(64 * WPB) copy_kernel(const uint4 *src, uint4 *dst, int rows, int strip,
                                                         int chunks_per_row)
{
    const int lane = threadIdx.x & 63;
    const int chunk = blockIdx.x * WPB + (threadIdx.x >> 6);
    if (chunk >= chunks_per_row) return;
    const int r0 = blockIdx.y * strip;
    const int r1 = min(r0 + strip, rows);
    const int64_t pitch = TILED ? 64 : (int64_t)chunks_per_row * 64;  // uint4 per row
    const int64_t col = TILED ? (int64_t)chunk * rows * 64 + lane : (int64_t)chunk * 64 + lane;
    uint4 b0 = src[(int64_t)r0 * pitch + col];
    uint4 b1 = r0 + 1 < r1 ? src[(int64_t)(r0 + 1) * pitch + col] : b0;
    uint4 b2 = r0 + 2 < r1 ? src[(int64_t)(r0 + 2) * pitch + col] : b0;
    for (int r = r0; r < r1; ++r) {
        const int rn = r + 3 < r1 ? r + 3 : r1 - 1;
        const uint4 n = src[(int64_t)rn * pitch + col];
        dst[(int64_t)r * pitch + col] = b0;
        b0 = b1;
        b1 = b2;
        b2 = n;
    }
}

template <int WPB, bool TILED = false>
void run(const uint4 *src, uint4 *dst, int rows, int cpr, int strip)
{
    const dim3 grid((cpr + WPB - 1) / WPB, (rows + strip - 1) / strip);
    hipLaunchKernelGGL((copy_kernel<WPB, TILED>), grid, dim3(64 * WPB), 0, 0, src, dst, rows, strip, cpr);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    const int reps = 5;
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((copy_kernel<WPB, TILED>), grid, dim3(64 * WPB), 0, 0, src, dst, rows, strip, cpr);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double bytes = 2.0 * rows * (double)cpr * 1024 * reps;
    printf("%s waves/WG %2d strip %5d: %.0f GB/s (read + write)\n", TILED ? "tiled  " : "rowmajor", WPB, strip,
           bytes / (ms * 1e-3) / 1e9);
}

int main()
{
    const int rows = 1 << 17, cpr = 128;  // 128 KiB rows = 2^20 cells per row, 16 GiB
    uint4 *src, *dst;
    if (hipMalloc(&src, (size_t)rows * cpr * 1024) != hipSuccess || hipMalloc(&dst, (size_t)rows * cpr * 1024) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(src, 0x5a, (size_t)rows * cpr * 1024);
    for (int strip : {512, 1024}) {
        run<4>(src, dst, rows, cpr, strip);
        run<16>(src, dst, rows, cpr, strip);
        run<1, true>(src, dst, rows, cpr, strip);
        run<4, true>(src, dst, rows, cpr, strip);
    }
    return 0;
}
