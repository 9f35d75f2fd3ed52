// gol_abi.cpp -- C ABI of libgolhip.so: library entry points, the worker's slab
// step, the row partition and the device launchers (include/golhip.h).  The
// board engine (one GPU or row shards) is gol_engine.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "golhip.h"
#include "gol_internal.h"
#include "gol_kernels.h"

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;

int gol_set_error(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return gol_set_error(GOL_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                 __FILE__, __LINE__);                                             \
    } while (0)

extern "C" int gol_abi_version(void) { return GOL_ABI_VERSION; }
extern "C" const char *gol_last_error(void) { return g_err.c_str(); }

extern "C" int gol_device_count(int *n)
{
    if (!n) return gol_set_error(GOL_EINVAL, "n is NULL");
    int c = 0;
    HIPCHK(hipGetDeviceCount(&c));
    *n = c;
    return GOL_OK;
}

extern "C" int gol_partition_rows(int64_t H, int64_t parts, int64_t i, int64_t *y0, int64_t *y1)
{
    if (!y0 || !y1 || parts <= 0 || i < 0 || i >= parts || H < 0)
        return gol_set_error(GOL_EINVAL, "bad partition arguments H=%lld parts=%lld i=%lld", (long long)H,
                             (long long)parts, (long long)i);
    // broker.go:135-139 (even) and broker.go:172-206 (first H%T slabs get one extra row)
    const int64_t base = H / parts, rem = H % parts;
    *y0 = i * base + std::min(i, rem);
    *y1 = *y0 + base + (i < rem ? 1 : 0);
    return GOL_OK;
}

// ------------------------------------------------------------------ worker path
extern "C" int gol_next_state_slab(const uint8_t *world, int64_t H, int64_t W, int64_t stride, int64_t y0,
                                   int64_t y1, uint8_t *out, int64_t out_stride)
{
    if (!world || !out || H <= 0 || W <= 0 || stride < W || out_stride < W || y0 < 0 || y1 > H || y0 > y1)
        return gol_set_error(GOL_EINVAL, "bad slab arguments H=%lld W=%lld y0=%lld y1=%lld", (long long)H,
                             (long long)W, (long long)y0, (long long)y1);
    if (y0 == y1) return GOL_OK;
    const int64_t ds = (W + 15) / 16 * 16;
    uint8_t *dworld = nullptr, *dout = nullptr;
    hipStream_t s = nullptr;
    int rc = GOL_OK;
    auto fail = [&](hipError_t e, const char *what) {
        rc = gol_set_error(GOL_EHIP, "%s: %s", what, hipGetErrorString(e));
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) { fail(e, "stream"); return rc; }
    if ((e = hipMalloc(&dworld, H * ds)) != hipSuccess) fail(e, "hipMalloc world");
    else if ((e = hipMalloc(&dout, (y1 - y0) * ds)) != hipSuccess) fail(e, "hipMalloc slab");
    else if ((e = hipMemcpy2DAsync(dworld, ds, world, stride, W, H, hipMemcpyHostToDevice, s)) != hipSuccess)
        fail(e, "copy in");
    else if ((e = golk_bytes_step(dworld, H, W, ds, y0, y1, dout, ds, s)) != hipSuccess) fail(e, "launch");
    else if ((e = hipMemcpy2DAsync(out, out_stride, dout, ds, W, y1 - y0, hipMemcpyDeviceToHost, s)) != hipSuccess)
        fail(e, "copy out");
    else if ((e = hipStreamSynchronize(s)) != hipSuccess) fail(e, "sync");
    if (dworld) (void)hipFree(dworld);
    if (dout) (void)hipFree(dout);
    (void)hipStreamDestroy(s);
    return rc;
}

// ------------------------------------------------------------------ device launchers
#define LAUNCH(expr)                                                                                      \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess) return gol_set_error(GOL_EHIP, "%s: %s", #expr, hipGetErrorString(e_));     \
        return GOL_OK;                                                                                    \
    } while (0)

extern "C" int gol_dev_bits_step(const uint32_t *top, const uint32_t *mid, const uint32_t *bot, uint32_t *dst,
                                 int64_t R, int64_t Wd, int64_t pitch, int64_t row0, int64_t rows, int32_t k,
                                 int32_t cells_per_lane, int32_t strip_rows, uint64_t *count_slots, void *stream)
{
    const int dw = cells_per_lane > 0 ? cells_per_lane / 32 : GOL_DEFAULT_DW;
    if (!top || !mid || !bot || !dst || R <= 0 || Wd <= 0 || pitch < Wd || row0 < 0 || rows < 0 ||
        row0 + rows > R || (dw != 1 && dw != 2 && dw != 4) || Wd % dw || pitch % dw ||
        !(k == 1 || k == 2 || k == 4 || k == 8 || (k == 16 && dw <= 2)) || k > R)
        return gol_set_error(GOL_EINVAL, "bad bits_step arguments (R=%lld Wd=%lld pitch=%lld k=%d dw=%d)",
                             (long long)R, (long long)Wd, (long long)pitch, k, dw);
    LAUNCH(golk_bits_step(top, mid, bot, dst, R, Wd, pitch, row0, rows, k, dw, strip_rows, count_slots,
                          (hipStream_t)stream));
}

extern "C" int gol_dev_band_step(const uint32_t *top, const uint32_t *mid, const uint32_t *bot, uint32_t *dst,
                                 int64_t R, int64_t Wd, int64_t pitch, int64_t row0, int64_t rows, int32_t k,
                                 int32_t cells_per_lane, int32_t strip_rows, uint64_t *count_slots, void *stream)
{
    const int dw = cells_per_lane == 64 ? 2 : (cells_per_lane == 128 ? 4 : (cells_per_lane <= 0 ? GOL_BAND_DEFAULT_DW : 0));
    if (!top || !mid || !bot || !dst || R <= 0 || Wd <= 0 || !dw || Wd % dw || pitch < Wd || pitch % dw ||
        row0 < 0 || rows < 0 || row0 + rows > R ||
        !(k == 1 || k == 2 || k == 4 || k == 8 || (k == 16 && dw == 2) || (k == 12 && dw == 4)) ||
        k > R || (((uintptr_t)mid | (uintptr_t)top | (uintptr_t)bot | (uintptr_t)dst) & (4 * dw - 1)))
        return gol_set_error(GOL_EINVAL, "bad band_step arguments (R=%lld Wd=%lld pitch=%lld k=%d cells_per_lane=%d)",
                             (long long)R, (long long)Wd, (long long)pitch, k, cells_per_lane);
    LAUNCH(golk_band_step(top, mid, bot, dst, R, Wd, pitch, row0, rows, k, dw, strip_rows, count_slots, nullptr,
                          (hipStream_t)stream));
}

extern "C" int gol_band_max_k(int32_t cells_per_lane)
{
    const int dw = cells_per_lane == 64 ? 2 : (cells_per_lane == 128 ? 4 : (cells_per_lane <= 0 ? GOL_BAND_DEFAULT_DW : 0));
    return dw == 2 ? 16 : (dw == 4 ? 12 : 0);
}

extern "C" int gol_dev_band_convert(int32_t to_band, const uint32_t *src, uint32_t *dst, int64_t rows, int64_t Wd,
                                    int64_t src_pitch, int64_t dst_pitch, void *stream)
{
    if (!src || !dst || src == dst || rows < 0 || Wd <= 0 || Wd % 32 || src_pitch < Wd || dst_pitch < Wd ||
        (to_band ? dst_pitch : src_pitch) % 4 || (((uintptr_t)(to_band ? dst : src)) & 15))
        return gol_set_error(GOL_EINVAL, "bad band_convert arguments (Wd=%lld)", (long long)Wd);
    LAUNCH(golk_band_convert(to_band != 0, src, dst, rows, Wd, src_pitch, dst_pitch, (hipStream_t)stream));
}

extern "C" int gol_dev_random_fill(uint32_t *dst, int64_t rows, int64_t grow0, int64_t W, int64_t pitch,
                                   uint64_t seed, void *stream)
{
    if (!dst || rows < 0 || grow0 < 0 || W <= 0 || W % 64 || pitch < W / 32 || pitch % 2)
        return gol_set_error(GOL_EINVAL, "bad random_fill arguments");
    LAUNCH(golk_random_fill(dst, rows, grow0, W, pitch, seed, (hipStream_t)stream));
}

extern "C" int gol_dev_popcount(const uint32_t *src, int64_t rows, int64_t Wd, int64_t pitch, uint64_t *slots,
                                void *stream)
{
    if (!src || !slots || rows < 0 || Wd <= 0 || pitch < Wd) return gol_set_error(GOL_EINVAL, "bad popcount arguments");
    LAUNCH(golk_popcount(src, rows, Wd, pitch, slots, (hipStream_t)stream));
}

extern "C" int gol_dev_hash(const uint32_t *src, int64_t rows, int64_t grow0, int64_t Wd, int64_t pitch,
                            uint64_t *slots, void *stream)
{
    if (!src || !slots || rows < 0 || grow0 < 0 || Wd <= 0 || Wd % 2 || pitch < Wd || pitch % 2)
        return gol_set_error(GOL_EINVAL, "bad hash arguments");
    LAUNCH(golk_hash(src, rows, grow0, Wd, pitch, slots, (hipStream_t)stream));
}

extern "C" int gol_dev_pack(const uint8_t *bytes, int64_t rows, int64_t W, int64_t stride, uint32_t *bits,
                            int64_t pitch, uint32_t *nonbinary, void *stream)
{
    if (!bytes || !bits || rows < 0 || W <= 0 || W % 32 || stride < W || pitch < W / 32)
        return gol_set_error(GOL_EINVAL, "bad pack arguments");
    LAUNCH(golk_pack(bytes, rows, W, stride, bits, pitch, nonbinary, (hipStream_t)stream));
}

extern "C" int gol_dev_unpack(const uint32_t *bits, int64_t rows, int64_t W, int64_t pitch, uint8_t *bytes,
                              int64_t stride, void *stream)
{
    if (!bytes || !bits || rows < 0 || W <= 0 || W % 32 || stride < W || pitch < W / 32)
        return gol_set_error(GOL_EINVAL, "bad unpack arguments");
    LAUNCH(golk_unpack(bits, rows, W, pitch, bytes, stride, (hipStream_t)stream));
}

extern "C" int gol_dev_bytes_step_k(const uint8_t *top, const uint8_t *mid, const uint8_t *bot, uint8_t *dst,
                                    int64_t R, int64_t W, int64_t stride, int64_t row0, int64_t rows, int32_t k,
                                    int32_t strip_rows, uint64_t *count_slots, void *stream)
{
    if (!top || !mid || !bot || !dst || R <= 0 || W <= 0 || W % 32 || stride < W || stride % 16 || row0 < 0 ||
        rows < 0 || row0 + rows > R || !(k == 1 || k == 2 || k == 4 || k == 8 || k == 16 || k == 32) || k > R ||
        (((uintptr_t)mid | (uintptr_t)top | (uintptr_t)bot | (uintptr_t)dst) & 15))
        return gol_set_error(GOL_EINVAL, "bad bytes_step_k arguments (R=%lld W=%lld stride=%lld k=%d)",
                             (long long)R, (long long)W, (long long)stride, k);
    LAUNCH(golk_bytes_blocked(top, mid, bot, dst, R, W, stride, row0, rows, k, strip_rows, count_slots, nullptr,
                              (hipStream_t)stream));
}

extern "C" int gol_dev_bytes_step(const uint8_t *world, int64_t H, int64_t W, int64_t stride, int64_t y0,
                                  int64_t y1, uint8_t *out, int64_t out_stride, void *stream)
{
    if (!world || !out || H <= 0 || W <= 0 || stride < W || out_stride < W || y0 < 0 || y1 > H || y0 > y1)
        return gol_set_error(GOL_EINVAL, "bad bytes_step arguments");
    LAUNCH(golk_bytes_step(world, H, W, stride, y0, y1, out, out_stride, (hipStream_t)stream));
}

extern "C" int gol_dev_error(int32_t device, uint32_t *flags)
{
    if (!flags) return gol_set_error(GOL_EINVAL, "flags is NULL");
    int dev = device;
    if (dev < 0) HIPCHK(hipGetDevice(&dev));
    int prev = 0;
    HIPCHK(hipGetDevice(&prev));
    uint32_t *w = golk_device_err_word(dev);
    if (!w) return gol_set_error(GOL_EHIP, "no error word on device %d", dev);
    HIPCHK(hipSetDevice(dev));
    uint32_t v = 0;
    hipError_t he = hipMemcpy(&v, w, sizeof v, hipMemcpyDeviceToHost);
    if (he == hipSuccess && v) he = hipMemset(w, 0, sizeof v);
    if (he == hipSuccess && v) he = golk_reset_claims_device(dev);  // a timed-out pair may have left its claims set
    (void)hipSetDevice(prev);
    if (he != hipSuccess) return gol_set_error(GOL_EHIP, "error word: %s", hipGetErrorString(he));
    *flags = v;
    if (v) return gol_set_error(GOL_EHIP, "device fault in a launch on device %d (error flags 0x%x)", dev, v);
    return GOL_OK;
}
