// gol_abi.cpp -- C ABI of libgolhip.so: library entry points, the single-GPU
// engine and the device launchers (include/golhip.h).
//
// The engine keeps the board resident in HBM and replaces the reference's
// per-turn state handling in broker.go:62-234 (scatter of the whole board to
// every worker, gather of the slabs, mirror copy into cWorld) with k-turn
// kernel launches on a double-buffered bit board.
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

// ------------------------------------------------------------------ engine
// Turns per launch: the largest supported k <= want, remaining turns and rows.  k = 12 is
// the band layout's split pipeline (4 words per lane, band = true); k = 16 needs <= 2 words.
static int pick_k(int want, int64_t remaining, int64_t H, int dw, bool band = false)
{
    static const int ks[] = {16, 12, 8, 4, 2, 1};
    for (int k : ks) {
        if (k == 16 && dw > 2) continue;
        if (k == 12 && !(band && dw == 4)) continue;
        if (k <= want && k <= remaining && k <= H) return k;
    }
    return 1;
}

static int engine_dev(gol_engine *e)
{
    HIPCHK(hipSetDevice(e->device));
    return GOL_OK;
}

// The band layout is a stepping detail: convert on the first step, convert back
// before anything reads the bits.  Both are one HBM pass (32x32 bit transposes).
static int to_band(gol_engine *e)
{
    if (e->band) return GOL_OK;
    HIPCHK(golk_band_convert(true, e->bits[e->cur], e->bits[1 - e->cur], e->H, e->Wd, e->pitch, e->pitch, e->stream));
    e->cur = 1 - e->cur;
    e->band = true;
    return GOL_OK;
}

static int ensure_standard(gol_engine *e)
{
    if (!e->bit_mode || !e->band) return GOL_OK;
    HIPCHK(golk_band_convert(false, e->bits[e->cur], e->bits[1 - e->cur], e->H, e->Wd, e->pitch, e->pitch,
                             e->stream));
    e->cur = 1 - e->cur;
    e->band = false;
    return GOL_OK;
}

static void free_bytes(gol_engine *e)
{
    for (auto &b : e->bytes)
        if (b) { (void)hipFree(b); b = nullptr; }
}

static int alloc_bytes(gol_engine *e)
{
    for (auto &b : e->bytes)
        if (!b) HIPCHK(hipMalloc(&b, e->H * e->bstride));
    return GOL_OK;
}

static int ensure_staging(gol_engine *e)
{
    if (!e->staging) {
        // byte staging for chunked load/store/PGM: >= 1 row, <= 64 MiB
        e->stage_rows = std::max<int64_t>(1, std::min<int64_t>(e->H, (64LL << 20) / e->bstride));
        HIPCHK(hipMalloc(&e->staging, e->stage_rows * e->bstride));
        HIPCHK(hipHostMalloc((void **)&e->host_staging, e->stage_rows * e->bstride, hipHostMallocDefault));
    }
    return GOL_OK;
}

extern "C" int gol_engine_create(int64_t H, int64_t W, const gol_config *cfg, gol_engine **out)
{
    if (!out || H <= 0 || W <= 0 || W > (int64_t)INT32_MAX * 32 || H > INT32_MAX)
        return gol_set_error(GOL_EINVAL, "bad board size %lldx%lld", (long long)W, (long long)H);
    *out = nullptr;
    gol_engine *e = new gol_engine();
    e->H = H;
    e->W = W;
    e->bit_capable = (W % 64) == 0;
    e->Wd = W / 32;
    e->pitch = (e->Wd + 3) / 4 * 4;
    e->bstride = (W + 15) / 16 * 16;
    int dev = cfg ? cfg->device : -1;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    }
    e->device = dev;
    e->k = (cfg && cfg->turns_per_launch > 0) ? cfg->turns_per_launch : 0;  // 0: per layout, below
    int cpl = (cfg && cfg->cells_per_lane > 0) ? cfg->cells_per_lane : 32 * GOL_DEFAULT_DW;
    if (cpl != 32 && cpl != 64 && cpl != 128) {
        delete e;
        return gol_set_error(GOL_EINVAL, "cells_per_lane must be 32, 64 or 128");
    }
    e->dw = cpl / 32;
    while (e->dw > 1 && (e->Wd % e->dw) != 0) e->dw >>= 1;
    const int req = cfg ? cfg->cells_per_lane : 0;
    e->band_dw = req == 64 ? 2 : (req == 128 ? 4 : GOL_BAND_DEFAULT_DW);
    e->strip = cfg ? cfg->strip_rows : 0;
    const int layout = cfg ? cfg->layout : GOL_LAYOUT_AUTO;
    if (layout != GOL_LAYOUT_AUTO && layout != GOL_LAYOUT_STANDARD && layout != GOL_LAYOUT_BAND) {
        delete e;
        return gol_set_error(GOL_EINVAL, "layout must be GOL_LAYOUT_AUTO, _STANDARD or _BAND");
    }
    if (layout == GOL_LAYOUT_BAND && W % 1024 != 0) {
        delete e;
        return gol_set_error(GOL_EINVAL, "the band layout needs W %% 1024 == 0");
    }
    e->band_capable = layout != GOL_LAYOUT_STANDARD && W % 1024 == 0;
    if (e->k == 0) e->k = (e->band_capable && e->band_dw == 4) ? GOL_DEFAULT_BAND_K : GOL_DEFAULT_K;
    int rc = engine_dev(e);
    if (rc == GOL_OK) {
        hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
        if (he == hipSuccess) he = hipMalloc(&e->slots, GOL_COUNT_SLOTS * 8 * sizeof(uint64_t));
        if (he == hipSuccess) he = hipMalloc(&e->flag, sizeof(uint32_t));
        if (he == hipSuccess && e->bit_capable) {
            const int64_t rows = H + 2 * GOL_GHOST_ROWS;
            for (int i = 0; i < 2; ++i) {
                he = hipMalloc(&e->bits_alloc[i], rows * e->pitch * sizeof(uint32_t));
                if (he != hipSuccess) break;
                // on the engine's stream: it is non-blocking, so a null-stream memset could still
                // be running when the first load or fill kernel writes the board
                he = hipMemsetAsync(e->bits_alloc[i], 0, rows * e->pitch * sizeof(uint32_t), e->stream);
                if (he != hipSuccess) break;
                e->bits[i] = e->bits_alloc[i] + GOL_GHOST_ROWS * e->pitch;
            }
            e->bit_mode = true;
        }
        if (he == hipSuccess && !e->bit_capable) {
            rc = alloc_bytes(e);
            if (rc == GOL_OK) he = hipMemsetAsync(e->bytes[0], 0, H * e->bstride, e->stream);
            e->bit_mode = false;
        }
        if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
        if (he != hipSuccess)
            rc = gol_set_error(he == hipErrorOutOfMemory ? GOL_ENOMEM : GOL_EHIP, "engine allocation: %s",
                               hipGetErrorString(he));
    }
    if (rc != GOL_OK) {
        gol_engine_destroy(e);
        return rc;
    }
    *out = e;
    return GOL_OK;
}

extern "C" void gol_engine_destroy(gol_engine *e)
{
    if (!e) return;
    (void)hipSetDevice(e->device);
    for (auto &b : e->bits_alloc)
        if (b) (void)hipFree(b);
    free_bytes(e);
    if (e->slots) (void)hipFree(e->slots);
    if (e->flag) (void)hipFree(e->flag);
    if (e->staging) (void)hipFree(e->staging);
    if (e->host_staging) (void)hipHostFree(e->host_staging);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

extern "C" int gol_engine_load_bytes(gol_engine *e, const uint8_t *world, int64_t stride)
{
    if (!e || !world || stride < e->W) return gol_set_error(GOL_EINVAL, "bad load arguments");
    int rc = engine_dev(e);
    if (rc) return rc;
    e->turn = 0;
    e->band = false;
    if (!e->bit_capable) {
        HIPCHK(hipMemcpy2DAsync(e->bytes[0], e->bstride, world, stride, e->W, e->H, hipMemcpyHostToDevice,
                                e->stream));
        e->bcur = 0;
        HIPCHK(hipMemsetAsync(e->flag, 0, sizeof(uint32_t), e->stream));
        HIPCHK(golk_nonbinary(e->bytes[0], e->H, e->W, e->bstride, e->flag, e->stream));
        uint32_t nb = 0;
        HIPCHK(hipMemcpyAsync(&nb, e->flag, sizeof nb, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        e->bytes_binary = nb == 0;
        return GOL_OK;
    }
    // pack row chunks into the bit board; remember whether any byte is neither 0 nor 255
    if ((rc = ensure_staging(e))) return rc;
    HIPCHK(hipMemsetAsync(e->flag, 0, sizeof(uint32_t), e->stream));
    e->cur = 0;
    for (int64_t y = 0; y < e->H; y += e->stage_rows) {
        const int64_t n = std::min(e->stage_rows, e->H - y);
        HIPCHK(hipMemcpy2DAsync(e->staging, e->bstride, world + y * stride, stride, e->W, n,
                                hipMemcpyHostToDevice, e->stream));
        HIPCHK(golk_pack(e->staging, n, e->W, e->bstride, e->bits[0] + y * e->pitch, e->pitch, e->flag, e->stream));
    }
    uint32_t nonbinary = 0;
    HIPCHK(hipMemcpyAsync(&nonbinary, e->flag, sizeof nonbinary, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (nonbinary) {
        // exact first turn needs the bytes (worker.go:26-37): keep a byte board until turn 1
        if ((rc = alloc_bytes(e))) return rc;
        HIPCHK(hipMemcpy2DAsync(e->bytes[0], e->bstride, world, stride, e->W, e->H, hipMemcpyHostToDevice,
                                e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        e->bcur = 0;
        e->bytes_binary = false;
        e->bit_mode = false;
    } else {
        free_bytes(e);
        e->bit_mode = true;
    }
    return GOL_OK;
}

extern "C" int gol_engine_load_random(gol_engine *e, uint64_t seed)
{
    if (!e) return gol_set_error(GOL_EINVAL, "engine is NULL");
    if (!e->bit_capable) return gol_set_error(GOL_EINVAL, "random boards need W %% 64 == 0");
    int rc = engine_dev(e);
    if (rc) return rc;
    free_bytes(e);
    e->bit_mode = true;
    e->band = false;
    e->cur = 0;
    e->turn = 0;
    HIPCHK(golk_random_fill(e->bits[0], e->H, 0, e->W, e->pitch, seed, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return GOL_OK;
}

int gol_engine_step_async(gol_engine *e, int64_t turns, uint64_t *count_slots)
{
    while (turns > 0) {
        if (!e->bit_mode && e->bytes_binary && e->W % 32 == 0) {
            // 0/255 byte board: k turns per launch on the bytes (torus wrap through top/bot)
            const int k = pick_k(e->k, turns, e->H, 1);
            const uint8_t *mid = e->bytes[e->bcur];
            HIPCHK(golk_bytes_blocked(mid + (e->H - k) * e->bstride, mid, mid, e->bytes[1 - e->bcur], e->H, e->W,
                                      e->bstride, 0, e->H, k, e->strip, turns == k ? count_slots : nullptr,
                                      e->stream));
            e->bcur = 1 - e->bcur;
            e->turn += k;
            turns -= k;
            continue;
        }
        if (!e->bit_mode) {
            const int nb = 1 - e->bcur;
            HIPCHK(golk_bytes_step(e->bytes[e->bcur], e->H, e->W, e->bstride, 0, e->H, e->bytes[nb], e->bstride,
                                   e->stream));
            e->bcur = nb;
            e->turn += 1;
            turns -= 1;
            e->bytes_binary = true;  // one exact turn leaves only 0/255
            if (e->bit_capable) {
                // board is now strictly 0/255: continue on the bit board
                HIPCHK(golk_pack(e->bytes[e->bcur], e->H, e->W, e->bstride, e->bits[0], e->pitch, nullptr,
                                 e->stream));
                HIPCHK(hipStreamSynchronize(e->stream));
                free_bytes(e);
                e->cur = 0;
                e->band = false;
                e->bit_mode = true;
            }
            continue;
        }
        if (e->band_capable) {
            // band layout: a lane of band_dw words keeps 2*ceil(k/band_dw) halo lanes per wave
            const int k = pick_k(e->k, turns, e->H, e->band_dw, true);
            int rc = to_band(e);
            if (rc) return rc;
            // torus wrap rows into the halo rows right above / below the board (contiguous rows)
            uint32_t *mid = e->bits[e->cur];
            const size_t hb = (size_t)k * e->pitch * sizeof(uint32_t);
            HIPCHK(hipMemcpyAsync(mid - k * e->pitch, mid + (e->H - k) * e->pitch, hb, hipMemcpyDeviceToDevice,
                                  e->stream));
            HIPCHK(hipMemcpyAsync(mid + e->H * e->pitch, mid, hb, hipMemcpyDeviceToDevice, e->stream));
            HIPCHK(golk_band_step(mid - k * e->pitch, mid, mid + e->H * e->pitch, e->bits[1 - e->cur], e->H, e->Wd,
                                  e->pitch, 0, e->H, k, e->band_dw, e->strip, turns == k ? count_slots : nullptr,
                                  e->stream));
            e->cur = 1 - e->cur;
            e->turn += k;
            turns -= k;
            continue;
        }
        const int k = pick_k(e->k, turns, e->H, e->dw);
        const uint32_t *mid = e->bits[e->cur];
        uint32_t *dst = e->bits[1 - e->cur];
        const bool last = turns == k;
        HIPCHK(golk_bits_step(mid + (e->H - k) * e->pitch, mid, mid, dst, e->H, e->Wd, e->pitch, 0, e->H, k, e->dw,
                              e->strip, last ? count_slots : nullptr, e->stream));
        e->cur = 1 - e->cur;
        e->turn += k;
        turns -= k;
    }
    return GOL_OK;
}

extern "C" int gol_engine_step(gol_engine *e, int64_t turns)
{
    if (!e || turns < 0) return gol_set_error(GOL_EINVAL, "bad step arguments");
    int rc = engine_dev(e);
    if (rc) return rc;
    if ((rc = gol_engine_step_async(e, turns, nullptr))) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    return GOL_OK;
}

extern "C" int gol_engine_turn(gol_engine *e, int64_t *turn)
{
    if (!e || !turn) return gol_set_error(GOL_EINVAL, "bad arguments");
    *turn = e->turn;
    return GOL_OK;
}

static int sum_slots(gol_engine *e, uint64_t *out)
{
    std::vector<uint64_t> h(GOL_COUNT_SLOTS * 8);
    HIPCHK(hipMemcpyAsync(h.data(), e->slots, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t s = 0;
    for (int i = 0; i < GOL_COUNT_SLOTS; ++i) s += h[i * 8];
    *out = s;
    return GOL_OK;
}

extern "C" int gol_engine_alive_count(gol_engine *e, uint64_t *count)
{
    if (!e || !count) return gol_set_error(GOL_EINVAL, "bad arguments");
    int rc = engine_dev(e);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(e->slots, 0, GOL_COUNT_SLOTS * 8 * sizeof(uint64_t), e->stream));
    if (e->bit_mode)
        HIPCHK(golk_popcount(e->bits[e->cur], e->H, e->Wd, e->pitch, e->slots, e->stream));
    else
        HIPCHK(golk_count_bytes(e->bytes[e->bcur], e->H, e->W, e->bstride, e->slots, e->stream));
    return sum_slots(e, count);
}

extern "C" int gol_engine_store_bytes(gol_engine *e, uint8_t *out, int64_t stride)
{
    if (!e || !out || stride < e->W) return gol_set_error(GOL_EINVAL, "bad store arguments");
    int rc = engine_dev(e);
    if (rc || (rc = ensure_standard(e))) return rc;
    if (!e->bit_mode) {
        HIPCHK(hipMemcpy2DAsync(out, stride, e->bytes[e->bcur], e->bstride, e->W, e->H, hipMemcpyDeviceToHost,
                                e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        return GOL_OK;
    }
    if ((rc = ensure_staging(e))) return rc;
    for (int64_t y = 0; y < e->H; y += e->stage_rows) {
        const int64_t n = std::min(e->stage_rows, e->H - y);
        HIPCHK(golk_unpack(e->bits[e->cur] + y * e->pitch, n, e->W, e->pitch, e->staging, e->bstride, e->stream));
        HIPCHK(hipMemcpy2DAsync(out + y * stride, stride, e->staging, e->bstride, e->W, n, hipMemcpyDeviceToHost,
                                e->stream));
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    return GOL_OK;
}

// Row-major (x, y) list of the cells of `board` that are alive (prev == NULL) or whose alive
// state differs from `prev`: per-row counts -> host exclusive scan -> one wave per row.
static int list_cells(gol_engine *e, bool bm, const void *board, const void *prev, int64_t units, int64_t pitch,
                      int32_t *xy, int64_t cap, int64_t *n, const char *what)
{
    int64_t *dcounts = nullptr;
    int32_t *dxy = nullptr;
    std::vector<int64_t> counts(e->H);
    HIPCHK(hipMalloc(&dcounts, e->H * sizeof(int64_t)));
    hipError_t he = golk_row_counts(bm, board, prev, e->H, units, pitch, dcounts, e->stream);
    if (he == hipSuccess)
        he = hipMemcpyAsync(counts.data(), dcounts, e->H * sizeof(int64_t), hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    int64_t total = 0;
    if (he == hipSuccess) {
        for (auto &c : counts) {  // exclusive prefix -> first index of each row
            const int64_t v = c;
            c = total;
            total += v;
        }
        *n = total;
    }
    const int64_t m = std::min(total, cap);
    if (he == hipSuccess && m > 0) {
        he = hipMemcpyAsync(dcounts, counts.data(), e->H * sizeof(int64_t), hipMemcpyHostToDevice, e->stream);
        if (he == hipSuccess) he = hipMalloc(&dxy, m * 2 * sizeof(int32_t));
        if (he == hipSuccess)
            he = golk_alive_list(bm, board, prev, e->H, units, pitch, dcounts, dxy, m, e->stream);
        if (he == hipSuccess)
            he = hipMemcpyAsync(xy, dxy, m * 2 * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream);
        if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    }
    (void)hipFree(dcounts);
    if (dxy) (void)hipFree(dxy);
    if (he != hipSuccess) return gol_set_error(GOL_EHIP, "%s: %s", what, hipGetErrorString(he));
    return GOL_OK;
}

extern "C" int gol_engine_alive_cells(gol_engine *e, int32_t *xy, int64_t cap, int64_t *n)
{
    if (!e || !n || cap < 0 || (cap > 0 && !xy)) return gol_set_error(GOL_EINVAL, "bad arguments");
    int rc = engine_dev(e);
    if (rc || (rc = ensure_standard(e))) return rc;
    const bool bm = e->bit_mode;
    const void *board = bm ? (const void *)e->bits[e->cur] : (const void *)e->bytes[e->bcur];
    return list_cells(e, bm, board, nullptr, bm ? e->Wd : e->W, bm ? e->pitch : e->bstride, xy, cap, n,
                      "alive_cells");
}

extern "C" int gol_engine_step_flips(gol_engine *e, int32_t *xy, int64_t cap, int64_t *n)
{
    if (!e || !n || cap < 0 || (cap > 0 && !xy)) return gol_set_error(GOL_EINVAL, "bad arguments");
    int rc = engine_dev(e);
    if (rc || (rc = ensure_standard(e))) return rc;
    if (e->bit_mode) {
        // one standard-layout turn; the previous generation stays in the other buffer
        const uint32_t *mid = e->bits[e->cur];
        HIPCHK(golk_bits_step(mid + (e->H - 1) * e->pitch, mid, mid, e->bits[1 - e->cur], e->H, e->Wd, e->pitch, 0,
                              e->H, 1, e->dw, e->strip, nullptr, e->stream));
        e->cur = 1 - e->cur;
        e->turn += 1;
        return list_cells(e, true, e->bits[e->cur], e->bits[1 - e->cur], e->Wd, e->pitch, xy, cap, n,
                          "step_flips");
    }
    // byte board (loaded bytes other than 0/255, or W % 64 != 0): keep the previous bytes; the
    // turn may move the board to the bit board, whose bytes are unpacked for the comparison
    uint8_t *prev = nullptr, *now = nullptr;
    HIPCHK(hipMalloc(&prev, e->H * e->bstride));
    hipError_t he = hipMemcpyAsync(prev, e->bytes[e->bcur], e->H * e->bstride, hipMemcpyDeviceToDevice, e->stream);
    if (he == hipSuccess && (rc = gol_engine_step_async(e, 1, nullptr)) == GOL_OK) {
        const uint8_t *cur = e->bit_mode ? nullptr : e->bytes[e->bcur];
        if (e->bit_mode) {
            he = hipMalloc(&now, e->H * e->bstride);
            if (he == hipSuccess)
                he = golk_unpack(e->bits[e->cur], e->H, e->W, e->pitch, now, e->bstride, e->stream);
            cur = now;
        }
        if (he == hipSuccess) rc = list_cells(e, false, cur, prev, e->W, e->bstride, xy, cap, n, "step_flips");
    }
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    (void)hipFree(prev);
    if (now) (void)hipFree(now);
    if (rc == GOL_OK && he != hipSuccess) rc = gol_set_error(GOL_EHIP, "step_flips: %s", hipGetErrorString(he));
    return rc;
}

extern "C" int gol_engine_write_pgm(gol_engine *e, const char *path)
{
    if (!e || !path) return gol_set_error(GOL_EINVAL, "bad arguments");
    int rc = engine_dev(e);
    if (rc || (rc = ensure_standard(e))) return rc;
    if ((rc = ensure_staging(e))) return rc;
    FILE *f = fopen(path, "wb");
    if (!f) return gol_set_error(GOL_EIO, "cannot create %s", path);
    // gol/io.go:52-59 header
    fprintf(f, "P5\n%lld %lld\n255\n", (long long)e->W, (long long)e->H);
    for (int64_t y = 0; y < e->H && rc == GOL_OK; y += e->stage_rows) {
        const int64_t n = std::min(e->stage_rows, e->H - y);
        hipError_t he;
        if (e->bit_mode) {
            he = golk_unpack(e->bits[e->cur] + y * e->pitch, n, e->W, e->pitch, e->staging, e->bstride, e->stream);
            if (he == hipSuccess)
                he = hipMemcpy2DAsync(e->host_staging, e->W, e->staging, e->bstride, e->W, n, hipMemcpyDeviceToHost,
                                      e->stream);
        } else {
            he = hipMemcpy2DAsync(e->host_staging, e->W, e->bytes[e->bcur] + y * e->bstride, e->bstride, e->W, n,
                                  hipMemcpyDeviceToHost, e->stream);
        }
        if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
        if (he != hipSuccess) rc = gol_set_error(GOL_EHIP, "write_pgm: %s", hipGetErrorString(he));
        else if (fwrite(e->host_staging, 1, (size_t)(n * e->W), f) != (size_t)(n * e->W))
            rc = gol_set_error(GOL_EIO, "short write to %s", path);
    }
    if (fclose(f) != 0 && rc == GOL_OK) rc = gol_set_error(GOL_EIO, "close %s", path);
    return rc;
}

extern "C" int gol_engine_hash(gol_engine *e, uint64_t *hash)
{
    if (!e || !hash) return gol_set_error(GOL_EINVAL, "bad arguments");
    if (!e->bit_capable) return gol_set_error(GOL_EINVAL, "hash needs W %% 64 == 0");
    int rc = engine_dev(e);
    if (rc || (rc = ensure_standard(e))) return rc;
    HIPCHK(hipMemsetAsync(e->slots, 0, GOL_COUNT_SLOTS * 8 * sizeof(uint64_t), e->stream));
    const uint32_t *bits = e->bits[e->cur];
    if (!e->bit_mode) {  // loaded non-binary bytes at turn 0: hash the 255-cells
        HIPCHK(golk_pack(e->bytes[e->bcur], e->H, e->W, e->bstride, e->bits[1 - e->cur], e->pitch, nullptr,
                         e->stream));
        bits = e->bits[1 - e->cur];
    }
    HIPCHK(golk_hash(bits, e->H, 0, e->Wd, e->pitch, e->slots, e->stream));
    return sum_slots(e, hash);
}

extern "C" int gol_engine_info(gol_engine *e, int32_t *k, int32_t *cells_per_lane, int32_t *strip_rows,
                               int32_t *bit_mode)
{
    if (!e) return gol_set_error(GOL_EINVAL, "engine is NULL");
    const bool band = e->bit_mode && e->band_capable;
    const int dw = band ? e->band_dw : e->dw;
    const int kk = pick_k(e->k, e->k, e->H, dw, band);
    if (k) *k = kk;
    if (cells_per_lane) *cells_per_lane = 32 * dw;
    if (strip_rows) {
        const int64_t u = band ? golk_band_useful_words(kk, dw) : 62 * dw;
        const int64_t ng = (e->Wd + u - 1) / u;
        *strip_rows = e->strip > 0 ? e->strip : golk_auto_strip(e->H, ng, kk);
    }
    if (bit_mode) *bit_mode = e->bit_mode ? (band ? 2 : 1) : 0;
    return GOL_OK;
}

extern "C" int gol_engine_device_bits(gol_engine *e, uint32_t **bits, int64_t *pitch)
{
    if (!e || !bits || !pitch) return gol_set_error(GOL_EINVAL, "bad arguments");
    if (!e->bit_mode) return gol_set_error(GOL_ESTATE, "board is not bit-resident");
    int rc = engine_dev(e);
    if (rc || (rc = ensure_standard(e))) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    *bits = e->bits[e->cur];
    *pitch = e->pitch;
    return GOL_OK;
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
        !(k == 1 || k == 2 || k == 4 || k == 8 || (k == 16 && dw == 2) || ((k == 12 || k == 24) && dw == 4)) ||
        k > R || (((uintptr_t)mid | (uintptr_t)top | (uintptr_t)bot | (uintptr_t)dst) & (4 * dw - 1)))
        return gol_set_error(GOL_EINVAL, "bad band_step arguments (R=%lld Wd=%lld pitch=%lld k=%d cells_per_lane=%d)",
                             (long long)R, (long long)Wd, (long long)pitch, k, cells_per_lane);
    LAUNCH(golk_band_step(top, mid, bot, dst, R, Wd, pitch, row0, rows, k, dw, strip_rows, count_slots,
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
    LAUNCH(golk_bytes_blocked(top, mid, bot, dst, R, W, stride, row0, rows, k, strip_rows, count_slots,
                              (hipStream_t)stream));
}

extern "C" int gol_dev_bytes_step(const uint8_t *world, int64_t H, int64_t W, int64_t stride, int64_t y0,
                                  int64_t y1, uint8_t *out, int64_t out_stride, void *stream)
{
    if (!world || !out || H <= 0 || W <= 0 || stride < W || out_stride < W || y0 < 0 || y1 > H || y0 > y1)
        return gol_set_error(GOL_EINVAL, "bad bytes_step arguments");
    LAUNCH(golk_bytes_step(world, H, W, stride, y0, y1, out, out_stride, (hipStream_t)stream));
}
