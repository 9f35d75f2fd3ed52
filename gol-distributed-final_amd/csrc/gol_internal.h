// gol_internal.h -- private state of libgolhip.so (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>

#include "golhip.h"

// Library defaults for the bit-board step (chosen from the gfx950 sweep recorded
// in DESIGN.md; overridable per engine through gol_config).
#ifndef GOL_DEFAULT_K
#define GOL_DEFAULT_K 8        // standard layout
#endif
#ifndef GOL_DEFAULT_BAND_K
#define GOL_DEFAULT_BAND_K 12  // band layout, 4 words per lane: the split pipeline
#endif
#ifndef GOL_DEFAULT_DW
#define GOL_DEFAULT_DW 2
#endif

// Halo rows kept above and below each bit buffer: the band kernel reads the torus wrap
// from them as contiguous rows (its CONTIG path, no per-row segment select).
#define GOL_GHOST_ROWS 16

struct gol_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    int64_t H = 0, W = 0;
    int64_t Wd = 0;      // uint32 words per row (W / 32)
    int64_t pitch = 0;   // bit-board row pitch in uint32 words (multiple of 4)
    int64_t bstride = 0; // byte-board row pitch in bytes (multiple of 16)
    bool bit_capable = false;  // W % 64 == 0
    bool bit_mode = false;     // board currently lives in bits[cur] (else bytes[bcur])
    bool band_capable = false; // step the bit board in the band layout (W % 1024 == 0, not disabled)
    bool band = false;         // bits[cur] currently holds the band layout
    uint32_t *bits[2] = {nullptr, nullptr};       // row 0 of each bit buffer
    uint32_t *bits_alloc[2] = {nullptr, nullptr}; // allocations: GOL_GHOST_ROWS halo rows above and below
    int cur = 0;
    uint8_t *bytes[2] = {nullptr, nullptr};
    int bcur = 0;
    bool bytes_binary = false;  // byte board holds only 0/255 (k-turn byte kernel allowed)
    uint64_t *slots = nullptr;  // GOL_COUNT_SLOTS * 8 uint64 reduction slots
    uint32_t *flag = nullptr;
    uint8_t *staging = nullptr;       // device byte rows for chunked copies
    uint8_t *host_staging = nullptr;  // pinned host rows (PGM writer)
    int64_t stage_rows = 0;
    int64_t turn = 0;
    int k = GOL_DEFAULT_K;
    int dw = GOL_DEFAULT_DW;
    int band_dw = 4;  // words per lane of the band kernel
    int strip = 0;
};

int gol_set_error(int code, const char *fmt, ...);
// Enqueue `turns` turns on e->stream without synchronising.
int gol_engine_step_async(gol_engine *e, int64_t turns, uint64_t *count_slots);
