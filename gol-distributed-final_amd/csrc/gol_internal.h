// gol_internal.h -- private state of libgolhip.so (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdint.h>

#include <vector>

#include "golhip.h"

struct gol_comm;
class gol_ipc;

// Library defaults for the bit-board step (chosen from the gfx950 sweep recorded
// in DESIGN.md; overridable per engine through gol_config).
#define GOL_DEFAULT_K 8        // standard layout
#ifndef GOL_DEFAULT_BAND_K
#define GOL_DEFAULT_BAND_K 12  // band layout, 4 words per lane: the split pipeline
#endif
#define GOL_DEFAULT_BYTES_K 32 // byte board: the byte pipeline (0/255 boards with W % 32 == 0)
#define GOL_DEFAULT_DW 2       // standard layout: 64 cells per lane

// A step whose launch runs more rounds of workgroups than this overlaps its edge launches with
// the interior (GOL_STEP_OVERLAP), else it runs as one launch (gol_engine.cpp step_mode).
#define GOL_OVERLAP_ROUNDS 4.0

// Ghost rows kept above and below each bit buffer: the halo (received from the neighbouring
// shards, or the torus wrap of a single shard) lands there, contiguous with the shard's rows,
// so the kernels address input row y as board + y*pitch for -k <= y < R + k.
#define GOL_GHOST_ROWS 16

// Device scratch words for the ranks' collectives, pinned host words per shard.
#define GOL_COLL_WORDS 16
#define GOL_HOST_WORDS 16

// Timing events per shard before the recorded steps are folded into running sums (at the start
// of a timed stepping call; within one call the pool grows instead, gol_engine.cpp timing_event).
#define GOL_TIMING_EVENTS 512

// One row shard: rows [y0, y1) of the board on one GPU.
struct gol_shard {
    int device = 0;
    int64_t y0 = 0, y1 = 0, R = 0;
    hipStream_t stream = nullptr;  // kernels (the interior of a step, loads, queries)
    hipStream_t edge = nullptr;    // the step's launches that read the halo (gol_step_plan)
    hipStream_t comm = nullptr;    // halo exchange
    hipEvent_t ev_start = nullptr; // a step's inputs are complete and its count slots zeroed
    hipEvent_t ev_edge = nullptr;  // the rows the next exchange sends are written
    hipEvent_t ev_halo = nullptr;  // this shard's latest halo exchange is done
    uint32_t *bits[2] = {nullptr, nullptr};        // row 0 of each bit buffer
    uint32_t *bits_alloc[2] = {nullptr, nullptr};  // allocations incl. the ghost rows
    // BYTES mode: the H x W byte board (double buffer).  EXACT mode: bytes[0] = rows
    // y0-1 .. y1 (R + 2 rows, the halo rows from the host board), bytes[1] = R output rows.
    uint8_t *bytes[2] = {nullptr, nullptr};
    uint64_t *slots = nullptr;        // 1 + GOL_SLOT_BATCH arrays of GOL_COUNT_SLOTS * 8 reduction slots
    bool slots_zero = false;          // array 0 zeroed by the last slots reduce (no memset before the next count)
    bool batch_zero = false;          // arrays 1.. zero except those of pending count points (flush_counts)
    uint64_t *counts = nullptr;       // per-count-point alive counts (step_counted)
    int64_t counts_cap = 0;
    uint32_t *flag = nullptr;         // nonbinary flag of a load
    uint32_t *err = nullptr;          // device error word of this shard's launches
    uint32_t *coll = nullptr;         // GOL_COLL_WORDS device words for collectives (agreement, barriers)
    uint32_t *ipc_out = nullptr;      // IPC transport: the rows this rank sends, 2 x 4 x GOL_GHOST_ROWS rows (exchange_ipc)
    uint32_t *host_word = nullptr;    // GOL_HOST_WORDS pinned words: readback of err / flag, collectives
    uint8_t *staging = nullptr;       // device byte rows for chunked copies
    uint8_t *host_staging = nullptr;  // pinned host rows
    int64_t stage_rows = 0;
    ncclComm_t nccl = nullptr;
    // timing (gol_engine_set_timing): events on `stream` around the timed launches
    std::vector<hipEvent_t> tev;
    size_t tused = 0;
};

enum gol_mode {
    GOL_MODE_BITS,   // bit board (W % 64 == 0)
    GOL_MODE_BYTES,  // byte board: W % 64 != 0 or GOL_LAYOUT_BYTES (one shard)
    GOL_MODE_EXACT   // bit-capable board loaded with bytes other than 0/255: turn 1 is exact
};

struct gol_timed {
    int shard;
    size_t ev;  // index of the start event in the shard's pool (stop = ev + 1)
    double cell_updates;
    int64_t steps;  // k-turn steps between the two events
    bool exchange = false;  // events around one halo exchange (GOL_TIMING_EXCHANGE), not a stepping call:
                            // ev, ev + 1 the whole exchange, ev + 2 .. ev + 3 its wait for the neighbours
};

struct gol_engine {
    int64_t H = 0, W = 0;
    int64_t Wd = 0;      // uint32 words per row (W / 32)
    int64_t pitch = 0;   // bit-board row pitch in uint32 words (multiple of 4)
    int64_t bstride = 0; // byte-board row pitch in bytes (multiple of 16)
    std::vector<gol_shard> sh;
    int nranks = 1;      // shards of the whole board
    int rank = 0;        // global rank of sh[0] (local shards are consecutive ranks)
    bool rank_mode = false;  // other ranks live in other processes
    int transport = GOL_TRANSPORT_LOCAL;
    gol_comm *comm = nullptr;  // rank mode: the collectives (RCCL, or the IPC transport's host segment)
    gol_ipc *ipc = nullptr;    // GOL_TRANSPORT_IPC: the neighbours' mapped buffers and flags (== comm)
    std::vector<int> ipc_peers;  // global ranks this rank pulls its halo from (itself excluded)
    uint32_t xn = 0;           // halo exchanges issued (IPC sequence numbers; equal on every rank)
    int64_t min_rows = 0;    // rows of the smallest shard (the broker split: H / nranks)
    bool bit_capable = false;  // W % 64 == 0 and not GOL_LAYOUT_BYTES
    bool band_capable = false; // step the bit board in the band layout
    bool band = false;         // bits[cur] currently hold the band layout
    gol_mode mode = GOL_MODE_BITS;
    bool bytes_binary = false; // BYTES mode: the board holds only 0/255
    int cur = 0, bcur = 0;
    int64_t turn = 0;
    int k = GOL_DEFAULT_K;
    int dw = GOL_DEFAULT_DW;
    int band_dw = 4;
    int strip = 0;
    int kx = 1;                // halo rows of every exchange (>= the k of any step; gol_step_plan)
    int step_flags = 0;        // GOL_STEP_SERIAL
    bool halo_ok = false;      // the ghost rows of bits[cur] hold the current halo (kx rows)
    bool halo_issued = false;  // an exchange was enqueued since the last synchronisation point
    bool halo_on_compute = false;  // the last exchange ran on the compute streams (RCCL after a SERIAL step)
    int64_t pend_first = 0, pend_n = 0;  // count points whose slot arrays await one reduce (flush_counts)
    bool timing = false;
    bool timing_x = false;             // also an event pair around every halo exchange of a timed call
    std::vector<gol_timed> timed;
    std::vector<size_t> tcall_ev;      // the current stepping call's start events (one per shard)
    std::vector<double> tcall_cells;   // and its cell-updates per shard
    int64_t tcall_steps = 0;           // and its k-turn steps
    double t_ms = 0, t_cells = 0;  // folded timing sums (timed pool recycled)
    int64_t t_n = 0;
    double x_ms = 0, x_wait_ms = 0;  // folded exchange timing sums (whole exchange, wait for the neighbours)
    int64_t x_n = 0;
};

int gol_set_error(int code, const char *fmt, ...);
// Enqueue `turns` turns on the shards' streams without synchronising.
int gol_engine_step_async(gol_engine *e, int64_t turns);
