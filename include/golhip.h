/*
 * golhip.h -- C ABI of libgolhip.so, the MI355X (gfx950) Game-of-Life hot path.
 *
 * The reference (ao22174/Gol-distributed-final) is Go; its hot path is reached
 * over net/rpc.  This ABI is what a cgo binding of that path would bind (the
 * stub is in INTEGRATION.md).  Every entry point names the reference
 * interface it replaces (file:line inside the reference tree).
 *
 * Conventions
 *  - Every call returns an int status: GOL_OK (0) or a negative GOL_E* code.
 *    It never aborts the process.  gol_last_error() gives a thread-local
 *    message for the last failing call on the calling thread.  (The
 *    reference panics on local failures, util/check.go:3-7, and its RPC
 *    handlers always return nil; a Go host maps nonzero codes to `error`.)
 *  - Host buffers are caller-owned and only borrowed for the duration of a
 *    call; the library never retains a host pointer.  Device memory created
 *    by an engine is engine-owned and released by gol_engine_destroy.
 *  - Boards: byte boards are row-major [y][x], one byte per cell, 255 = alive,
 *    0 = dead (README.md:25-32); `stride` is the row pitch in bytes.
 *    Bit boards are row-major, 64 cells per uint64 (LSB = lowest x), i.e. 32
 *    cells per uint32 little-endian; `pitch` is the row pitch in uint32 words.
 *  - Torus semantics: rows wrap with H, columns with W.  The reference wraps
 *    both axes with len(world[0]) (worker.go:48-59) and is only defined for
 *    square boards, where the two agree.
 *  - Thread safety: gol_next_state_slab and the gol_dev_* launchers are
 *    re-entrant.  A gol_engine handle is not internally synchronised; callers
 *    serialise access (the broker mirror does, like broker.go's `mt`).
 */
#ifndef GOLHIP_H
#define GOLHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GOL_ABI_VERSION 6

enum {
    GOL_OK = 0,
    GOL_EINVAL = -1,   /* bad argument */
    GOL_EHIP = -2,     /* HIP runtime error, or a kernel reported a device-side fault */
    GOL_ENOMEM = -3,   /* allocation failed */
    GOL_EIO = -4,      /* file I/O */
    GOL_EFORMAT = -5,  /* malformed PGM (io.go:101-117 panics) */
    GOL_ESTATE = -6,   /* call not valid in the current state */
    GOL_EQUIT = -7,    /* broker was shut down (SuperQuit) */
    GOL_ECOMM = -8     /* RCCL (halo exchange / reduction) error */
};

/* ---------------------------------------------------------------- library */
int gol_abi_version(void);
const char *gol_last_error(void);
int gol_device_count(int *n);

/* ---------------------------------------------------------------- worker path
 * Replaces worker.go:15-42 calculateNextState + worker.go:44-70
 * calculateSurroundings, as called by GameOfLifeOperations.Update
 * (worker.go:77-80).  Exact reference semantics per byte: a cell that is
 * exactly 0 with exactly 3 neighbours equal to 255 becomes 255; a cell equal to
 * 255 with 2 or 3 such neighbours stays 255; every other cell becomes 0.
 * world: H x W bytes (row pitch `stride`); out: (y1-y0) x W bytes (pitch
 * out_stride) = next state of rows [y0, y1).  Runs on the current device. */
int gol_next_state_slab(const uint8_t *world, int64_t H, int64_t W, int64_t stride,
                        int64_t y0, int64_t y1, uint8_t *out, int64_t out_stride);

/* Replaces the row split of broker.go:135-139 (H % T == 0: StartY = i*H/T,
 * EndY = (i+1)*H/T) and broker.go:172-206 (else the first H % T slabs get
 * H/T + 1 rows, the rest H/T, in order).  Also used to row-shard a board over
 * GPUs. */
int gol_partition_rows(int64_t H, int64_t parts, int64_t i, int64_t *y0, int64_t *y1);

/* ---------------------------------------------------------------- engine
 * A board resident in HBM, on one GPU or row-sharded over several.  Replaces
 * the broker's per-turn state (`world`, `cWorld`, `cTurn`: broker.go:22-36,
 * 62-234) and the per-turn scatter/gather to workers (broker.go:143-157,
 * 182-211): the board stays in HBM and is stepped in k-turn launches.
 *
 * Row sharding (broker.go:135-206 applied to GPUs): the board's rows are split
 * with gol_partition_rows over `nranks` shards; shard r keeps rows
 * [y0_r, y1_r) plus 16 ghost rows above and below.  Every k-turn step needs in
 * its ghost rows the k rows above the shard (from shard r-1) and below it
 * (from shard r+1, mod nranks): gol_halo_plan.  A step first computes the kx
 * rows at each edge of the shard (they read the halo) and, beside them, the
 * interior; the next step's halo is exchanged as soon as the edge rows are
 * written, while the interior is still running (gol_step_plan).  One shard
 * (the whole torus) runs the same step with its own rows as the halo.
 * k <= kx <= min shard rows.
 *  - one process, `shards` local shards (gol_config.shards): GPUs device,
 *    device+1, ... (or all on `device` with GOL_SHARDS_SAME_DEVICE);
 *  - one process per GPU (gol_engine_create_rank): this process holds shard
 *    `rank` of `nranks`; whole-board queries (alive count, hash, PGM write,
 *    counted steps) are collective: every rank calls them.
 * Transports of the halo rows: RCCL ncclSend/ncclRecv on a per-shard comm
 * stream (xGMI between GPUs), LOOPBACK device copies between the shards of
 * one process (shards may share a GPU: multi-shard logic on a 1-GPU box), or
 * IPC between the rank processes of one node: each rank copies its ghost rows
 * out of its neighbours' HBM through HIP IPC mappings, ordered by sequence
 * flags in device memory, and the collectives (counts, error words, barriers)
 * run on the host through a shared-memory segment.  IPC ranks may share a GPU
 * (RCCL refuses two ranks on one GPU), so the one-process-per-GPU engine runs
 * with 2-16 processes on a 1-GPU box exactly as it runs on 8 GPUs. */
typedef struct gol_engine gol_engine;

/* Bit-board layout used while stepping.  STANDARD: word s of a row holds cells
 * 32s .. 32s+31.  BAND: word w holds, at bit b, cell b*(W/32) + w (32 column
 * bands), which makes a generation shift-free.  AUTO picks
 * BAND when W % 1024 == 0.  The layout is internal: every reader (store,
 * alive list, PGM, hash, device_bits) sees the standard layout.  BYTES keeps
 * the board as the reference's one byte per cell (a W % 64 != 0 board always
 * does): one shard, 32 turns per launch on a 0/255 board with W % 32 == 0 (the
 * byte pipeline), the exact byte kernel otherwise; the
 * bit-board calls (load_words, store_words, device_bits, hash) are EINVAL. */
#define GOL_LAYOUT_AUTO 0
#define GOL_LAYOUT_STANDARD 1
#define GOL_LAYOUT_BAND 2
#define GOL_LAYOUT_BYTES 3
/* Halo transport between shards. */
#define GOL_TRANSPORT_AUTO 0     /* 1 shard: local torus wrap; shards on distinct GPUs: RCCL; else LOOPBACK */
#define GOL_TRANSPORT_LOOPBACK 1 /* device copies between the shards of this process */
#define GOL_TRANSPORT_RCCL 2     /* ncclSend/ncclRecv (with one shard: send to self) */
#define GOL_TRANSPORT_LOCAL 3    /* (reported only) one shard, wrap rows read from the board itself */
#define GOL_TRANSPORT_IPC 4      /* gol_engine_create_rank only: HIP IPC halo pulls + host collectives */
/* gol_config.flags */
#define GOL_SHARDS_SAME_DEVICE 1 /* every local shard on `device` (loopback testing on one GPU) */
#define GOL_STEP_SERIAL 2        /* one launch per shard and step, after the halo exchange (gol_step_plan) */
#define GOL_STEP_EDGE_FIRST 4    /* the edge rows first on the compute stream, then the interior (gol_step_plan) */
#define GOL_STEP_OVERLAP 8       /* the edge rows on the edge stream beside the interior (gol_step_plan) */
                                 /* (16: ABI 3's persistent multi-round launch, removed in ABI 4) */
typedef struct gol_config {
    int32_t device;           /* HIP device ordinal (first shard); -1 = current device */
    int32_t turns_per_launch; /* k (temporal blocking); 0 = library default */
    int32_t strip_rows;       /* rows per wave strip; 0 = automatic */
    int32_t cells_per_lane;   /* 32, 64 or 128 bits per lane; 0 = automatic */
    int32_t layout;           /* bit-board layout while stepping: GOL_LAYOUT_* */
    int32_t shards;           /* row shards in this process (0 or 1 = one GPU, no sharding) */
    int32_t transport;        /* GOL_TRANSPORT_* */
    int32_t flags;            /* GOL_SHARDS_* */
} gol_config;

int gol_engine_create(int64_t H, int64_t W, const gol_config *cfg, gol_engine **out);
/* One process per GPU: every rank calls this (collective) with the same H, W,
 * nranks and unique id, made on one rank and shared by the caller's own means
 * (e.g. torch.distributed or the Go broker's RPC): gol_rccl_unique_id for
 * cfg->transport GOL_TRANSPORT_RCCL (the default with nranks > 1),
 * gol_ipc_unique_id for GOL_TRANSPORT_IPC (at most GOL_IPC_MAX_RANKS ranks, one
 * node; the id names the ranks' shared-memory segment, which exists only while
 * they connect).  cfg->device is this rank's GPU (IPC ranks may name the same
 * one).  Needs W % 64 == 0 and H >= nranks.  With several ranks every stepping
 * call starts by agreeing on the halo state: a rank whose rows changed outside
 * a step (load_words on it alone) makes every rank exchange its halo again. */
#define GOL_RCCL_ID_BYTES 128
#define GOL_IPC_ID_BYTES 128
#define GOL_IPC_MAX_RANKS 16
int gol_rccl_unique_id(uint8_t *id, int64_t len);
int gol_ipc_unique_id(uint8_t *id, int64_t len);
int gol_engine_create_rank(int64_t H, int64_t W, int32_t nranks, int32_t rank, const uint8_t *id,
                           const gol_config *cfg, gol_engine **out);
void gol_engine_destroy(gol_engine *e);
/* Layout of the engine: local shards, global ranks, the first local shard's
 * global rank, and the halo transport in use (GOL_TRANSPORT_LOOPBACK, _RCCL or
 * _LOCAL). */
int gol_engine_topology(gol_engine *e, int32_t *shards, int32_t *nranks, int32_t *rank, int32_t *transport);
/* Local shard i: its GPU and its global rows [y0, y1). */
int gol_engine_shard(gol_engine *e, int32_t i, int32_t *device, int64_t *y0, int64_t *y1);
/* Load a byte board (operations.Run's req.World, broker.go:65) and reset the
 * turn counter to 0.  Any byte value is accepted (exact semantics above).
 * `world` is the whole H x W board (as the reference ships it to every
 * worker); every rank reads its own rows. */
int gol_engine_load_bytes(gol_engine *e, const uint8_t *world, int64_t stride);
/* Load images/<W>x<H>.pgm-style P5 (readPgmImage, gol/io.go:90-126: fields
 * "P5", W, H, 255, then the raster): every shard streams its own rows from
 * the file.  GOL_EFORMAT with the reference's panic text on a bad header, a
 * short raster or (the reference's strings.Fields split) whitespace bytes in
 * it. */
int gol_engine_load_pgm(gol_engine *e, const char *path);
/* Synthetic board: word(y, w) = splitmix64(seed ^ (y*W/64 + w)), Bernoulli(1/2)
 * per cell (W % 64 == 0 only; on a GOL_LAYOUT_BYTES board as 0/255 bytes).
 * Resets the turn counter. */
int gol_engine_load_random(gol_engine *e, uint64_t seed);
/* Advance exactly `turns` turns (blocking).  Replaces the turn loop body of
 * broker.go:75-226. */
int gol_engine_step(gol_engine *e, int64_t turns);
/* Advance exactly `turns` turns and record the alive count every `every`
 * turns (the AliveCellsCount events of distributor.go:39-51, computed on the
 * GPU: fused into the launch that ends at each such turn, then reduced on the
 * device and, between ranks, with one RCCL all-reduce at the end).  counts[i]
 * = alive cells after turn (start + (i+1)*every); writes turns/every counts
 * (cap >= turns/every).  One host synchronisation for the whole call. */
int gol_engine_step_counted(gol_engine *e, int64_t turns, int64_t every, uint64_t *counts, int64_t cap);
int gol_engine_turn(gol_engine *e, int64_t *turn);
/* Number of cells != 0 -- len(calculateAliveCells(...)), broker.go:273. */
int gol_engine_alive_count(gol_engine *e, uint64_t *count);
/* Copy the board out as bytes (0/255, or the loaded bytes before turn 1).
 * Needs every row local (not with nranks > 1 ranks: use store_rows). */
int gol_engine_store_bytes(gol_engine *e, uint8_t *out, int64_t stride);
/* Rows [y0, y1) of the board (global row numbers, all held by this process). */
int gol_engine_store_rows(gol_engine *e, int64_t y0, int64_t y1, uint8_t *out, int64_t stride);
/* calculateAliveCells (broker.go:47-58): (x, y) int32 pairs in row-major
 * order; writes min(n, cap) pairs, *n = total alive cells.  With ranks in
 * several processes: the cells of this rank's rows. */
int gol_engine_alive_cells(gol_engine *e, int32_t *xy, int64_t cap, int64_t *n);
/* Advance exactly one turn and list the cells whose state changed, (x, y) int32
 * pairs in row-major order: the CellFlipped{CompletedTurns, Cell} events of
 * that turn (gol/event.go:50-60; sent per flipped cell by the controller the
 * reference never finished, README.md:260-262).  Writes min(n, cap) pairs,
 * *n = number of flipped cells (of this rank's rows with several processes). */
int gol_engine_step_flips(gol_engine *e, int32_t *xy, int64_t cap, int64_t *n);
/* writePgmImage byte stream (gol/io.go:52-81): "P5\n<W> <H>\n255\n" + H*W
 * bytes, streamed from the device in chunks; with several processes every
 * rank writes its own rows at their offset (collective). */
int gol_engine_write_pgm(gol_engine *e, const char *path);
/* The same byte stream handed to a caller's sink instead of a file (a pipe,
 * a socket, a hash, a compressor: config 5's 2^20 x 2^20 board is 1 TiB as
 * P5).  The sink gets (user, file offset, bytes, length) for the header and
 * then every chunk of rows (at most 64 MiB each) of the shards of this process
 * in row order, and returns 0 (nonzero aborts the write with GOL_EIO).  With
 * ranks in several processes every rank calls it (collective) and its sink
 * sees its own rows at their offsets; rank 0's also gets the header. */
typedef int (*gol_write_fn)(void *user, int64_t offset, const uint8_t *data, int64_t len);
int gol_engine_write_pgm_to(gol_engine *e, gol_write_fn sink, void *user);
/* Bit-packed rows [y0, y1) (global, held by this process) in or out: 64 cells
 * per uint64 (LSB = lowest x), `stride` uint64 words per row, W % 64 == 0.
 * load_words overwrites those rows of the current board (several calls may
 * load a board piece by piece), resets the turn counter to 0.  store_words
 * reads them (GOL_ESTATE before turn 1 of a board loaded with bytes other than
 * 0/255: use store_bytes).  One eighth of the PCIe traffic of the byte calls. */
int gol_engine_load_words(gol_engine *e, int64_t y0, int64_t y1, const uint64_t *words, int64_t stride);
int gol_engine_store_words(gol_engine *e, int64_t y0, int64_t y1, uint64_t *words, int64_t stride);
/* Order-independent board hash (same definition as oracle_hash_words):
 * sum over 64-bit words of splitmix64(word ^ splitmix64(y*W/64 + w)).
 * W % 64 == 0 only. */
int gol_engine_hash(gol_engine *e, uint64_t *hash);
/* Chosen kernel parameters (k, cells per lane, strip rows, resident mode: 0 =
 * byte board, 1 = standard bit board, 2 = band bit board). */
int gol_engine_info(gol_engine *e, int32_t *k, int32_t *cells_per_lane, int32_t *strip_rows,
                    int32_t *bit_mode);
/* Raw device pointer to the current bit board of local shard 0 (pitch in
 * uint32 words), for tests. */
int gol_engine_device_bits(gol_engine *e, uint32_t **bits, int64_t *pitch);
/* Step timing: with timing on, HIP events on each shard's compute stream
 * bracket every k-turn step of the shard: from before its first launch to the
 * end of its last one, the edge launches included (gol_step_plan).
 * gol_engine_timing returns the number of timed shard-steps since timing was
 * (re)enabled, their mean duration and their mean cell-updates (R x W x k). */
int gol_engine_set_timing(gol_engine *e, int32_t enable);
int gol_engine_timing(gol_engine *e, int64_t *launches, double *mean_ms, double *mean_cell_updates);
/* enable = GOL_TIMING_EXCHANGE (ABI 5): also one event pair around every halo
 * exchange of a timed stepping call, on the stream the exchange runs on (the
 * RCCL send/recv group, or the IPC transport's copies and flag waits, from the
 * moment its sent rows are written); gol_engine_exchange_timing returns how many
 * were timed since timing was (re)enabled and their mean duration.  Local (this
 * process's shards); an engine whose one shard is the whole torus exchanges
 * nothing (0). */
#define GOL_TIMING_EXCHANGE 2
int gol_engine_exchange_timing(gol_engine *e, int64_t *exchanges, double *mean_ms);
/* ABI 6: the same exchanges split in two.  mean_wait_ms is the part spent
 * waiting for the ring neighbours to reach the exchange: the IPC transport's
 * poll of their READY flags; on RCCL a one-word send/recv with each neighbour
 * issued first (only while exchanges are timed), whose completion means every
 * neighbour has posted its side.  mean_transfer_ms is the rest (the halo rows
 * themselves once both sides are there).  Transports without peers in other
 * processes (LOCAL, LOOPBACK) wait for nothing on the exchange's stream: 0. */
int gol_engine_exchange_split(gol_engine *e, int64_t *exchanges, double *mean_wait_ms, double *mean_transfer_ms);

/* ---------------------------------------------------------------- plans
 * The schedule of a sharded step as data (host functions, no GPU needed).  The
 * engine runs exactly these plans; golhip.sharded (the torch.distributed
 * mirror) and the tests read them.  Replaces the broker's per-turn fan-out
 * (broker.go:135-206: every worker gets the whole board) by a k-row halo with
 * the ring neighbours.
 *
 * gol_halo_plan: the halo exchange of global rank `rank` of an H-row board
 * split over nranks shards (gol_partition_rows), k rows each way, in issue
 * order.  Sends read shard-local rows [row, row + rows) of the shard, receives
 * write its ghost rows [row, row + rows) (row = -k or R).  A receiver matches
 * the sends addressed to it by one sender with its receives from that sender
 * in issue order (ncclSend/ncclRecv semantics; for nranks = 2 both neighbours
 * are one peer, for nranks = 1 the shard sends to itself: the torus wrap).
 * Writes min(4, cap) ops; *n = 4. */
#define GOL_HALO_SEND 0
#define GOL_HALO_RECV 1
typedef struct gol_halo_op {
    int32_t kind;  /* GOL_HALO_SEND / GOL_HALO_RECV */
    int32_t peer;  /* global rank of the other side */
    int64_t row;   /* first shard-local row of the block */
    int64_t rows;  /* k */
} gol_halo_op;
int gol_halo_plan(int64_t H, int32_t nranks, int32_t rank, int32_t k, gol_halo_op *ops, int32_t cap, int32_t *n);
/* gol_step_plan: the launches of one k-turn step of a shard of R rows whose
 * halo exchanges carry kx >= k rows, in launch order.  EDGE launches run on
 * the shard's edge stream, MAIN launches on its compute stream; a launch that
 * needs_halo waits for the exchange.  The next step's exchange starts when the
 * last launch that needs the halo (they write rows [0, kx) and [R - kx, R),
 * the rows it sends) is done.  With R >= 3 kx:
 *  - GOL_STEP_OVERLAP: rows [0, kx) and [R - kx, R) on the edge stream, the
 *    interior [kx, R - kx) (it reads no ghost row) on the compute stream
 *    beside them: nothing waits for the exchange but the edge launches;
 *  - GOL_STEP_EDGE_FIRST: the same three launches in order on the compute
 *    stream (the exchange overlaps the interior; no second kernel competes
 *    with the interior for the CUs);
 *  - neither (or GOL_STEP_SERIAL, or R < 3 kx): one MAIN launch over [0, R).
 * The engine picks per step: OVERLAP for launches of many
 * rounds of workgroups, SERIAL below, unless gol_config.flags forces one.
 * Writes min(n, cap) launches. */
#define GOL_LAUNCH_MAIN 0
#define GOL_LAUNCH_EDGE 1
typedef struct gol_launch {
    int32_t stream;     /* GOL_LAUNCH_MAIN / GOL_LAUNCH_EDGE */
    int32_t needs_halo; /* reads the ghost rows: waits for the exchange */
    int64_t row0;       /* first shard-local output row */
    int64_t rows;
} gol_launch;
int gol_step_plan(int64_t R, int32_t k, int32_t kx, int32_t flags, gol_launch *out, int32_t cap, int32_t *n);

/* ---------------------------------------------------------------- device launchers
 * Asynchronous kernel launches on caller-owned device memory and a caller
 * stream (hipStream_t passed as void*; NULL = default stream).  These are the
 * building blocks of the row-sharded multi-GPU board (one process per GPU;
 * broker.go:135-206's partition applied to GPUs) and of bench.py.
 *
 * Bit board of one shard: R local rows, Wd = W/32 uint32 words per row, row
 * pitch `pitch` words.  Input row y of the shard (-k <= y < R + k) is read
 * from: top + (y + k)*pitch for y < 0, mid + y*pitch for 0 <= y < R,
 * bot + (y - R)*pitch for y >= R.  (One GPU: top = mid + (R-k)*pitch,
 * bot = mid, the torus wrap; several GPUs: the k-row halo buffers received
 * from the neighbouring ranks.)  Writes rows [row0, row0 + rows) of dst
 * after k turns.  If count_slots is non-NULL the alive cells of the written
 * rows are added to count_slots[0 .. GOL_COUNT_SLOTS*8) (sum them all). */
#define GOL_COUNT_SLOTS 256
int gol_dev_bits_step(const uint32_t *top, const uint32_t *mid, const uint32_t *bot, uint32_t *dst,
                      int64_t R, int64_t Wd, int64_t pitch, int64_t row0, int64_t rows, int32_t k,
                      int32_t cells_per_lane, int32_t strip_rows, uint64_t *count_slots,
                      void *stream);
/* Fill rows [0, rows) of a bit board with the synthetic board rows
 * [grow0, grow0 + rows) of a W-wide torus (W % 64 == 0). */
int gol_dev_random_fill(uint32_t *dst, int64_t rows, int64_t grow0, int64_t W, int64_t pitch,
                        uint64_t seed, void *stream);
/* Add popcount(rows x Wd words) to slots (GOL_COUNT_SLOTS*8 uint64). */
int gol_dev_popcount(const uint32_t *src, int64_t rows, int64_t Wd, int64_t pitch,
                     uint64_t *slots, void *stream);
/* Add the board-hash contribution of rows whose first global row is grow0. */
int gol_dev_hash(const uint32_t *src, int64_t rows, int64_t grow0, int64_t Wd, int64_t pitch,
                 uint64_t *slots, void *stream);
/* Bytes <-> bits for rows x W cells; pack also ORs 1 into *nonbinary when a
 * byte other than 0/255 is seen (may be NULL). */
int gol_dev_pack(const uint8_t *bytes, int64_t rows, int64_t W, int64_t stride, uint32_t *bits,
                 int64_t pitch, uint32_t *nonbinary, void *stream);
int gol_dev_unpack(const uint32_t *bits, int64_t rows, int64_t W, int64_t pitch, uint8_t *bytes,
                   int64_t stride, void *stream);
/* One exact-semantics byte turn (worker.go:15-70) for rows [y0, y1) of an
 * H x W byte torus; out row i = next state of row y0 + i. */
int gol_dev_bytes_step(const uint8_t *world, int64_t H, int64_t W, int64_t stride, int64_t y0,
                       int64_t y1, uint8_t *out, int64_t out_stride, void *stream);

/* k turns (1, 2, 4, 8, 16 or 32; 32 runs as 8 waves x 4 turns of one workgroup, the
 * byte pipeline) of a byte board whose bytes are all 0 or 255 (every
 * board after its first turn), W % 32 == 0, stride % 16 == 0, 16-byte aligned
 * rows; row addressing as gol_dev_bits_step (top/mid/bot are byte rows, pitch
 * `stride`).  Same results as k exact turns on such boards; 2 bytes of HBM
 * traffic per cell per k turns.  count_slots as in gol_dev_bits_step. */
int gol_dev_bytes_step_k(const uint8_t *top, const uint8_t *mid, const uint8_t *bot, uint8_t *dst, int64_t R,
                         int64_t W, int64_t stride, int64_t row0, int64_t rows, int32_t k, int32_t strip_rows,
                         uint64_t *count_slots, void *stream);

/* k turns of a BAND-layout bit board (bit b of word w = cell b*Wd + w); row
 * addressing and count_slots as gol_dev_bits_step.  cells_per_lane: 64 or 128
 * (2 or 4 words per lane; 0 = library default); k in {1, 2, 4, 8}, 16 with 64
 * cells per lane, 12 with 128 (the split pipeline: 4 waves x 3 turns); Wd and
 * pitch multiples of the words per lane, rows aligned to 4 bytes x words per
 * lane.  Same cells as gol_dev_bits_step on the standard layout, with no bit
 * shifts in the generation.  The pipelined kernels (k = 12 here, k = 32 in
 * gol_dev_bytes_step_k) report a device-side protocol fault in the device's
 * error word: check it with gol_dev_error after synchronising the stream. */
int gol_dev_band_step(const uint32_t *top, const uint32_t *mid, const uint32_t *bot, uint32_t *dst,
                      int64_t R, int64_t Wd, int64_t pitch, int64_t row0, int64_t rows, int32_t k,
                      int32_t cells_per_lane, int32_t strip_rows, uint64_t *count_slots, void *stream);
/* Largest k gol_dev_band_step accepts for this cells_per_lane (0 = default);
 * 0 if cells_per_lane is not supported. */
int gol_band_max_k(int32_t cells_per_lane);
/* Convert rows x Wd words between the standard and the band layout (to_band
 * != 0: standard -> band), out of place; Wd % 32 == 0 (W % 1024 == 0). */
int gol_dev_band_convert(int32_t to_band, const uint32_t *src, uint32_t *dst, int64_t rows, int64_t Wd,
                         int64_t src_pitch, int64_t dst_pitch, void *stream);
/* Read and clear the error word of `device` (-1 = current) that the gol_dev_*
 * launchers' kernels report into (*flags = 0: no fault; nonzero: a pipeline
 * wave timed out waiting for its neighbour, so the launch's output is not
 * valid).  Synchronous; returns GOL_EHIP when *flags != 0. */
int gol_dev_error(int32_t device, uint32_t *flags);
/* ---------------------------------------------------------------- RPC service mirror
 * The broker's net/rpc service `Operations` (broker.go:62-277) and the
 * worker's `GameOfLifeOperations` (worker.go:77-86) with the gob field names
 * of stubs.go:13-38.  A Go drop-in registers these names and forwards here. */
typedef struct gol_request {     /* stubs.Request, stubs.go:20-29 */
    const uint8_t *World;        /* ImageHeight x ImageWidth bytes, row pitch world_stride */
    int64_t world_stride;
    int64_t Turns;
    int64_t ImageHeight;
    int64_t ImageWidth;
    int64_t Threads;
    int64_t EndY;
    int64_t StartY;
    int64_t Worker;
} gol_request;

typedef struct gol_response {    /* stubs.Response, stubs.go:31-38 */
    int32_t *Alive;              /* caller buffer for (X, Y) pairs (util.Cell, util/cell.go:4-5) */
    int64_t alive_cap;           /* capacity in pairs */
    int64_t alive_len;           /* out: len(Alive) (may exceed alive_cap: then truncated) */
    int64_t AliveCount;          /* out */
    int64_t TurnsCompleted;      /* out */
    uint8_t *World;              /* caller buffer, ImageHeight x ImageWidth, pitch world_stride */
    int64_t world_stride;
    uint8_t *WorkSlice;          /* caller buffer, (EndY-StartY) x width, pitch work_stride */
    int64_t work_stride;
    int64_t Worker;
} gol_response;

typedef struct gol_broker gol_broker;
int gol_broker_create(const gol_config *cfg, gol_broker **out);
void gol_broker_destroy(gol_broker *b);
int gol_broker_run(gol_broker *b, const gol_request *req, gol_response *res);      /* Operations.Run, broker.go:62-234 */
int gol_broker_retrieve(gol_broker *b, const gol_request *req, gol_response *res); /* Operations.RetrieveCurrentData, broker.go:256-277 */
int gol_broker_pause(gol_broker *b);                                              /* Operations.Pause, broker.go:251-254 */
int gol_broker_quit(gol_broker *b);                                               /* Operations.Quit, broker.go:236-239 */
int gol_broker_superquit(gol_broker *b);                                          /* Operations.SuperQuit, broker.go:241-249 */
int gol_broker_paused(gol_broker *b, int32_t *paused);
int gol_worker_update(const gol_request *req, gol_response *res);                 /* GameOfLifeOperations.Update, worker.go:77-80 */

#ifdef __cplusplus
}
#endif
#endif /* GOLHIP_H */
