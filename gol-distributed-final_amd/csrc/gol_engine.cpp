// gol_engine.cpp -- the board engine of libgolhip.so: a Game-of-Life torus resident in HBM,
// on one GPU or row-sharded over several (include/golhip.h, "engine").
//
// The reference keeps the board in the broker and ships ALL of it to every worker every turn
// (broker.go:143-157, 182-211), then gathers the slabs and copies them into cWorld
// (broker.go:153-169).  Here the broker's row partition (broker.go:135-206) is applied once,
// to GPUs: shard r keeps rows [y0_r, y1_r) bit-packed in its own HBM for the whole run, and the
// only traffic between shards is a k-row halo every k turns (RCCL send/recv over xGMI, or
// device copies between the shards of one process).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <climits>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "golhip.h"
#include "gol_comm.h"
#include "gol_internal.h"
#include "gol_kernels.h"

#define HIPCHK(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return gol_set_error(e_ == hipErrorOutOfMemory ? GOL_ENOMEM : GOL_EHIP, "%s failed: %s (%s:%d)", #expr, \
                                 hipGetErrorString(e_), __FILE__, __LINE__);                      \
    } while (0)

#define NCCLCHK(expr)                                                                             \
    do {                                                                                          \
        ncclResult_t r_ = (expr);                                                                 \
        if (r_ != ncclSuccess)                                                                    \
            return gol_set_error(GOL_ECOMM, "%s failed: %s", #expr, ncclGetErrorString(r_));      \
    } while (0)

#define RCCHK(expr)                  \
    do {                             \
        int rc_ = (expr);            \
        if (rc_ != GOL_OK) return rc_; \
    } while (0)

static constexpr size_t SLOT_BYTES = GOL_COUNT_SLOTS * 8 * sizeof(uint64_t);
// The count points of a stepping call: the launch that ends point ci adds its cells into slot
// array 1 + ci % GOL_SLOT_BATCH, and one reduce kernel sums a run of such arrays into counts[]
// (flush_counts); array 0 serves single counts (count_into_slots, hash).  Against a reduce per
// point: 65536^2 139.5 -> 140.3 TCUPS, the big boards +0.3 % (same box, 3 reps, same counts;
// profiles/r04/r04l_count_batch.jsonl).
#define GOL_SLOT_BATCH 64
static constexpr size_t SLOT_WORDS = GOL_COUNT_SLOTS * 8;
// The IPC transport's send buffer (exchange_ipc): 2 exchange parities x 4 plan ops x the ghost rows.
static size_t ipc_out_bytes(const gol_engine *e) { return (size_t)2 * 4 * GOL_GHOST_ROWS * e->pitch * sizeof(uint32_t); }

static int set_dev(int d)
{
    HIPCHK(hipSetDevice(d));
    return GOL_OK;
}

// Turns per launch: the largest supported k <= want, the remaining turns and the smallest
// shard.  k = 12 is the band layout's (the split pipeline at 4 words per lane, one wave for
// all 12 turns at 2); k = 16 needs <= 2 words per lane.
static int pick_k(int want, int64_t remaining, int64_t rows, int dw, bool band)
{
    static const int ks[] = {16, 12, 8, 4, 2, 1};
    for (int k : ks) {
        if (k == 16 && dw > 2) continue;
        if (k == 12 && !band) continue;  // band: the split pipeline (4 words per lane) or one wave (2)
        if (k <= want && k <= remaining && k <= rows) return k;
    }
    return 1;
}

// ------------------------------------------------------------------ allocation
static int ensure_staging(gol_engine *e, gol_shard &s)
{
    if (!s.staging) {
        // byte staging for chunked load/store/PGM: >= 1 row, <= 64 MiB
        const int64_t rows = std::max<int64_t>(s.R, 1);
        s.stage_rows = std::max<int64_t>(1, std::min<int64_t>(rows, (64LL << 20) / e->bstride));
        HIPCHK(hipMalloc(&s.staging, s.stage_rows * e->bstride));
        HIPCHK(hipHostMalloc((void **)&s.host_staging, s.stage_rows * e->bstride, hipHostMallocDefault));
    }
    return GOL_OK;
}

static int ensure_counts(gol_shard &s, int64_t n)
{
    if (s.counts_cap >= n) return GOL_OK;
    if (s.counts) (void)hipFree(s.counts);
    s.counts = nullptr;
    s.counts_cap = 0;
    const int64_t cap = std::max<int64_t>(n, 64);
    HIPCHK(hipMalloc(&s.counts, cap * sizeof(uint64_t)));
    s.counts_cap = cap;
    return GOL_OK;
}

static void free_exact_bytes(gol_shard &s)
{
    for (auto &b : s.bytes)
        if (b) { (void)hipFree(b); b = nullptr; }
}

static void shard_release(gol_shard &s)
{
    (void)hipSetDevice(s.device);
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.edge) (void)hipStreamSynchronize(s.edge);
    if (s.comm) (void)hipStreamSynchronize(s.comm);
    if (s.nccl) (void)ncclCommDestroy(s.nccl);
    if (s.stream) golk_release_claims(s.stream);
    if (s.edge) golk_release_claims(s.edge);
    for (auto &b : s.bits_alloc)
        if (b) (void)hipFree(b);
    free_exact_bytes(s);
    if (s.slots) (void)hipFree(s.slots);
    if (s.counts) (void)hipFree(s.counts);
    if (s.flag) (void)hipFree(s.flag);
    if (s.err) (void)hipFree(s.err);
    if (s.coll) (void)hipFree(s.coll);
    if (s.ipc_out) (void)hipFree(s.ipc_out);
    if (s.host_word) (void)hipHostFree(s.host_word);
    if (s.staging) (void)hipFree(s.staging);
    if (s.host_staging) (void)hipHostFree(s.host_staging);
    for (auto ev : s.tev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : {s.ev_start, s.ev_edge, s.ev_halo})
        if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t st : {s.stream, s.edge, s.comm})
        if (st) (void)hipStreamDestroy(st);
    s = gol_shard();
}

static int shard_alloc(gol_engine *e, gol_shard &s)
{
    RCCHK(set_dev(s.device));
    for (hipStream_t *st : {&s.stream, &s.edge, &s.comm}) HIPCHK(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
    golk_own_stream(s.stream);
    golk_own_stream(s.edge);
    for (hipEvent_t *ev : {&s.ev_start, &s.ev_edge, &s.ev_halo}) HIPCHK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    HIPCHK(hipMalloc(&s.slots, SLOT_BYTES * (1 + GOL_SLOT_BATCH)));
    HIPCHK(hipMalloc(&s.flag, sizeof(uint32_t)));
    HIPCHK(hipMalloc(&s.err, sizeof(uint32_t)));
    HIPCHK(hipMalloc(&s.coll, GOL_COLL_WORDS * sizeof(uint32_t)));
    HIPCHK(hipHostMalloc((void **)&s.host_word, GOL_HOST_WORDS * sizeof(uint32_t), hipHostMallocDefault));
    // on the shard's stream: it is non-blocking, so a null-stream memset could still be running
    // when the first load or fill kernel writes the board
    HIPCHK(hipMemsetAsync(s.err, 0, sizeof(uint32_t), s.stream));
    if (e->bit_capable) {
        const int64_t rows = s.R + 2 * GOL_GHOST_ROWS;
        for (int i = 0; i < 2; ++i) {
            HIPCHK(hipMalloc(&s.bits_alloc[i], rows * e->pitch * sizeof(uint32_t)));
            HIPCHK(hipMemsetAsync(s.bits_alloc[i], 0, rows * e->pitch * sizeof(uint32_t), s.stream));
            s.bits[i] = s.bits_alloc[i] + GOL_GHOST_ROWS * e->pitch;
        }
    } else {
        for (auto &b : s.bytes) HIPCHK(hipMalloc(&b, e->H * e->bstride));
        HIPCHK(hipMemsetAsync(s.bytes[0], 0, e->H * e->bstride, s.stream));
        e->bytes_binary = true;  // an all-dead board: 0/255 only
    }
    HIPCHK(hipStreamSynchronize(s.stream));
    return GOL_OK;
}

// Board geometry and kernel parameters from the configuration (shared by both constructors).
static int engine_setup(gol_engine *e, int64_t H, int64_t W, const gol_config *cfg)
{
    if (H <= 0 || W <= 0 || W > (int64_t)INT32_MAX * 32 || H > INT32_MAX)
        return gol_set_error(GOL_EINVAL, "bad board size %lldx%lld", (long long)W, (long long)H);
    e->H = H;
    e->W = W;
    const int layout = cfg ? cfg->layout : GOL_LAYOUT_AUTO;
    if (layout < GOL_LAYOUT_AUTO || layout > GOL_LAYOUT_BYTES)
        return gol_set_error(GOL_EINVAL, "layout must be GOL_LAYOUT_AUTO, _STANDARD, _BAND or _BYTES");
    e->bit_capable = (W % 64) == 0 && layout != GOL_LAYOUT_BYTES;
    e->mode = e->bit_capable ? GOL_MODE_BITS : GOL_MODE_BYTES;
    e->Wd = W / 32;
    e->pitch = (e->Wd + 3) / 4 * 4;
    e->bstride = (W + 15) / 16 * 16;
    e->k = (cfg && cfg->turns_per_launch > 0) ? cfg->turns_per_launch : 0;  // 0: per layout, below
    const int req = cfg ? cfg->cells_per_lane : 0;
    const int cpl = req > 0 ? req : 32 * GOL_DEFAULT_DW;
    if (cpl != 32 && cpl != 64 && cpl != 128) return gol_set_error(GOL_EINVAL, "cells_per_lane must be 32, 64 or 128");
    e->dw = cpl / 32;
    while (e->dw > 1 && (e->Wd % e->dw) != 0) e->dw >>= 1;
    e->band_dw = req == 64 ? 2 : (req == 128 ? 4 : GOL_BAND_DEFAULT_DW);
    e->strip = cfg ? cfg->strip_rows : 0;
    if (layout == GOL_LAYOUT_BAND && W % 1024 != 0) return gol_set_error(GOL_EINVAL, "the band layout needs W %% 1024 == 0");
    e->band_capable = e->bit_capable && layout != GOL_LAYOUT_STANDARD && W % 1024 == 0;
    if (e->k == 0)
        e->k = !e->bit_capable ? GOL_DEFAULT_BYTES_K
                               : ((e->band_capable && e->band_dw == 4) ? GOL_DEFAULT_BAND_K : GOL_DEFAULT_K);
    e->step_flags = cfg ? (cfg->flags & (GOL_STEP_SERIAL | GOL_STEP_EDGE_FIRST | GOL_STEP_OVERLAP)) : 0;
    return GOL_OK;
}

// Shards [0, n) of this process are global ranks e->rank + i of e->nranks.
static int engine_shards(gol_engine *e, const std::vector<int> &devices)
{
    if (e->nranks > 1 && !e->bit_capable)
        return gol_set_error(GOL_EINVAL, "a sharded board needs a bit board: W %% 64 == 0 (W = %lld), layout not BYTES", (long long)e->W);
    if (e->H < e->nranks)
        return gol_set_error(GOL_EINVAL, "%d shards cannot split %lld rows", e->nranks, (long long)e->H);
    e->min_rows = e->H / e->nranks;  // broker.go:172-206: the smallest shard
    // every exchange carries the rows of the longest launch the engine makes
    e->kx = pick_k(e->k, INT64_MAX, e->min_rows, e->band_capable ? e->band_dw : e->dw, e->band_capable);
    e->sh.resize(devices.size());
    for (size_t i = 0; i < devices.size(); ++i) {
        gol_shard &s = e->sh[i];
        s.device = devices[i];
        const int64_t r = e->rank + (int64_t)i;
        int rc = gol_partition_rows(e->H, e->nranks, r, &s.y0, &s.y1);
        if (rc) return rc;
        s.R = s.y1 - s.y0;
        RCCHK(shard_alloc(e, s));
    }
    return GOL_OK;
}

extern "C" int gol_engine_create(int64_t H, int64_t W, const gol_config *cfg, gol_engine **out)
{
    if (!out) return gol_set_error(GOL_EINVAL, "out is NULL");
    *out = nullptr;
    gol_engine *e = new gol_engine();
    int rc = engine_setup(e, H, W, cfg);
    const int n = cfg && cfg->shards > 1 ? cfg->shards : 1;
    const int same = cfg && (cfg->flags & GOL_SHARDS_SAME_DEVICE);
    int transport = cfg ? cfg->transport : GOL_TRANSPORT_AUTO;
    std::vector<int> devs(n);
    if (rc == GOL_OK) {
        int dev0 = cfg ? cfg->device : -1, ndev = 0;
        if (dev0 < 0 && hipGetDevice(&dev0) != hipSuccess) dev0 = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
            rc = gol_set_error(GOL_EHIP, "no HIP device");
        for (int i = 0; rc == GOL_OK && i < n; ++i) devs[i] = same ? dev0 : (dev0 + i) % ndev;
        std::vector<int> sorted(devs);
        std::sort(sorted.begin(), sorted.end());
        const bool distinct = std::unique(sorted.begin(), sorted.end()) == sorted.end();
        if (transport == GOL_TRANSPORT_AUTO)
            transport = n == 1 ? GOL_TRANSPORT_LOCAL : (distinct ? GOL_TRANSPORT_RCCL : GOL_TRANSPORT_LOOPBACK);
        if (transport != GOL_TRANSPORT_LOCAL && transport != GOL_TRANSPORT_LOOPBACK && transport != GOL_TRANSPORT_RCCL)
            rc = gol_set_error(GOL_EINVAL, "unknown transport %d", transport);
        if (transport == GOL_TRANSPORT_LOCAL && n > 1) rc = gol_set_error(GOL_EINVAL, "the local transport has one shard");
    }
    e->nranks = n;
    e->rank = 0;
    e->transport = transport;
    if (rc == GOL_OK) rc = engine_shards(e, devs);
    if (rc == GOL_OK && transport == GOL_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> comms(n);
        ncclResult_t r = ncclCommInitAll(comms.data(), n, devs.data());
        if (r != ncclSuccess) rc = gol_set_error(GOL_ECOMM, "ncclCommInitAll(%d GPUs): %s", n, ncclGetErrorString(r));
        else
            for (int i = 0; i < n; ++i) e->sh[i].nccl = comms[i];
    }
    if (rc == GOL_OK && transport == GOL_TRANSPORT_LOOPBACK)  // peer access between distinct GPUs (copies work without)
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j)
                if (devs[i] != devs[j] && hipSetDevice(devs[i]) == hipSuccess) {
                    (void)hipDeviceEnablePeerAccess(devs[j], 0);
                    (void)hipGetLastError();
                }
    if (rc != GOL_OK) {
        gol_engine_destroy(e);
        return rc;
    }
    *out = e;
    return GOL_OK;
}

extern "C" int gol_rccl_unique_id(uint8_t *id, int64_t len)
{
    if (!id || len < (int64_t)sizeof(ncclUniqueId)) return gol_set_error(GOL_EINVAL, "id needs %d bytes", GOL_RCCL_ID_BYTES);
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return GOL_OK;
}

extern "C" int gol_engine_create_rank(int64_t H, int64_t W, int32_t nranks, int32_t rank, const uint8_t *id,
                                      const gol_config *cfg, gol_engine **out)
{
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || (!id && nranks > 1))
        return gol_set_error(GOL_EINVAL, "bad rank arguments (rank %d of %d)", rank, nranks);
    if (cfg && cfg->shards > 1) return gol_set_error(GOL_EINVAL, "one shard per rank");
    *out = nullptr;
    gol_engine *e = new gol_engine();
    int rc = engine_setup(e, H, W, cfg);
    int dev = cfg ? cfg->device : -1;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    int transport = cfg ? cfg->transport : GOL_TRANSPORT_AUTO;
    if (transport == GOL_TRANSPORT_AUTO) transport = nranks > 1 ? GOL_TRANSPORT_RCCL : GOL_TRANSPORT_LOCAL;
    if (rc == GOL_OK && transport != GOL_TRANSPORT_RCCL && transport != GOL_TRANSPORT_IPC &&
        !(transport == GOL_TRANSPORT_LOCAL && nranks == 1))
        rc = gol_set_error(GOL_EINVAL, "ranks in several processes exchange halos over RCCL or IPC");
    if (rc == GOL_OK && transport == GOL_TRANSPORT_IPC && !id) rc = gol_set_error(GOL_EINVAL, "the IPC transport needs an id");
    e->nranks = nranks;
    e->rank = rank;
    e->rank_mode = true;
    e->transport = transport;
    if (rc == GOL_OK) rc = engine_shards(e, {dev});
    if (rc == GOL_OK && transport == GOL_TRANSPORT_RCCL) {
        ncclUniqueId u;
        if (id) memcpy(&u, id, sizeof u);
        else if (ncclGetUniqueId(&u) != ncclSuccess) rc = gol_set_error(GOL_ECOMM, "ncclGetUniqueId failed");
        ncclResult_t r = rc == GOL_OK ? ncclCommInitRank(&e->sh[0].nccl, nranks, u, rank) : ncclSuccess;
        if (r != ncclSuccess) rc = gol_set_error(GOL_ECOMM, "ncclCommInitRank(rank %d of %d): %s", rank, nranks, ncclGetErrorString(r));
        if (rc == GOL_OK) e->comm = gol_comm_rccl(e->sh[0].nccl);
    }
    if (rc == GOL_OK && transport == GOL_TRANSPORT_IPC) {
        // the ring neighbours this rank pulls its ghost rows from (gol_halo_plan's peers)
        for (int p : {(rank + nranks - 1) % nranks, (rank + 1) % nranks})
            if (p != rank && std::find(e->ipc_peers.begin(), e->ipc_peers.end(), p) == e->ipc_peers.end())
                e->ipc_peers.push_back(p);
        rc = set_dev(dev);
        // the peers pull from a small send buffer, not from the board: importing whole boards
        // (2 GiB each for config 4 over 4 ranks) hung inside the runtime's IPC import
        gol_shard &s0 = e->sh[0];
        const size_t ob = ipc_out_bytes(e);
        if (rc == GOL_OK && hipMalloc(&s0.ipc_out, ob) != hipSuccess) rc = gol_set_error(GOL_EHIP, "IPC send rows: hipMalloc failed");
        if (rc == GOL_OK && (hipMemset(s0.ipc_out, 0, ob) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
            rc = gol_set_error(GOL_EHIP, "IPC send rows: hipMemset failed");
        uint32_t *const bufs[2] = {s0.ipc_out, nullptr};
        if (rc == GOL_OK) rc = gol_ipc::open(id, nranks, rank, dev, H, W, e->kx, bufs, e->ipc_peers, &e->ipc);
        e->comm = e->ipc;
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
    for (auto &s : e->sh) {  // (an IPC wait or signal may still read or write the flag words)
        (void)hipSetDevice(s.device);
        for (hipStream_t st : {s.stream, s.edge, s.comm})
            if (st) (void)hipStreamSynchronize(st);
    }
    delete e->comm;  // the IPC transport unmaps the peers' buffers; RCCL's comm is the shard's
    for (auto &s : e->sh) shard_release(s);
    delete e;
}

extern "C" int gol_engine_topology(gol_engine *e, int32_t *shards, int32_t *nranks, int32_t *rank, int32_t *transport)
{
    if (!e) return gol_set_error(GOL_EINVAL, "engine is NULL");
    if (shards) *shards = (int32_t)e->sh.size();
    if (nranks) *nranks = e->nranks;
    if (rank) *rank = e->rank;
    if (transport) *transport = e->transport;
    return GOL_OK;
}

extern "C" int gol_engine_shard(gol_engine *e, int32_t i, int32_t *device, int64_t *y0, int64_t *y1)
{
    if (!e || i < 0 || i >= (int32_t)e->sh.size()) return gol_set_error(GOL_EINVAL, "no local shard %d", i);
    if (device) *device = e->sh[i].device;
    if (y0) *y0 = e->sh[i].y0;
    if (y1) *y1 = e->sh[i].y1;
    return GOL_OK;
}

// ------------------------------------------------------------------ synchronisation, errors
// Ranks in several processes: whole-board calls are collective (gol_comm).
static bool several(const gol_engine *e) { return e->rank_mode && e->nranks > 1; }

// Wait for every shard's work and read the shards' device error words (one pinned readback
// queued behind the work, so the check costs no extra synchronisation).
// With ranks in several processes the error words are all-reduced first (max), so a fault on
// one rank -- whose rows reach the others through the halo -- fails the call on every rank; it
// also ends every rank's halo copies (the IPC transport's all-reduce is a host barrier behind
// the streams), so no rank reads a neighbour's buffers past this point.  `collective` = false:
// this process's shards only (a call that other ranks do not make).
static int sync_all(gol_engine *e, bool collective = true)
{
    const bool coll = collective && several(e);
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        HIPCHK(hipStreamWaitEvent(s.stream, s.ev_edge, 0));  // (the edge launches' error word writes)
        HIPCHK(hipStreamWaitEvent(s.stream, s.ev_halo, 0));  // (the halo copies, the IPC waits' error word)
        if (coll) RCCHK(e->comm->allreduce_max_u32(s.err, 1, s.stream));
        HIPCHK(hipMemcpyAsync(s.host_word, s.err, sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
    }
    uint32_t flags = 0;
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        HIPCHK(hipStreamSynchronize(s.stream));
        HIPCHK(hipStreamSynchronize(s.edge));
        HIPCHK(hipStreamSynchronize(s.comm));
        flags |= s.host_word[0];
    }
    e->halo_issued = false;
    if (flags) {
        for (auto &s : e->sh) {
            RCCHK(set_dev(s.device));
            HIPCHK(hipMemsetAsync(s.err, 0, sizeof(uint32_t), s.stream));
            s.slots_zero = false;  // a faulted launch may have left counts in them
            s.batch_zero = false;
            // a timed-out pair may have left its claims set: this engine's streams only
            HIPCHK(golk_reset_claims(s.stream));
            HIPCHK(golk_reset_claims(s.edge));
            // a workgroup that gave up may not have freed its CU slot (role placement: speed only)
            HIPCHK(golk_reset_cu_slots(s.device, s.stream));
            HIPCHK(hipStreamSynchronize(s.stream));
            HIPCHK(hipStreamSynchronize(s.edge));
        }
        e->halo_ok = false;
        return gol_set_error(GOL_EHIP, "device fault in a step kernel (error flags 0x%x: %s); the board is not valid",
                             flags, (flags & GOLK_ERR_SPIN) ? "a pipeline wave timed out waiting for its neighbour"
                                    : (flags & GOLK_ERR_IPC) ? "an IPC rank timed out waiting for a neighbour's halo rows"
                                                             : "?");
    }
    if (e->mode == GOL_MODE_BITS)
        for (auto &s : e->sh) free_exact_bytes(s);  // the exact first turn's byte rows, once used
    return GOL_OK;
}

// Collective barrier of the ranks of a several-process engine (a one-element all-reduce).
static int rank_barrier(gol_engine *e)
{
    if (!several(e)) return GOL_OK;
    gol_shard &s = e->sh[0];
    RCCHK(set_dev(s.device));
    return e->comm->barrier(s.coll, s.stream);
}

// Before a stepping call with several ranks: the ranks agree on the board state, and any rank
// whose halo is stale (its rows changed outside a step: load_words on that rank alone) makes
// every rank exchange again, so the exchanges -- collective, paired in order -- stay matched.
static int agree_step_state(gol_engine *e)
{
    if (!several(e)) return GOL_OK;
    gol_shard &s = e->sh[0];
    RCCHK(set_dev(s.device));
    uint32_t *v = s.host_word + 4;  // [stale halo, mode, cur, band, ~mode, ~cur, ~band]: max of x and of ~x
    const uint32_t st[3] = {(uint32_t)e->mode, (uint32_t)e->cur, (uint32_t)e->band};
    v[0] = e->halo_ok ? 0u : 1u;
    for (int i = 0; i < 3; ++i) {
        v[1 + i] = st[i];
        v[4 + i] = ~st[i];
    }
    HIPCHK(hipMemcpyAsync(s.coll, v, 7 * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream));
    RCCHK(e->comm->allreduce_max_u32(s.coll, 7, s.stream));
    HIPCHK(hipMemcpyAsync(v, s.coll, 7 * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipStreamSynchronize(s.stream));
    for (int i = 0; i < 3; ++i)
        if (v[1 + i] != ~v[4 + i])
            return gol_set_error(GOL_ESTATE, "the ranks disagree on the board state (mode / buffer / layout)");
    if (v[0]) e->halo_ok = false;
    return GOL_OK;
}

// The board is about to change outside a step (load, layout conversion, exact first turn):
// the halo of the current buffer is no longer the board's, and the exchange still in flight
// (it reads and writes the buffers) finishes before the compute stream writes them.
static int invalidate_halo(gol_engine *e)
{
    if (e->halo_issued)
        for (auto &s : e->sh) {
            RCCHK(set_dev(s.device));
            HIPCHK(hipStreamWaitEvent(s.stream, s.ev_edge, 0));
            for (auto &t : e->sh) HIPCHK(hipStreamWaitEvent(s.stream, t.ev_halo, 0));  // (loopback: t reads my rows)
            // (IPC: the neighbours read only this rank's send buffer ipc_out, never its board, and
            // its own copies into ipc_out are behind ev_halo: nothing to wait for across processes)
        }
    e->halo_ok = false;
    return GOL_OK;
}

// ------------------------------------------------------------------ layout conversion
// The band layout is a stepping detail: convert on the first step, convert back before
// anything reads the bits.  Both are one HBM pass (32x32 bit transposes) per shard.
static int convert(gol_engine *e, bool to_band)
{
    if (e->band == to_band || e->mode != GOL_MODE_BITS) return GOL_OK;
    RCCHK(invalidate_halo(e));
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        HIPCHK(golk_band_convert(to_band, s.bits[e->cur], s.bits[1 - e->cur], s.R, e->Wd, e->pitch, e->pitch, s.stream));
    }
    e->cur = 1 - e->cur;
    e->band = to_band;
    return GOL_OK;
}
static int ensure_standard(gol_engine *e) { return convert(e, false); }

// ------------------------------------------------------------------ one k-turn step
static int copy_rows(gol_shard &dst_s, uint32_t *dst, const gol_shard &src_s, const uint32_t *src, size_t bytes,
                     hipStream_t st)
{
    if (dst_s.device == src_s.device) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
    else HIPCHK(hipMemcpyPeerAsync(dst, dst_s.device, src, src_s.device, bytes, st));
    return GOL_OK;
}

// The halo plan of local shard i (gol_halo_plan: the schedule golhip.sharded runs as well).
static int plan_of(gol_engine *e, int i, gol_halo_op (&ops)[4])
{
    int32_t n = 0;
    RCCHK(gol_halo_plan(e->H, e->nranks, e->rank + i, e->kx, ops, 4, &n));
#ifdef GOL_TEST_MISPAIR
    // Test build only (make mispair -> libgolhip_mispair.so, tests/test_gpu_ranks.py): the rows
    // received from below land in the ghost rows above and vice versa -- a mis-paired halo that
    // bench.py's parity check must catch.
    int r[2], nr = 0;
    for (int j = 0; j < 4; ++j)
        if (ops[j].kind == GOL_HALO_RECV && nr < 2) r[nr++] = j;
    if (nr == 2) std::swap(ops[r[0]].row, ops[r[1]].row);
#endif
    return n == 4 ? GOL_OK : gol_set_error(GOL_EINVAL, "halo plan of %d ops", n);
}

// Exchange the kx halo rows of bits[cur] on the comm streams, once every shard's ev_edge (the
// rows it sends are written) has been recorded; records ev_halo.  Every transport runs the
// shards' gol_halo_plan in issue order.  LOCAL / LOOPBACK execute it as device copies, pairing
// each receive with the sender's matching send exactly as RCCL does (the n-th receive of shard
// s from shard p gets p's n-th send to s), so the one-GPU loopback tests exercise the RCCL
// matching of the same plan, including nranks = 2 (one peer on both sides) and the one-shard
// torus wrap (a shard sending to itself).
// One shard that is the whole torus (LOCAL transport): the step launches read the wrap rows from
// the board itself (step_launch), so there is nothing to exchange.  (Copying them into the ghost
// rows beside the interior instead, for the contiguous-row kernel that ran 1.3-2 % faster in
// tools/step_cost.py, measured -0.5 % on the weak board through bench.py, same box:
// profiles/r04/r04d_ab_steps.jsonl.)
static bool local_wrap(const gol_engine *e)
{
    return e->transport == GOL_TRANSPORT_LOCAL && e->sh.size() == 1 && e->nranks == 1;
}

static int xtime_start(gol_engine *e, gol_shard &s, hipStream_t st, size_t *ev);
static int xtime_wait(gol_shard &s, hipStream_t st, size_t ev);
static int xtime_waited(gol_shard &s, hipStream_t st, size_t ev);
static int xtime_stop(gol_engine *e, gol_shard &s, hipStream_t st, size_t ev, int shard);

// IPC transport (one shard per process): this rank's exchange xn on its comm stream, pulling
// each ghost block out of the neighbour's send buffer (ipc_out, mapped by the peers):
//   1. once the rows this rank sends are written (ev_edge), copy every send of my gol_halo_plan
//      into ipc_out slot (xn & 1, op index), then signal READY = xn;
//   2. wait until each neighbour's READY has reached xn (its send rows for this exchange are in);
//   3. copy every receive of my gol_halo_plan from the peer's matching send slot (the peer's nth
//      send to me for my nth receive from it: the pairing RCCL applies to the same plans).
// A neighbour overwrites send slot (xn & 1) only at its exchange xn+2, which follows (on its comm
// stream) its exchange xn+1, which waited for my READY xn+1, which I signal on my comm stream
// after my pulls of xn: so nothing else orders my copies against its writes, whether or not steps
// run between the exchanges.  Peers never read my board, so writes of the board outside a step
// (a load, a layout conversion, the exact first turn) need no cross-process wait either.
static int exchange_ipc(gol_engine *e)
{
    gol_shard &s = e->sh[0];
    RCCHK(set_dev(s.device));
    const int c = e->cur;
    const int64_t P = e->pitch;
    gol_halo_op mine[4];
    RCCHK(plan_of(e, 0, mine));
    const uint32_t xn = ++e->xn;
    const int64_t slot_words = (int64_t)GOL_GHOST_ROWS * P;
    auto out_slot = [&](uint32_t *base, int m) { return base + ((int64_t)(xn & 1) * 4 + m) * slot_words; };
    HIPCHK(hipStreamWaitEvent(s.comm, s.ev_edge, 0));
    size_t xev;
    RCCHK(xtime_start(e, s, s.comm, &xev));
    for (int m = 0; m < 4; ++m)
        if (mine[m].kind == GOL_HALO_SEND) {
            if (mine[m].rows > GOL_GHOST_ROWS) return gol_set_error(GOL_EINVAL, "halo plan: %d rows per send", mine[m].rows);
            HIPCHK(hipMemcpyAsync(out_slot(s.ipc_out, m), s.bits[c] + mine[m].row * P, (size_t)mine[m].rows * P * sizeof(uint32_t),
                                  hipMemcpyDeviceToDevice, s.comm));
        }
    RCCHK(e->ipc->signal(s.comm, GOL_IPC_READY, xn));
    RCCHK(xtime_wait(s, s.comm, xev));
    RCCHK(e->ipc->wait(s.comm, e->ipc_peers, GOL_IPC_READY, xn, s.err));
    RCCHK(xtime_waited(s, s.comm, xev));
    for (int j = 0; j < 4; ++j) {
        const gol_halo_op &rv = mine[j];
        if (rv.kind != GOL_HALO_RECV) continue;
        int nth = 0;  // this is my nth receive from rv.peer
        for (int jj = 0; jj < j; ++jj) nth += mine[jj].kind == GOL_HALO_RECV && mine[jj].peer == rv.peer;
        gol_halo_op theirs[4];
        int32_t n = 0;
        RCCHK(gol_halo_plan(e->H, e->nranks, rv.peer, e->kx, theirs, 4, &n));
        int sm = -1;  // the peer's nth send to me (its op index)
        for (int m = 0, cnt = 0; m < n && sm < 0; ++m)
            if (theirs[m].kind == GOL_HALO_SEND && theirs[m].peer == e->rank && cnt++ == nth) sm = m;
        if (sm < 0 || theirs[sm].rows != rv.rows) return gol_set_error(GOL_EINVAL, "halo plan: unmatched receive");
        uint32_t *base = rv.peer == e->rank ? s.ipc_out : e->ipc->peer_buf(rv.peer, 0);
        if (!base) return gol_set_error(GOL_ESTATE, "IPC: rank %d is not mapped", rv.peer);
        HIPCHK(hipMemcpyAsync(s.bits[c] + rv.row * P, out_slot(base, sm), (size_t)rv.rows * P * sizeof(uint32_t),
                              hipMemcpyDeviceToDevice, s.comm));
    }
    RCCHK(xtime_stop(e, s, s.comm, xev, 0));
    HIPCHK(hipEventRecord(s.ev_halo, s.comm));
    e->halo_issued = true;
    return GOL_OK;
}

static int exchange(gol_engine *e, bool on_compute = false)
{
    if (local_wrap(e)) {
        e->halo_issued = false;
        return GOL_OK;
    }
    if (e->transport == GOL_TRANSPORT_IPC) return exchange_ipc(e);
    const int n = (int)e->sh.size();
    const int c = e->cur;
    const int64_t P = e->pitch;
    const size_t hb = (size_t)e->kx * P * sizeof(uint32_t);
    std::vector<std::array<gol_halo_op, 4>> plans(n);
    for (int i = 0; i < n; ++i) {
        gol_halo_op ops[4];
        RCCHK(plan_of(e, i, ops));
        std::copy(ops, ops + 4, plans[i].begin());
    }
    auto local = [&](int global) { return global - e->rank; };  // local shard index of a global rank
    if (e->transport != GOL_TRANSPORT_RCCL) {
        for (int i = 0; i < n; ++i) {
            gol_shard &s = e->sh[i];
            RCCHK(set_dev(s.device));
            // my ghost rows are no longer read (my edge launches) and the rows my peers send me
            // are written (theirs)
            for (const auto &op : plans[i])
                HIPCHK(hipStreamWaitEvent(s.comm, e->sh[local(op.peer)].ev_edge, 0));
            size_t xev = SIZE_MAX;
            for (int j = 0; j < 4; ++j) {
                const gol_halo_op &rv = plans[i][j];
                if (rv.kind != GOL_HALO_RECV) continue;
                int nth = 0;  // this is my nth receive from rv.peer
                for (int jj = 0; jj < j; ++jj) nth += plans[i][jj].kind == GOL_HALO_RECV && plans[i][jj].peer == rv.peer;
                const int p = local(rv.peer);
                const gol_halo_op *sd = nullptr;  // the peer's nth send to me
                for (int m = 0, cnt = 0; m < 4 && !sd; ++m) {
                    const gol_halo_op &o = plans[p][m];
                    if (o.kind == GOL_HALO_SEND && o.peer == e->rank + i && cnt++ == nth) sd = &o;
                }
                if (!sd || sd->rows != rv.rows) return gol_set_error(GOL_EINVAL, "halo plan: unmatched receive");
                gol_shard &ps = e->sh[p];
                if (xev == SIZE_MAX) {  // (the peers' rows are in once the event waits above pass: no wait here)
                    RCCHK(xtime_start(e, s, s.comm, &xev));
                    RCCHK(xtime_wait(s, s.comm, xev));
                    RCCHK(xtime_waited(s, s.comm, xev));
                }
                RCCHK(copy_rows(s, s.bits[c] + rv.row * P, ps, ps.bits[c] + sd->row * P, hb, s.comm));
            }
            RCCHK(xtime_stop(e, s, s.comm, xev, i));
            HIPCHK(hipEventRecord(s.ev_halo, s.comm));
        }
        e->halo_issued = true;
        return GOL_OK;
    }
    // RCCL: one group over every local shard (ncclCommInitAll comms must be driven together),
    // on the comm streams once ev_edge is in, or -- on_compute: after a step whose launches were
    // all on the compute stream (SERIAL) -- right on the compute stream, which orders it after
    // the step and before the next without two cross-stream event hops (config 4's 32768-row
    // share: 0.77 -> 0.74 ms per step)
    auto xs = [&](gol_shard &s) { return on_compute ? s.stream : s.comm; };
    if (!on_compute)
        for (auto &s : e->sh) {
            RCCHK(set_dev(s.device));
            HIPCHK(hipStreamWaitEvent(s.comm, s.ev_edge, 0));
        }
    std::vector<size_t> xev(n);
    bool timed = false;
    for (int i = 0; i < n; ++i) {
        RCCHK(set_dev(e->sh[i].device));
        RCCHK(xtime_start(e, e->sh[i], xs(e->sh[i]), &xev[i]));
        RCCHK(xtime_wait(e->sh[i], xs(e->sh[i]), xev[i]));
        timed |= xev[i] != SIZE_MAX;
    }
    ncclResult_t first = ncclSuccess;
    if (timed) {
        // Only while exchanges are timed (gol_engine_exchange_split): one word to and from each
        // distinct ring neighbour first.  It completes once every neighbour has reached its
        // exchange, so its duration is this rank's wait for them and the group after it is the
        // transfer of the halo rows.  (Device words coll[8..10]: not used by the agreement.)
        first = ncclGroupStart();
        for (int i = 0; i < n && first == ncclSuccess; ++i) {
            gol_shard &s = e->sh[i];
            int peers[4], np = 0;
            for (const auto &op : plans[i])
                if (std::find(peers, peers + np, op.peer) == peers + np) peers[np++] = op.peer;
            for (int j = 0; j < np; ++j) {
                ncclResult_t x = ncclSend(s.coll + 8, 1, ncclUint32, peers[j], s.nccl, xs(s));
                if (x == ncclSuccess) x = ncclRecv(s.coll + 9 + (j & 1), 1, ncclUint32, peers[j], s.nccl, xs(s));
                if (x != ncclSuccess && first == ncclSuccess) first = x;
            }
        }
        const ncclResult_t end = ncclGroupEnd();
        if (first != ncclSuccess || end != ncclSuccess)
            return gol_set_error(GOL_ECOMM, "halo handshake: %s", ncclGetErrorString(first != ncclSuccess ? first : end));
    }
    for (int i = 0; i < n; ++i) {
        RCCHK(set_dev(e->sh[i].device));
        RCCHK(xtime_waited(e->sh[i], xs(e->sh[i]), xev[i]));
    }
    first = ncclGroupStart();
    for (int i = 0; i < n && first == ncclSuccess; ++i) {
        gol_shard &s = e->sh[i];
        uint32_t *mid = s.bits[c];
        for (const auto &op : plans[i]) {
            const size_t cnt = (size_t)op.rows * P;
            const ncclResult_t x = op.kind == GOL_HALO_SEND
                                       ? ncclSend(mid + op.row * P, cnt, ncclUint32, op.peer, s.nccl, xs(s))
                                       : ncclRecv(mid + op.row * P, cnt, ncclUint32, op.peer, s.nccl, xs(s));
            if (x != ncclSuccess && first == ncclSuccess) first = x;
        }
    }
    const ncclResult_t end = ncclGroupEnd();
    if (first != ncclSuccess || end != ncclSuccess)
        return gol_set_error(GOL_ECOMM, "halo exchange: %s", ncclGetErrorString(first != ncclSuccess ? first : end));
    for (int i = 0; i < n; ++i) {
        gol_shard &s = e->sh[i];
        RCCHK(set_dev(s.device));
        RCCHK(xtime_stop(e, s, xs(s), xev[i], i));
        HIPCHK(hipEventRecord(s.ev_halo, xs(s)));
    }
    e->halo_issued = true;
    return GOL_OK;
}

// Exchange the halo of the board as it stands (after a load, a conversion or a step outside
// launch_k): the sent rows are whatever the compute stream wrote last.
static int exchange_current(gol_engine *e)
{
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        HIPCHK(hipStreamWaitEvent(s.stream, s.ev_edge, 0));
        HIPCHK(hipEventRecord(s.ev_edge, s.stream));
    }
    e->halo_on_compute = false;
    RCCHK(exchange(e));
    e->halo_ok = true;
    return GOL_OK;
}

static int step_launch(gol_engine *e, gol_shard &s, hipStream_t st, int k, int64_t row0, int64_t rows, uint64_t *slots)
{
    if (rows <= 0) return GOL_OK;
    uint32_t *mid = s.bits[e->cur];
    const uint32_t *top = mid - (int64_t)k * e->pitch, *bot = mid + s.R * e->pitch;  // the ghost rows
    if (local_wrap(e)) {  // the torus wrap straight from the board: rows R-k .. R-1 above, 0 .. k-1 below
        top = mid + (s.R - k) * e->pitch;
        bot = mid;
    }
    uint32_t *dst = s.bits[1 - e->cur];
    if (e->band)
        HIPCHK(golk_band_step(top, mid, bot, dst, s.R, e->Wd, e->pitch, row0, rows, k, e->band_dw, e->strip, slots, s.err, st));
    else
        HIPCHK(golk_bits_step(top, mid, bot, dst, s.R, e->Wd, e->pitch, row0, rows, k, e->dw, e->strip, slots, st));
    return GOL_OK;
}

// Timing of one shard-step: events on the compute stream from the step's start to its end
// (the edge stream joined).  The pool is folded into running sums when it is full -- only between
// stepping calls (timing_begin): a call still open holds its start event and its exchanges' events,
// unrecorded or unfolded, so within a call the pool grows instead.
static int fold_timing(gol_engine *e)
{
    for (const auto &t : e->timed) {
        gol_shard &s = e->sh[t.shard];
        RCCHK(set_dev(s.device));
        HIPCHK(hipEventSynchronize(s.tev[t.ev + 1]));
        float x = 0;
        HIPCHK(hipEventElapsedTime(&x, s.tev[t.ev], s.tev[t.ev + 1]));
        if (t.exchange) {
            float w = 0;
            HIPCHK(hipEventElapsedTime(&w, s.tev[t.ev + 2], s.tev[t.ev + 3]));
            e->x_ms += x;
            e->x_wait_ms += w;
            e->x_n += 1;
            continue;
        }
        e->t_ms += x;
        e->t_cells += t.cell_updates;
        e->t_n += t.steps;
    }
    e->timed.clear();
    for (auto &s : e->sh) s.tused = 0;
    return GOL_OK;
}

// n consecutive events of shard s's pool (never folds: see fold_timing).
static int timing_event(gol_shard &s, size_t *ev, size_t n = 2)
{
    while (s.tused + n > s.tev.size()) {
        hipEvent_t x;
        HIPCHK(hipEventCreate(&x));
        s.tev.push_back(x);
    }
    *ev = s.tused;
    s.tused += n;
    return GOL_OK;
}

// Timing of one stepping call (gol_engine_set_timing): one event pair per shard on its compute
// stream around all the call's launches (per-launch events cost the GPU ~10-30 us each, a large
// share of a 0.4 ms step), averaged over its steps by gol_engine_timing.
static int timing_begin(gol_engine *e)
{
    if (!e->timing) return GOL_OK;
    bool full = false;
    for (const auto &s : e->sh) full |= s.tused + 2 > GOL_TIMING_EVENTS;
    if (full) RCCHK(fold_timing(e));  // (no call is open here)
    e->tcall_ev.assign(e->sh.size(), 0);
    e->tcall_cells.assign(e->sh.size(), 0.0);
    e->tcall_steps = 0;
    for (size_t i = 0; i < e->sh.size(); ++i) {
        gol_shard &s = e->sh[i];
        int rc = set_dev(s.device);
        if (rc == GOL_OK) rc = timing_event(s, &e->tcall_ev[i]);
        if (rc == GOL_OK && hipEventRecord(s.tev[e->tcall_ev[i]], s.stream) != hipSuccess)
            rc = gol_set_error(GOL_EHIP, "timing: hipEventRecord failed");
        if (rc != GOL_OK) {
            e->tcall_ev.clear();  // no call is open
            return rc;
        }
    }
    return GOL_OK;
}

// A stepping call is being timed (timing_begin .. timing_end): launches outside such a call
// (gol_engine_step_flips) are not.
static bool timing_open(const gol_engine *e) { return e->timing && e->tcall_ev.size() == e->sh.size(); }

// GOL_TIMING_EXCHANGE: four events around one shard's part of a halo exchange on stream st --
// xtime_start before the exchange's first operation on st, xtime_wait / xtime_waited around the
// part that waits for the neighbours (gol_engine_exchange_split), xtime_stop after its last.
static int xtime_start(gol_engine *e, gol_shard &s, hipStream_t st, size_t *ev)
{
    *ev = SIZE_MAX;
    if (!e->timing_x || !timing_open(e)) return GOL_OK;
    RCCHK(timing_event(s, ev, 4));
    HIPCHK(hipEventRecord(s.tev[*ev], st));
    return GOL_OK;
}
static int xtime_wait(gol_shard &s, hipStream_t st, size_t ev)
{
    if (ev != SIZE_MAX) HIPCHK(hipEventRecord(s.tev[ev + 2], st));
    return GOL_OK;
}
static int xtime_waited(gol_shard &s, hipStream_t st, size_t ev)
{
    if (ev != SIZE_MAX) HIPCHK(hipEventRecord(s.tev[ev + 3], st));
    return GOL_OK;
}
static int xtime_stop(gol_engine *e, gol_shard &s, hipStream_t st, size_t ev, int shard)
{
    if (ev == SIZE_MAX) return GOL_OK;
    HIPCHK(hipEventRecord(s.tev[ev + 1], st));
    gol_timed t{shard, ev, 0.0, 0};
    t.exchange = true;
    e->timed.push_back(t);
    return GOL_OK;
}

static int timing_end(gol_engine *e)
{
    if (!timing_open(e)) return GOL_OK;
    for (size_t i = 0; i < e->sh.size(); ++i) {
        gol_shard &s = e->sh[i];
        RCCHK(set_dev(s.device));
        HIPCHK(hipStreamWaitEvent(s.stream, s.ev_edge, 0));  // (edge launches of the last step)
        HIPCHK(hipEventRecord(s.tev[e->tcall_ev[i] + 1], s.stream));
        if (e->tcall_steps > 0) e->timed.push_back({(int)i, e->tcall_ev[i], e->tcall_cells[i], e->tcall_steps});
    }
    e->tcall_ev.clear();
    return GOL_OK;
}

// The step plan of shard s (gol_step_plan flags): as configured, else OVERLAP when the shard's
// launch runs many rounds of workgroups (the edge launches then share the CUs with the interior
// at no cost: +1 % on the 2^17 x 2^20 board), SERIAL when it is a launch of one or a few rounds,
// whose rank-weighted strips (gol_kernels.hip StripMap) assume they have the CUs to themselves
// (a concurrent edge launch cost 7 % on a 32768 x 262144 shard, profiles/r03a_step_cost).
static int step_mode(gol_engine *e, const gol_shard &s, int k)
{
    if (e->step_flags) return e->step_flags;
    if (local_wrap(e)) return GOL_STEP_SERIAL;  // nothing to exchange, nothing to overlap
    const double rounds = golk_step_rounds(e->band, s.R, e->Wd, e->pitch, k, e->band ? e->band_dw : e->dw, e->strip);
    return rounds > GOL_OVERLAP_ROUNDS ? GOL_STEP_OVERLAP : GOL_STEP_SERIAL;
}

// k turns of every shard, as gol_step_plan lays them out: the edge rows (they read the halo)
// on the edge stream and the interior beside them on the compute stream; the next step's halo
// exchange starts as soon as the edge rows are written, while the interior is still running.
// With `count` the alive cells of the output are added to each shard's slots.
static uint64_t *batch_slots(gol_shard &s, int64_t ci) { return s.slots + (1 + ci % GOL_SLOT_BATCH) * SLOT_WORDS; }

// Reduce the pending count points' slot arrays into counts[pend_first, pend_first + pend_n) (the
// reduce leaves them zeroed).
static int flush_counts(gol_engine *e)
{
    if (e->pend_n == 0) return GOL_OK;
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        HIPCHK(golk_slots_reduce(batch_slots(s, e->pend_first), e->pend_n, s.counts + e->pend_first, s.stream));
    }
    e->pend_n = 0;
    return GOL_OK;
}

// Before the counted launch of point ci: the pending run must stay contiguous in the arrays, and
// after a fault every array is zeroed again.
static int batch_begin(gol_engine *e, int64_t ci)
{
    if (e->pend_n && (e->pend_first + e->pend_n != ci || ci % GOL_SLOT_BATCH == 0)) RCCHK(flush_counts(e));
    for (auto &s : e->sh) {
        if (s.batch_zero) continue;
        RCCHK(set_dev(s.device));
        HIPCHK(hipMemsetAsync(s.slots + SLOT_WORDS, 0, SLOT_BYTES * GOL_SLOT_BATCH, s.stream));
        s.batch_zero = true;
    }
    return GOL_OK;
}

#ifndef GOL_LAZY_EVENTS
#define GOL_LAZY_EVENTS 1
#endif
#ifndef GOL_HALO_ON_COMPUTE
#define GOL_HALO_ON_COMPUTE 1
#endif
static int launch_k(gol_engine *e, int k, int64_t count_ci)
{
    const bool count = count_ci >= 0;
    if (k > e->kx) return gol_set_error(GOL_EINVAL, "k %d > the exchanged halo (%d rows)", k, e->kx);
    if (!e->halo_ok) RCCHK(exchange_current(e));
    const int n = (int)e->sh.size();
    bool serial = true;  // every shard's launches on its compute stream
    for (int i = 0; i < n; ++i) serial &= step_mode(e, e->sh[i], k) == GOL_STEP_SERIAL;
    // the next step's halo: RCCL after a SERIAL step goes on the compute streams themselves
    const bool on_compute = GOL_HALO_ON_COMPUTE && serial && e->transport == GOL_TRANSPORT_RCCL;
    // A step whose events no other stream reads records none: one shard with nothing to exchange,
    // or an RCCL exchange on the compute streams, and every launch on the compute stream.  Each
    // record is a marker between two band launches that left the GPU idle ~10 us (65536^2: 3 % of
    // a 0.33 ms launch).  ev_edge then keeps an older record, which later waits pass at once
    // (they are all on the compute stream).
    const bool quiet = GOL_LAZY_EVENTS && (local_wrap(e) || on_compute);
    for (int i = 0; i < n; ++i) {
        gol_shard &s = e->sh[i];
        RCCHK(set_dev(s.device));
        gol_launch plan[3];
        int32_t np = 0;
        const int mode = step_mode(e, s, k);
        RCCHK(gol_step_plan(s.R, k, e->kx, mode, plan, 3, &np));
        uint64_t *slots = count ? batch_slots(s, count_ci) : nullptr;  // (zeroed: batch_begin)
        if (timing_open(e)) e->tcall_cells[i] += (double)s.R * (double)e->W * k;
        bool plan_edge = false;
        for (int j = 0; j < np; ++j) plan_edge |= plan[j].stream == GOL_LAUNCH_EDGE;
        const bool markers = !(quiet && !plan_edge);
        if (markers) HIPCHK(hipEventRecord(s.ev_start, s.stream));  // the step's inputs are complete, slots zeroed
        bool edge_used = false, waited[2] = {false, false};
        int last_halo = -1;  // the last launch that reads the halo writes the rows the exchange sends
        for (int j = 0; j < np; ++j)
            if (plan[j].needs_halo) last_halo = j;
        for (int j = 0; j < np; ++j) {
            const gol_launch &L = plan[j];
            const bool on_edge = L.stream == GOL_LAUNCH_EDGE;
            hipStream_t st = on_edge ? s.edge : s.stream;
            if (on_edge && !edge_used) HIPCHK(hipStreamWaitEvent(st, s.ev_start, 0));
            edge_used |= on_edge;
            if (L.needs_halo && !waited[on_edge]) {
                waited[on_edge] = true;
                // the halo is in; and my rows the peers' copies read (LOCAL / LOOPBACK) are no
                // longer read when this launch overwrites them (RCCL on the compute stream:
                // stream order, no wait)
                if (!(e->halo_on_compute && e->transport == GOL_TRANSPORT_RCCL))
                    for (auto &t : e->sh) HIPCHK(hipStreamWaitEvent(st, t.ev_halo, 0));
            }
            RCCHK(step_launch(e, s, st, k, L.row0, L.rows, slots));
            if (j == last_halo && markers) HIPCHK(hipEventRecord(s.ev_edge, st));
        }
        if (edge_used) HIPCHK(hipStreamWaitEvent(s.stream, s.ev_edge, 0));
    }
    if (timing_open(e)) e->tcall_steps += 1;
    e->cur = 1 - e->cur;
    // the next step's halo: waits only for each shard's ev_edge (or, on_compute, stream order)
    e->halo_on_compute = on_compute;
    RCCHK(exchange(e, e->halo_on_compute));
    e->halo_ok = true;
    return GOL_OK;
}

// Turn 1 of a board loaded with bytes other than 0/255 (worker.go:26-37): every shard runs the
// exact byte kernel over its R rows plus the two halo rows it loaded, then packs the result.
static int exact_turn(gol_engine *e)
{
    RCCHK(invalidate_halo(e));
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        HIPCHK(golk_bytes_step(s.bytes[0], s.R + 2, e->W, e->bstride, 1, s.R + 1, s.bytes[1], e->bstride, s.stream));
        HIPCHK(golk_pack(s.bytes[1], s.R, e->W, e->bstride, s.bits[0], e->pitch, nullptr, s.stream));
    }
    e->cur = 0;
    e->band = false;
    e->mode = GOL_MODE_BITS;
    return GOL_OK;
}

// Alive count of the current board into each shard's slots (zeroed first).
static int count_into_slots(gol_engine *e)
{
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        if (!s.slots_zero) HIPCHK(hipMemsetAsync(s.slots, 0, SLOT_BYTES, s.stream));
        s.slots_zero = false;
        if (e->mode == GOL_MODE_BITS)
            HIPCHK(golk_popcount(s.bits[e->cur], s.R, e->Wd, e->pitch, s.slots, s.stream));
        else if (e->mode == GOL_MODE_EXACT)
            HIPCHK(golk_count_bytes(s.bytes[0] + e->bstride, s.R, e->W, e->bstride, s.slots, s.stream));
        else
            HIPCHK(golk_count_bytes(s.bytes[e->bcur], e->H, e->W, e->bstride, s.slots, s.stream));
    }
    return GOL_OK;
}

// Advance n turns; with ci >= 0 store the alive count after them in every shard's counts[ci].
static int advance(gol_engine *e, int64_t n, int64_t ci)
{
    bool counted = false;  // the last launch fused the count
    while (n > 0) {
        counted = false;
        if (e->mode == GOL_MODE_EXACT) {
            RCCHK(exact_turn(e));
            e->turn += 1;
            n -= 1;
            continue;
        }
        if (e->mode == GOL_MODE_BYTES) {  // W % 64 != 0 or GOL_LAYOUT_BYTES: one shard, the byte board
            gol_shard &s = e->sh[0];
            RCCHK(set_dev(s.device));
            const uint8_t *mid = s.bytes[e->bcur];
            if (e->bytes_binary && e->W % 32 == 0) {
                // 0/255 byte board: k turns per launch on the bytes (torus wrap through top/bot)
                const int k = e->k >= 32 && n >= 32 && e->H >= 32 ? 32 : pick_k(e->k, n, e->H, 1, false);
                const bool last = n == k && ci >= 0;
                if (last) RCCHK(batch_begin(e, ci));
                HIPCHK(golk_bytes_blocked(mid + (e->H - k) * e->bstride, mid, mid, s.bytes[1 - e->bcur], e->H, e->W,
                                          e->bstride, 0, e->H, k, e->strip, last ? batch_slots(s, ci) : nullptr, s.err,
                                          s.stream));
                if (timing_open(e)) {
                    e->tcall_cells[0] += (double)e->H * (double)e->W * k;
                    e->tcall_steps += 1;
                }
                e->bcur = 1 - e->bcur;
                e->turn += k;
                n -= k;
                counted = last;
                continue;
            }
            HIPCHK(golk_bytes_step(mid, e->H, e->W, e->bstride, 0, e->H, s.bytes[1 - e->bcur], e->bstride, s.stream));
            e->bcur = 1 - e->bcur;
            e->bytes_binary = true;  // one exact turn leaves only 0/255
            e->turn += 1;
            n -= 1;
            continue;
        }
        if (e->band_capable) RCCHK(convert(e, true));
        const int k = pick_k(e->k, n, e->min_rows, e->band ? e->band_dw : e->dw, e->band);
        const bool last = n == k && ci >= 0;
        if (last) RCCHK(batch_begin(e, ci));
        RCCHK(launch_k(e, k, last ? ci : -1));
        e->turn += k;
        n -= k;
        counted = last;
    }
    if (ci >= 0 && counted) {  // reduced with its run (flush_counts)
        if (e->pend_n == 0) e->pend_first = ci;
        ++e->pend_n;
    } else if (ci >= 0) {
        RCCHK(flush_counts(e));
        RCCHK(count_into_slots(e));
        for (auto &s : e->sh) {
            RCCHK(set_dev(s.device));
            HIPCHK(golk_slots_reduce(s.slots, 1, s.counts + ci, s.stream));
            s.slots_zero = true;
        }
    }
    return GOL_OK;
}

int gol_engine_step_async(gol_engine *e, int64_t turns) { return advance(e, turns, -1); }

extern "C" int gol_engine_step(gol_engine *e, int64_t turns)
{
    if (!e || turns < 0) return gol_set_error(GOL_EINVAL, "bad step arguments");
    RCCHK(agree_step_state(e));
    RCCHK(timing_begin(e));
    int rc = advance(e, turns, -1);
    const int rt = timing_end(e);
    if (!rc) rc = rt;
    const int rs = sync_all(e);
    return rc ? rc : rs;
}

// Per-shard counts[0..n) -> the whole board's counts (host sum over local shards, RCCL sum
// over the ranks of other processes).
static int collect_counts(gol_engine *e, int64_t n, uint64_t *out)
{
    std::vector<uint64_t> tmp(e->sh.size() * n);
    for (size_t i = 0; i < e->sh.size(); ++i) {
        gol_shard &s = e->sh[i];
        RCCHK(set_dev(s.device));
        if (several(e)) RCCHK(e->comm->allreduce_sum_u64(s.counts, n, s.stream));
        HIPCHK(hipMemcpyAsync(tmp.data() + i * n, s.counts, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream));
    }
    RCCHK(sync_all(e));
    for (int64_t j = 0; j < n; ++j) {
        uint64_t v = 0;
        for (size_t i = 0; i < e->sh.size(); ++i) v += tmp[i * n + j];
        out[j] = v;
    }
    return GOL_OK;
}

extern "C" int gol_engine_step_counted(gol_engine *e, int64_t turns, int64_t every, uint64_t *counts, int64_t cap)
{
    if (!e || turns < 0 || every <= 0 || (turns / every > 0 && (!counts || cap < turns / every)))
        return gol_set_error(GOL_EINVAL, "bad step_counted arguments (turns %lld, every %lld, cap %lld)", (long long)turns,
                             (long long)every, (long long)cap);
    const int64_t n = turns / every;
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        RCCHK(ensure_counts(s, n));
    }
    RCCHK(agree_step_state(e));
    e->pend_n = 0;
    int rc = timing_begin(e);
    int64_t left = turns, ci = 0;
    while (left > 0 && rc == GOL_OK) {
        const int64_t seg = std::min(every, left);
        rc = advance(e, seg, seg == every ? ci : -1);
        if (seg == every) ++ci;
        left -= seg;
    }
    if (rc == GOL_OK) rc = flush_counts(e);
    if (rc != GOL_OK && e->pend_n) {  // (arrays of points never reduced: zeroed before the next use)
        e->pend_n = 0;
        for (auto &s : e->sh) s.batch_zero = false;
    }
    if (rc == GOL_OK) rc = timing_end(e);
    else e->tcall_ev.clear();  // (a failed call is not timed: the timing queries stay usable)
    if (rc != GOL_OK) {
        (void)sync_all(e);
        return rc;
    }
    if (n == 0) return sync_all(e);
    return collect_counts(e, n, counts);
}

extern "C" int gol_engine_turn(gol_engine *e, int64_t *turn)
{
    if (!e || !turn) return gol_set_error(GOL_EINVAL, "bad arguments");
    *turn = e->turn;
    return GOL_OK;
}

extern "C" int gol_engine_alive_count(gol_engine *e, uint64_t *count)
{
    if (!e || !count) return gol_set_error(GOL_EINVAL, "bad arguments");
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        RCCHK(ensure_counts(s, 1));
    }
    RCCHK(count_into_slots(e));
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        HIPCHK(golk_slots_reduce(s.slots, 1, s.counts, s.stream));
        s.slots_zero = true;
    }
    return collect_counts(e, 1, count);
}

extern "C" int gol_engine_hash(gol_engine *e, uint64_t *hash)
{
    if (!e || !hash) return gol_set_error(GOL_EINVAL, "bad arguments");
    if (!e->bit_capable) return gol_set_error(GOL_EINVAL, "hash needs a bit board (W %% 64 == 0, layout not BYTES)");
    RCCHK(ensure_standard(e));
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        RCCHK(ensure_counts(s, 1));
        if (!s.slots_zero) HIPCHK(hipMemsetAsync(s.slots, 0, SLOT_BYTES, s.stream));
        s.slots_zero = false;
        const uint32_t *bits = s.bits[e->cur];
        if (e->mode == GOL_MODE_EXACT) {  // loaded non-binary bytes at turn 0: hash the 255-cells
            HIPCHK(golk_pack(s.bytes[0] + e->bstride, s.R, e->W, e->bstride, s.bits[0], e->pitch, nullptr, s.stream));
            bits = s.bits[0];
        }
        HIPCHK(golk_hash(bits, s.R, s.y0, e->Wd, e->pitch, s.slots, s.stream));
        HIPCHK(golk_slots_reduce(s.slots, 1, s.counts, s.stream));
        s.slots_zero = true;
    }
    return collect_counts(e, 1, hash);
}

// ------------------------------------------------------------------ load
// Rows [y, y+n) of shard s (global rows) from host rows `src` (pitch `stride`) into the bit
// board, through the staging buffer; ORs a nonbinary flag into s.flag.
static int pack_rows_from_host(gol_engine *e, gol_shard &s, int64_t y, int64_t n, const uint8_t *src, int64_t stride)
{
    HIPCHK(hipMemcpy2DAsync(s.staging, e->bstride, src, stride, e->W, n, hipMemcpyHostToDevice, s.stream));
    HIPCHK(golk_pack(s.staging, n, e->W, e->bstride, s.bits[0] + (y - s.y0) * e->pitch, e->pitch, s.flag, s.stream));
    return GOL_OK;
}

// After the bit rows of every shard were packed with s.flag set on bytes other than 0/255:
// the global decision (every shard, every rank) whether turn 1 must run on the bytes.
static int any_nonbinary(gol_engine *e, bool *out)
{
    uint32_t f = 0;
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        if (several(e)) RCCHK(e->comm->allreduce_max_u32(s.flag, 1, s.stream));
        HIPCHK(hipMemcpyAsync(s.host_word + 1, s.flag, sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
    }
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        HIPCHK(hipStreamSynchronize(s.stream));
        f |= s.host_word[1];
    }
    *out = f != 0;
    return GOL_OK;
}

static int alloc_exact_bytes(gol_engine *e, gol_shard &s)
{
    free_exact_bytes(s);
    HIPCHK(hipMalloc(&s.bytes[0], (s.R + 2) * e->bstride));
    HIPCHK(hipMalloc(&s.bytes[1], s.R * e->bstride));
    return GOL_OK;
}

static int reset_board_state(gol_engine *e)
{
    RCCHK(invalidate_halo(e));
    e->turn = 0;
    e->band = false;
    e->cur = 0;
    e->bcur = 0;
    return GOL_OK;
}

extern "C" int gol_engine_load_bytes(gol_engine *e, const uint8_t *world, int64_t stride)
{
    if (!e || !world || stride < e->W) return gol_set_error(GOL_EINVAL, "bad load arguments");
    RCCHK(reset_board_state(e));
    if (e->mode == GOL_MODE_BYTES || !e->bit_capable) {  // one shard, byte board
        gol_shard &s = e->sh[0];
        RCCHK(set_dev(s.device));
        HIPCHK(hipMemcpy2DAsync(s.bytes[0], e->bstride, world, stride, e->W, e->H, hipMemcpyHostToDevice, s.stream));
        HIPCHK(hipMemsetAsync(s.flag, 0, sizeof(uint32_t), s.stream));
        HIPCHK(golk_nonbinary(s.bytes[0], e->H, e->W, e->bstride, s.flag, s.stream));
        HIPCHK(hipMemcpyAsync(s.host_word + 1, s.flag, sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
        HIPCHK(hipStreamSynchronize(s.stream));
        e->bytes_binary = s.host_word[1] == 0;
        e->mode = GOL_MODE_BYTES;
        return GOL_OK;
    }
    // pack each shard's rows into its bit board, noting bytes other than 0 / 255
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        RCCHK(ensure_staging(e, s));
        HIPCHK(hipMemsetAsync(s.flag, 0, sizeof(uint32_t), s.stream));
        for (int64_t y = s.y0; y < s.y1; y += s.stage_rows) {
            const int64_t n = std::min(s.stage_rows, s.y1 - y);
            RCCHK(pack_rows_from_host(e, s, y, n, world + y * stride, stride));
        }
    }
    bool nonbinary = false;
    RCCHK(any_nonbinary(e, &nonbinary));
    if (!nonbinary) {
        for (auto &s : e->sh) free_exact_bytes(s);
        e->mode = GOL_MODE_BITS;
        return GOL_OK;
    }
    // exact first turn (worker.go:26-37) needs the bytes: every shard keeps rows y0-1 .. y1
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        RCCHK(alloc_exact_bytes(e, s));
        const int64_t above = (s.y0 + e->H - 1) % e->H, below = s.y1 % e->H;
        HIPCHK(hipMemcpyAsync(s.bytes[0], world + above * stride, e->W, hipMemcpyHostToDevice, s.stream));
        HIPCHK(hipMemcpy2DAsync(s.bytes[0] + e->bstride, e->bstride, world + s.y0 * stride, stride, e->W, s.R,
                                hipMemcpyHostToDevice, s.stream));
        HIPCHK(hipMemcpyAsync(s.bytes[0] + (s.R + 1) * e->bstride, world + below * stride, e->W, hipMemcpyHostToDevice,
                              s.stream));
        HIPCHK(hipStreamSynchronize(s.stream));
    }
    e->mode = GOL_MODE_EXACT;
    return GOL_OK;
}

extern "C" int gol_engine_load_random(gol_engine *e, uint64_t seed)
{
    if (!e) return gol_set_error(GOL_EINVAL, "engine is NULL");
    if (e->W % 64 != 0) return gol_set_error(GOL_EINVAL, "random boards need W %% 64 == 0");
    RCCHK(reset_board_state(e));
    if (!e->bit_capable) {  // GOL_LAYOUT_BYTES: the same cells as 0/255 bytes (fill bits, then unpack)
        gol_shard &s = e->sh[0];
        RCCHK(set_dev(s.device));
        uint32_t *bits = nullptr;
        HIPCHK(hipMalloc((void **)&bits, e->H * e->pitch * sizeof(uint32_t)));
        hipError_t err = golk_random_fill(bits, e->H, 0, e->W, e->pitch, seed, s.stream);
        if (err == hipSuccess) err = golk_unpack(bits, e->H, e->W, e->pitch, s.bytes[0], e->bstride, s.stream);
        if (err == hipSuccess) err = hipStreamSynchronize(s.stream);
        const hipError_t ferr = hipFree(bits);
        HIPCHK(err);
        HIPCHK(ferr);
        e->bytes_binary = true;
        e->mode = GOL_MODE_BYTES;
        return GOL_OK;
    }
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        free_exact_bytes(s);
        HIPCHK(golk_random_fill(s.bits[0], s.R, s.y0, e->W, e->pitch, seed, s.stream));
    }
    e->mode = GOL_MODE_BITS;
    return sync_all(e);
}

// readPgmImage header (gol/io.go:97-117): fields = strings.Fields(data): "P5", width, height,
// maxval; the raster is fields[4], i.e. it starts at the first non-space byte after maxval.
static bool is_space(uint8_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
// strconv.Atoi with its error dropped (io.go:104-116 `v, _ := strconv.Atoi(f)`): an optional sign
// and ASCII digits; anything else gives 0, out of range gives the clamped int64.
static int64_t go_atoi(const std::string &f)
{
    size_t i = (!f.empty() && (f[0] == '+' || f[0] == '-')) ? 1 : 0;
    if (i == f.size()) return 0;
    const bool neg = f[0] == '-';
    uint64_t v = 0;
    bool big = false;
    for (size_t j = i; j < f.size(); ++j) {
        if (f[j] < '0' || f[j] > '9') return 0;
        const uint64_t d = (uint64_t)(f[j] - '0');
        if (v > (UINT64_MAX - d) / 10) big = true;
        else v = v * 10 + d;
    }
    if (big || v > (uint64_t)INT64_MAX + (neg ? 1 : 0)) return neg ? INT64_MIN : INT64_MAX;
    return neg ? (int64_t)(0 - v) : (int64_t)v;
}
static int parse_pgm_header(const uint8_t *h, size_t n, int64_t W, int64_t H, int64_t *off)
{
    std::string f[4];
    size_t i = 0;
    int nf = 0;
    while (nf < 4) {
        while (i < n && is_space(h[i])) ++i;
        size_t j = i;
        while (j < n && !is_space(h[j])) ++j;
        if (j == i) break;
        f[nf++] = std::string((const char *)h + i, j - i);
        i = j;
    }
    if (nf < 1 || f[0] != "P5") return gol_set_error(GOL_EFORMAT, "Not a pgm file");
    if (nf < 4) return gol_set_error(GOL_EFORMAT, "Not a pgm file");
    if (go_atoi(f[1]) != W) return gol_set_error(GOL_EFORMAT, "Incorrect width");
    if (go_atoi(f[2]) != H) return gol_set_error(GOL_EFORMAT, "Incorrect height");
    if (go_atoi(f[3]) != 255) return gol_set_error(GOL_EFORMAT, "Incorrect maxval/bit depth");
    while (i < n && is_space(h[i])) ++i;
    if (i >= n) return gol_set_error(GOL_EFORMAT, "no pixel data after the header");
    *off = (int64_t)i;
    return GOL_OK;
}

static int pread_all(int fd, void *buf, size_t n, int64_t off)
{
    uint8_t *p = (uint8_t *)buf;
    while (n > 0) {
        const ssize_t r = pread(fd, p, n, off);
        if (r <= 0) return gol_set_error(GOL_EIO, "short read at offset %lld", (long long)off);
        p += r;
        n -= (size_t)r;
        off += r;
    }
    return GOL_OK;
}

// Stream rows [y, y+n) of the raster (at file offset `data`) through pinned staging.
struct FileRows {
    int fd;
    int64_t data, W;
};

static int load_pgm_impl(gol_engine *e, const FileRows &fr)
{
    RCCHK(reset_board_state(e));
    if (e->mode == GOL_MODE_BYTES || !e->bit_capable) {  // one shard, small byte board
        std::vector<uint8_t> all(e->H * e->W);
        RCCHK(pread_all(fr.fd, all.data(), all.size(), fr.data));
        for (uint8_t c : all)
            if (is_space(c)) return gol_set_error(GOL_EFORMAT, "pixel data shorter than W*H (a whitespace byte ends the field)");
        return gol_engine_load_bytes(e, all.data(), e->W);
    }
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        RCCHK(ensure_staging(e, s));
        HIPCHK(hipMemsetAsync(s.flag, 0, sizeof(uint32_t), s.stream));
        for (int64_t y = s.y0; y < s.y1; y += s.stage_rows) {
            const int64_t n = std::min(s.stage_rows, s.y1 - y);
            HIPCHK(hipStreamSynchronize(s.stream));  // the pinned rows are free again
            RCCHK(pread_all(fr.fd, s.host_staging, (size_t)(n * e->W), fr.data + y * e->W));
            RCCHK(pack_rows_from_host(e, s, y, n, s.host_staging, e->W));
        }
    }
    bool nonbinary = false;
    RCCHK(any_nonbinary(e, &nonbinary));
    if (!nonbinary) {
        e->mode = GOL_MODE_BITS;
        return GOL_OK;
    }
    // bytes other than 0/255: check for whitespace bytes (the reference's strings.Fields
    // split would end the raster there), then keep rows y0-1 .. y1 for the exact first turn
    uint32_t ws = 0;
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        RCCHK(alloc_exact_bytes(e, s));
        for (int64_t i = -1; i < s.R + 1; i += s.stage_rows) {
            const int64_t n = std::min(s.stage_rows, s.R + 1 - i);
            HIPCHK(hipStreamSynchronize(s.stream));
            for (int64_t r = 0; r < n; ++r) {
                const int64_t gy = ((s.y0 + i + r) % e->H + e->H) % e->H;
                uint8_t *row = s.host_staging + r * e->W;
                RCCHK(pread_all(fr.fd, row, (size_t)e->W, fr.data + gy * e->W));
                if (i + r >= 0 && i + r < s.R)
                    for (int64_t x = 0; x < e->W; ++x) ws |= is_space(row[x]);
            }
            HIPCHK(hipMemcpy2DAsync(s.bytes[0] + (i + 1) * e->bstride, e->bstride, s.host_staging, e->W, e->W, n,
                                    hipMemcpyHostToDevice, s.stream));
        }
        HIPCHK(hipStreamSynchronize(s.stream));
    }
    if (several(e)) {  // agree on the verdict
        gol_shard &s = e->sh[0];
        s.host_word[2] = ws;
        HIPCHK(hipMemcpyAsync(s.flag, s.host_word + 2, sizeof(uint32_t), hipMemcpyHostToDevice, s.stream));
        RCCHK(e->comm->allreduce_max_u32(s.flag, 1, s.stream));
        HIPCHK(hipMemcpyAsync(s.host_word + 2, s.flag, sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
        HIPCHK(hipStreamSynchronize(s.stream));
        ws = s.host_word[2];
    }
    if (ws) {
        for (auto &s : e->sh) free_exact_bytes(s);
        return gol_set_error(GOL_EFORMAT, "pixel data shorter than W*H (a whitespace byte ends the field)");
    }
    e->mode = GOL_MODE_EXACT;
    return GOL_OK;
}

extern "C" int gol_engine_load_pgm(gol_engine *e, const char *path)
{
    if (!e || !path) return gol_set_error(GOL_EINVAL, "bad arguments");
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return gol_set_error(GOL_EIO, "cannot open %s", path);
    uint8_t head[4096];
    const ssize_t got = pread(fd, head, sizeof head, 0);
    struct stat st;
    int64_t off = 0;
    int rc = got > 0 ? parse_pgm_header(head, (size_t)got, e->W, e->H, &off) : gol_set_error(GOL_EFORMAT, "Not a pgm file");
    if (rc == GOL_OK && (fstat(fd, &st) != 0 || st.st_size < off + e->H * e->W))
        rc = gol_set_error(GOL_EFORMAT, "pixel data shorter than W*H");
    if (rc == GOL_OK) rc = load_pgm_impl(e, FileRows{fd, off, e->W});
    close(fd);
    return rc;
}

// ------------------------------------------------------------------ store / list / PGM
// Rows [a, b) (global) of shard s as bytes into host `out` (pitch stride), chunked.
static int shard_rows_to_host(gol_engine *e, gol_shard &s, int64_t a, int64_t b, uint8_t *out, int64_t stride)
{
    RCCHK(set_dev(s.device));
    if (e->mode == GOL_MODE_BYTES) {
        HIPCHK(hipMemcpy2DAsync(out, stride, s.bytes[e->bcur] + a * e->bstride, e->bstride, e->W, b - a,
                                hipMemcpyDeviceToHost, s.stream));
    } else if (e->mode == GOL_MODE_EXACT) {
        HIPCHK(hipMemcpy2DAsync(out, stride, s.bytes[0] + (1 + a - s.y0) * e->bstride, e->bstride, e->W, b - a,
                                hipMemcpyDeviceToHost, s.stream));
    } else {
        RCCHK(ensure_staging(e, s));
        for (int64_t y = a; y < b; y += s.stage_rows) {
            const int64_t n = std::min(s.stage_rows, b - y);
            HIPCHK(golk_unpack(s.bits[e->cur] + (y - s.y0) * e->pitch, n, e->W, e->pitch, s.staging, e->bstride, s.stream));
            HIPCHK(hipMemcpy2DAsync(out + (y - a) * stride, stride, s.staging, e->bstride, e->W, n, hipMemcpyDeviceToHost,
                                    s.stream));
        }
    }
    HIPCHK(hipStreamSynchronize(s.stream));
    return GOL_OK;
}

extern "C" int gol_engine_store_rows(gol_engine *e, int64_t y0, int64_t y1, uint8_t *out, int64_t stride)
{
    if (!e || !out || stride < e->W || y0 < 0 || y1 > e->H || y0 > y1) return gol_set_error(GOL_EINVAL, "bad store arguments");
    if (y0 < e->sh.front().y0 || y1 > e->sh.back().y1)
        return gol_set_error(GOL_EINVAL, "rows [%lld, %lld) are not held by this process (rows [%lld, %lld))", (long long)y0,
                             (long long)y1, (long long)e->sh.front().y0, (long long)e->sh.back().y1);
    RCCHK(ensure_standard(e));
    for (auto &s : e->sh) {
        const int64_t a = std::max(y0, s.y0), b = std::min(y1, s.y1);
        if (a < b) RCCHK(shard_rows_to_host(e, s, a, b, out + (a - y0) * stride, stride));
    }
    return GOL_OK;
}

extern "C" int gol_engine_store_bytes(gol_engine *e, uint8_t *out, int64_t stride)
{
    if (!e) return gol_set_error(GOL_EINVAL, "engine is NULL");
    return gol_engine_store_rows(e, 0, e->H, out, stride);
}

// Row-major (x, y) list of the cells of rows [0, rows) of `board` (global row gy0) that are
// alive (prev == NULL) or whose alive state differs from `prev`: per-row counts -> host
// exclusive scan -> one wave per row.  Writes min(total, cap) pairs, *n = total.
static int list_cells(gol_engine *e, gol_shard &s, bool bm, const void *board, const void *prev, int64_t rows,
                      int64_t units, int64_t pitch, int64_t gy0, int32_t *xy, int64_t cap, int64_t *n)
{
    RCCHK(set_dev(s.device));
    int64_t *dcounts = nullptr;
    int32_t *dxy = nullptr;
    std::vector<int64_t> counts(std::max<int64_t>(rows, 1));
    HIPCHK(hipMalloc(&dcounts, counts.size() * sizeof(int64_t)));
    hipError_t he = golk_row_counts(bm, board, prev, rows, units, pitch, dcounts, s.stream);
    if (he == hipSuccess)
        he = hipMemcpyAsync(counts.data(), dcounts, rows * sizeof(int64_t), hipMemcpyDeviceToHost, s.stream);
    if (he == hipSuccess) he = hipStreamSynchronize(s.stream);
    int64_t total = 0;
    if (he == hipSuccess) {
        for (int64_t y = 0; y < rows; ++y) {  // exclusive prefix -> first index of each row
            const int64_t v = counts[y];
            counts[y] = total;
            total += v;
        }
        *n = total;
    }
    const int64_t m = std::min(total, cap);
    if (he == hipSuccess && m > 0) {
        he = hipMemcpyAsync(dcounts, counts.data(), rows * sizeof(int64_t), hipMemcpyHostToDevice, s.stream);
        if (he == hipSuccess) he = hipMalloc(&dxy, m * 2 * sizeof(int32_t));
        if (he == hipSuccess) he = golk_alive_list(bm, board, prev, rows, units, pitch, dcounts, dxy, m, gy0, s.stream);
        if (he == hipSuccess) he = hipMemcpyAsync(xy, dxy, m * 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s.stream);
        if (he == hipSuccess) he = hipStreamSynchronize(s.stream);
    }
    (void)hipFree(dcounts);
    if (dxy) (void)hipFree(dxy);
    if (he != hipSuccess) return gol_set_error(GOL_EHIP, "cell list: %s", hipGetErrorString(he));
    return GOL_OK;
}

extern "C" int gol_engine_alive_cells(gol_engine *e, int32_t *xy, int64_t cap, int64_t *n)
{
    if (!e || !n || cap < 0 || (cap > 0 && !xy)) return gol_set_error(GOL_EINVAL, "bad arguments");
    RCCHK(ensure_standard(e));
    int64_t total = 0;
    for (auto &s : e->sh) {
        int64_t got = 0;
        const int64_t room = std::max<int64_t>(0, cap - total);
        int32_t *dst = room > 0 ? xy + 2 * total : nullptr;
        if (e->mode == GOL_MODE_BITS)
            RCCHK(list_cells(e, s, true, s.bits[e->cur], nullptr, s.R, e->Wd, e->pitch, s.y0, dst, room, &got));
        else if (e->mode == GOL_MODE_EXACT)
            RCCHK(list_cells(e, s, false, s.bytes[0] + e->bstride, nullptr, s.R, e->W, e->bstride, s.y0, dst, room, &got));
        else
            RCCHK(list_cells(e, s, false, s.bytes[e->bcur], nullptr, e->H, e->W, e->bstride, 0, dst, room, &got));
        total += got;
    }
    *n = total;
    return GOL_OK;
}

extern "C" int gol_engine_step_flips(gol_engine *e, int32_t *xy, int64_t cap, int64_t *n)
{
    if (!e || !n || cap < 0 || (cap > 0 && !xy)) return gol_set_error(GOL_EINVAL, "bad arguments");
    RCCHK(agree_step_state(e));
    RCCHK(ensure_standard(e));
    int64_t total = 0;
    if (e->mode == GOL_MODE_BITS) {
        // one standard-layout turn; the previous generation stays in the other buffer
        RCCHK(launch_k(e, 1, -1));
        e->turn += 1;
        RCCHK(sync_all(e));
        for (auto &s : e->sh) {
            int64_t got = 0;
            const int64_t room = std::max<int64_t>(0, cap - total);
            RCCHK(list_cells(e, s, true, s.bits[e->cur], s.bits[1 - e->cur], s.R, e->Wd, e->pitch, s.y0,
                             room > 0 ? xy + 2 * total : nullptr, room, &got));
            total += got;
        }
        *n = total;
        return GOL_OK;
    }
    if (e->mode == GOL_MODE_EXACT) {
        // turn 1 from the loaded bytes: compare the new state (unpacked) with the loaded bytes
        RCCHK(exact_turn(e));
        e->turn += 1;
        for (auto &s : e->sh) {
            RCCHK(set_dev(s.device));
            HIPCHK(golk_unpack(s.bits[e->cur], s.R, e->W, e->pitch, s.bytes[1], e->bstride, s.stream));
        }
        for (auto &s : e->sh) {
            int64_t got = 0;
            const int64_t room = std::max<int64_t>(0, cap - total);
            RCCHK(list_cells(e, s, false, s.bytes[1], s.bytes[0] + e->bstride, s.R, e->W, e->bstride, s.y0,
                             room > 0 ? xy + 2 * total : nullptr, room, &got));
            total += got;
        }
        *n = total;
        return sync_all(e);  // frees the byte rows
    }
    // byte board (W % 64 != 0): one shard; the previous bytes stay in the other buffer
    RCCHK(advance(e, 1, -1));
    RCCHK(sync_all(e));
    gol_shard &s = e->sh[0];
    RCCHK(list_cells(e, s, false, s.bytes[e->bcur], s.bytes[1 - e->bcur], e->H, e->W, e->bstride, 0, xy, cap, &total));
    *n = total;
    return GOL_OK;
}

// writePgmImage's byte stream (gol/io.go:52-81): the header (rank 0) and this process's rows at
// their file offsets, chunk by chunk (device unpack -> pinned staging), into `sink`.
static int pgm_stream(gol_engine *e, gol_write_fn sink, void *user, int64_t *hlen_out)
{
    RCCHK(ensure_standard(e));
    char header[96];
    const int hlen = snprintf(header, sizeof header, "P5\n%lld %lld\n255\n", (long long)e->W, (long long)e->H);  // io.go:52-59
    *hlen_out = hlen;
    const bool coll = several(e);
    if (!coll || e->rank == 0) {
        if (sink(user, 0, (const uint8_t *)header, hlen) != 0) return gol_set_error(GOL_EIO, "the PGM sink failed (header)");
    }
    for (auto &s : e->sh) {
        RCCHK(set_dev(s.device));
        RCCHK(ensure_staging(e, s));
        const int64_t r0 = e->mode == GOL_MODE_BYTES ? 0 : s.y0, r1 = e->mode == GOL_MODE_BYTES ? e->H : s.y1;
        if (e->mode != GOL_MODE_BITS || s.stage_rows < 2) {
            for (int64_t y = r0; y < r1; y += s.stage_rows) {
                const int64_t n = std::min(s.stage_rows, r1 - y);
                RCCHK(shard_rows_to_host(e, s, y, y + n, s.host_staging, e->W));
                if (sink(user, hlen + y * e->W, s.host_staging, n * e->W) != 0)
                    return gol_set_error(GOL_EIO, "the PGM sink failed at row %lld", (long long)y);
            }
            continue;
        }
        // bit board: two halves of the staging buffers; chunk i+1 is unpacked and copied to the
        // host while the sink consumes chunk i
        const int64_t half = s.stage_rows / 2;
        hipEvent_t done[2] = {nullptr, nullptr};
        int rc = GOL_OK;
        for (auto &d : done)
            if (rc == GOL_OK && hipEventCreateWithFlags(&d, hipEventDisableTiming) != hipSuccess)
                rc = gol_set_error(GOL_EHIP, "event for the PGM stream");
        auto enqueue = [&](int64_t y, int h) -> int {
            const int64_t n = std::min(half, r1 - y);
            uint8_t *dst = s.staging + h * half * e->bstride;
            HIPCHK(golk_unpack(s.bits[e->cur] + (y - s.y0) * e->pitch, n, e->W, e->pitch, dst, e->bstride, s.stream));
            HIPCHK(hipMemcpy2DAsync(s.host_staging + h * half * e->W, e->W, dst, e->bstride, e->W, n, hipMemcpyDeviceToHost,
                                    s.stream));
            HIPCHK(hipEventRecord(done[h], s.stream));
            return GOL_OK;
        };
        if (rc == GOL_OK) rc = enqueue(r0, 0);
        for (int64_t y = r0, i = 0; y < r1 && rc == GOL_OK; y += half, ++i) {
            const int h = (int)(i & 1);
            if (y + half < r1) rc = enqueue(y + half, 1 - h);  // the other half's sink call has returned
            if (rc == GOL_OK && hipEventSynchronize(done[h]) != hipSuccess) rc = gol_set_error(GOL_EHIP, "PGM stream copy");
            if (rc == GOL_OK && sink(user, hlen + y * e->W, s.host_staging + h * half * e->W, std::min(half, r1 - y) * e->W) != 0)
                rc = gol_set_error(GOL_EIO, "the PGM sink failed at row %lld", (long long)y);
        }
        (void)hipStreamSynchronize(s.stream);
        for (auto d : done)
            if (d) (void)hipEventDestroy(d);
        RCCHK(rc);
    }
    return GOL_OK;
}

struct FdSink {
    int fd;
};
static int fd_sink(void *user, int64_t off, const uint8_t *data, int64_t len)
{
    const int fd = static_cast<FdSink *>(user)->fd;
    while (len > 0) {
        const ssize_t w = pwrite(fd, data, (size_t)len, off);
        if (w <= 0) return -1;
        data += w;
        len -= w;
        off += w;
    }
    return 0;
}

extern "C" int gol_engine_write_pgm_to(gol_engine *e, gol_write_fn sink, void *user)
{
    if (!e || !sink) return gol_set_error(GOL_EINVAL, "bad arguments");
    int64_t hlen = 0;
    int rc = pgm_stream(e, sink, user, &hlen);
    if (e->rank_mode && e->nranks > 1) {
        const int rb = rank_barrier(e);  // every rank's rows are in its sink when any rank returns
        if (rc == GOL_OK) rc = rb;
    }
    return rc;
}

extern "C" int gol_engine_write_pgm(gol_engine *e, const char *path)
{
    if (!e || !path) return gol_set_error(GOL_EINVAL, "bad arguments");
    const bool coll = several(e);
    int rc = GOL_OK;
    if (!coll || e->rank == 0) {
        char header[96];
        const int hlen = snprintf(header, sizeof header, "P5\n%lld %lld\n255\n", (long long)e->W, (long long)e->H);
        const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd < 0) rc = gol_set_error(GOL_EIO, "cannot create %s", path);
        else {
            if (ftruncate(fd, hlen + e->H * e->W) != 0) rc = gol_set_error(GOL_EIO, "cannot size %s", path);
            if (close(fd) != 0 && rc == GOL_OK) rc = gol_set_error(GOL_EIO, "close %s", path);
        }
    }
    if (coll) {
        const int rb = rank_barrier(e);  // the file exists and is sized before any rank writes
        if (rc == GOL_OK) rc = rb;
    }
    FdSink fs{rc == GOL_OK ? open(path, O_WRONLY) : -1};
    if (rc == GOL_OK && fs.fd < 0) rc = gol_set_error(GOL_EIO, "cannot open %s", path);
    int64_t hlen = 0;
    if (rc == GOL_OK) {
        rc = pgm_stream(e, fd_sink, &fs, &hlen);
        if (rc == GOL_EIO) gol_set_error(GOL_EIO, "short write to %s", path);
    }
    if (fs.fd >= 0 && close(fs.fd) != 0 && rc == GOL_OK) rc = gol_set_error(GOL_EIO, "close %s", path);
    if (coll) {
        const int rb = rank_barrier(e);  // every rank's rows are written when any rank returns
        if (rc == GOL_OK) rc = rb;
    }
    return rc;
}

// ------------------------------------------------------------------ bit-packed rows in / out
static int rows_check(gol_engine *e, int64_t y0, int64_t y1, const void *p, int64_t stride)
{
    if (!e || !p || y0 < 0 || y1 > e->H || y0 > y1 || stride < e->W / 64)
        return gol_set_error(GOL_EINVAL, "bad word-row arguments");
    if (!e->bit_capable) return gol_set_error(GOL_EINVAL, "bit-packed rows need a bit board (W %% 64 == 0, layout not BYTES)");
    if (y0 < e->sh.front().y0 || y1 > e->sh.back().y1)
        return gol_set_error(GOL_EINVAL, "rows [%lld, %lld) are not held by this process", (long long)y0, (long long)y1);
    return GOL_OK;
}

extern "C" int gol_engine_load_words(gol_engine *e, int64_t y0, int64_t y1, const uint64_t *words, int64_t stride)
{
    RCCHK(rows_check(e, y0, y1, words, stride));
    if (e->mode == GOL_MODE_EXACT) {  // the loaded bytes' turn 1 is void now: bits[0] holds their 255-cells
        for (auto &s : e->sh) free_exact_bytes(s);
        e->mode = GOL_MODE_BITS;
    }
    RCCHK(ensure_standard(e));
    RCCHK(invalidate_halo(e));
    e->turn = 0;
    for (auto &s : e->sh) {
        const int64_t a = std::max(y0, s.y0), b = std::min(y1, s.y1);
        if (a >= b) continue;
        RCCHK(set_dev(s.device));
        HIPCHK(hipMemcpy2DAsync(s.bits[e->cur] + (a - s.y0) * e->pitch, e->pitch * sizeof(uint32_t), words + (a - y0) * stride,
                                stride * sizeof(uint64_t), e->W / 8, b - a, hipMemcpyHostToDevice, s.stream));
        HIPCHK(hipStreamSynchronize(s.stream));  // the caller's buffer is only borrowed
    }
    return GOL_OK;
}

extern "C" int gol_engine_store_words(gol_engine *e, int64_t y0, int64_t y1, uint64_t *words, int64_t stride)
{
    RCCHK(rows_check(e, y0, y1, words, stride));
    if (e->mode == GOL_MODE_EXACT)
        return gol_set_error(GOL_ESTATE, "the board holds bytes other than 0/255 until turn 1: use store_bytes");
    RCCHK(ensure_standard(e));
    for (auto &s : e->sh) {
        const int64_t a = std::max(y0, s.y0), b = std::min(y1, s.y1);
        if (a >= b) continue;
        RCCHK(set_dev(s.device));
        HIPCHK(hipMemcpy2DAsync(words + (a - y0) * stride, stride * sizeof(uint64_t), s.bits[e->cur] + (a - s.y0) * e->pitch,
                                e->pitch * sizeof(uint32_t), e->W / 8, b - a, hipMemcpyDeviceToHost, s.stream));
        HIPCHK(hipStreamSynchronize(s.stream));
    }
    return GOL_OK;
}

// ------------------------------------------------------------------ info
extern "C" int gol_engine_info(gol_engine *e, int32_t *k, int32_t *cells_per_lane, int32_t *strip_rows,
                               int32_t *bit_mode)
{
    if (!e) return gol_set_error(GOL_EINVAL, "engine is NULL");
    const bool bits = e->mode == GOL_MODE_BITS;
    const bool band = bits && e->band_capable;
    const int dw = band ? e->band_dw : e->dw;
    // the k of the next launch, as advance() picks it
    int kk = 1;  // the exact one-turn kernel: a board before its exact first turn, a byte board of W % 32 != 0 or non-0/255 bytes
    if (bits) kk = pick_k(e->k, e->k, e->min_rows, dw, band);
    else if (e->mode == GOL_MODE_BYTES && e->bytes_binary && e->W % 32 == 0)
        kk = e->k >= 32 && e->H >= 32 ? 32 : pick_k(e->k, e->k, e->H, 1, false);
    if (k) *k = kk;
    if (cells_per_lane) *cells_per_lane = 32 * dw;
    if (strip_rows) {
        const int64_t u = band ? golk_band_useful_words(kk, dw) : 62 * dw;
        const int64_t ng = (e->Wd + u - 1) / u;
        *strip_rows = e->strip > 0 ? e->strip : golk_auto_strip(e->min_rows, ng, kk);
    }
    if (bit_mode) *bit_mode = bits ? (band ? 2 : 1) : 0;
    return GOL_OK;
}

extern "C" int gol_engine_device_bits(gol_engine *e, uint32_t **bits, int64_t *pitch)
{
    if (!e || !bits || !pitch) return gol_set_error(GOL_EINVAL, "bad arguments");
    if (e->mode != GOL_MODE_BITS) return gol_set_error(GOL_ESTATE, "board is not bit-resident");
    RCCHK(ensure_standard(e));
    RCCHK(sync_all(e, false));
    *bits = e->sh[0].bits[e->cur];
    *pitch = e->pitch;
    return GOL_OK;
}

extern "C" int gol_engine_set_timing(gol_engine *e, int32_t enable)
{
    if (!e) return gol_set_error(GOL_EINVAL, "engine is NULL");
    for (auto &s : e->sh) {  // events of earlier steps may still be pending
        RCCHK(set_dev(s.device));
        HIPCHK(hipStreamSynchronize(s.stream));
    }
    e->timing = enable != 0;
    e->timing_x = enable == GOL_TIMING_EXCHANGE;
    e->timed.clear();
    for (auto &s : e->sh) s.tused = 0;
    e->t_ms = e->t_cells = 0;
    e->t_n = 0;
    e->x_ms = e->x_wait_ms = 0;
    e->x_n = 0;
    return GOL_OK;
}

// Local, like gol_engine_timing.
extern "C" int gol_engine_exchange_timing(gol_engine *e, int64_t *exchanges, double *mean_ms)
{
    if (!e || !exchanges || !mean_ms) return gol_set_error(GOL_EINVAL, "bad arguments");
    if (timing_open(e)) return gol_set_error(GOL_ESTATE, "a timed stepping call is in progress");
    RCCHK(fold_timing(e));
    *exchanges = e->x_n;
    *mean_ms = e->x_n ? e->x_ms / e->x_n : 0.0;
    return GOL_OK;
}

extern "C" int gol_engine_exchange_split(gol_engine *e, int64_t *exchanges, double *mean_wait_ms, double *mean_transfer_ms)
{
    if (!e || !exchanges || !mean_wait_ms || !mean_transfer_ms) return gol_set_error(GOL_EINVAL, "bad arguments");
    if (timing_open(e)) return gol_set_error(GOL_ESTATE, "a timed stepping call is in progress");
    RCCHK(fold_timing(e));
    *exchanges = e->x_n;
    *mean_wait_ms = e->x_n ? e->x_wait_ms / e->x_n : 0.0;
    *mean_transfer_ms = e->x_n ? (e->x_ms - e->x_wait_ms) / e->x_n : 0.0;
    return GOL_OK;
}

// Local (not collective): waits only for this process's timed steps.
extern "C" int gol_engine_timing(gol_engine *e, int64_t *launches, double *mean_ms, double *mean_cell_updates)
{
    if (!e || !launches || !mean_ms || !mean_cell_updates) return gol_set_error(GOL_EINVAL, "bad arguments");
    if (timing_open(e)) return gol_set_error(GOL_ESTATE, "a timed stepping call is in progress");
    RCCHK(fold_timing(e));
    const int64_t n = e->t_n;
    *launches = n;
    *mean_ms = n ? e->t_ms / n : 0.0;
    *mean_cell_updates = n ? e->t_cells / n : 0.0;
    return GOL_OK;
}
