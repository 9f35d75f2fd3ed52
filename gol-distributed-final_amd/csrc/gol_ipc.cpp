// gol_ipc.cpp -- the IPC transport of the rank engine (gol_comm.h) and the RCCL collectives.
//
// The reference's broker ships the whole board to every worker process each turn over TCP
// (broker.go:143-157, 182-206).  The rank engine keeps each rank's rows resident on its GPU and
// moves only k halo rows per k turns.  Between the processes of one node this transport moves
// them without RCCL: every rank exports a small halo send buffer and a few flag words with
// hipIpcGetMemHandle, its ring neighbours map them, and each rank copies its own ghost rows out
// of its neighbours' HBM (a pull, device to device; the same GPU when ranks share one).  The
// order between processes is carried by sequence numbers in those flag words, stored and polled
// by one-wave kernels on the streams (gol_kernels.hip ipc_*_kernel), never by the host.  The
// small collectives (error words, counts, verdicts, barriers) go through a POSIX shared-memory
// segment named by the caller's id.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/random.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gol_comm.h"
#include "gol_internal.h"
#include "gol_kernels.h"

// ------------------------------------------------------------------ RCCL
namespace {
struct RcclComm final : gol_comm {
    ncclComm_t c;
    explicit RcclComm(ncclComm_t cc) : c(cc) {}
    int rc(ncclResult_t r, const char *what)
    {
        return r == ncclSuccess ? GOL_OK : gol_set_error(GOL_ECOMM, "%s: %s", what, ncclGetErrorString(r));
    }
    int allreduce_max_u32(uint32_t *dev, int64_t n, hipStream_t st) override
    {
        return rc(ncclAllReduce(dev, dev, (size_t)n, ncclUint32, ncclMax, c, st), "ncclAllReduce(max)");
    }
    int allreduce_sum_u64(uint64_t *dev, int64_t n, hipStream_t st) override
    {
        return rc(ncclAllReduce(dev, dev, (size_t)n, ncclUint64, ncclSum, c, st), "ncclAllReduce(sum)");
    }
    int barrier(uint32_t *scratch, hipStream_t st) override
    {
        const int r = allreduce_max_u32(scratch, 1, st);
        if (r) return r;
        const hipError_t e = hipStreamSynchronize(st);
        return e == hipSuccess ? GOL_OK : gol_set_error(GOL_EHIP, "barrier: %s", hipGetErrorString(e));
    }
};
}  // namespace

gol_comm *gol_comm_rccl(ncclComm_t c) { return new RcclComm(c); }

// ------------------------------------------------------------------ the shared segment
static constexpr char IPC_MAGIC[8] = {'G', 'O', 'L', 'I', 'P', 'C', '1', 0};
static constexpr int64_t IPC_REDUCE_WORDS = 4096;  // uint64 per rank per all-reduce round

struct gol_ipc_slot {
    std::atomic<uint32_t> claimed;    // a process has joined as this rank
    std::atomic<uint32_t> published;  // its handles below are valid
    int32_t pid, device;
    hipIpcMemHandle_t buf[2];
    hipIpcMemHandle_t flags;
    uint64_t data[IPC_REDUCE_WORDS];  // this rank's contribution to the current all-reduce round
};

struct gol_ipc_seg {
    std::atomic<uint64_t> key;       // (nranks, H, W) of the first rank to join; every rank must match
    std::atomic<uint32_t> arrived;   // host barrier: ranks arrived in the current generation
    std::atomic<uint32_t> gen;       // host barrier: generation
    std::atomic<uint32_t> abort;     // a rank gave up (timeout): every later barrier fails at once
    gol_ipc_slot slot[GOL_IPC_MAX_RANKS];
};
static_assert(std::atomic<uint32_t>::is_always_lock_free && std::atomic<uint64_t>::is_always_lock_free,
              "process-shared atomics must be lock-free");

static void seg_name(const uint8_t *id, char (&out)[64])
{
    static const char *hex = "0123456789abcdef";
    char h[33];
    for (int i = 0; i < 16; ++i) {
        h[2 * i] = hex[id[8 + i] >> 4];
        h[2 * i + 1] = hex[id[8 + i] & 15];
    }
    h[32] = 0;
    snprintf(out, sizeof out, "/golhip-ipc-%s", h);
}

extern "C" int gol_ipc_unique_id(uint8_t *id, int64_t len)
{
    if (!id || len < GOL_IPC_ID_BYTES) return gol_set_error(GOL_EINVAL, "id needs %d bytes", GOL_IPC_ID_BYTES);
    memset(id, 0, GOL_IPC_ID_BYTES);
    memcpy(id, IPC_MAGIC, sizeof IPC_MAGIC);
    uint8_t *r = id + 8;
    size_t got = 0;
    while (got < 16) {
        const ssize_t n = getrandom(r + got, 16 - got, 0);
        if (n <= 0) return gol_set_error(GOL_EIO, "getrandom failed");
        got += (size_t)n;
    }
    return GOL_OK;
}

static int64_t ipc_timeout_ms()
{
    // how long a rank waits for the others (host barriers, and on the GPU for a neighbour's flag)
    const char *v = getenv("GOL_IPC_TIMEOUT_MS");
    const long long t = v ? atoll(v) : 0;
    return t > 0 ? (int64_t)t : 120000;
}

// Spin, then yield, then sleep: ranks may outnumber the cores they run on.
static void backoff(int &n)
{
    if (++n < 200) return;
    if (n < 400) {
        sched_yield();
        return;
    }
    const timespec ts{0, 20000};
    nanosleep(&ts, nullptr);
}

int gol_ipc::host_barrier()
{
    gol_ipc_seg *s = seg_;
    if (s->abort.load(std::memory_order_acquire)) return gol_set_error(GOL_ECOMM, "IPC ranks: an earlier collective failed");
    const uint32_t g = s->gen.load(std::memory_order_acquire);
    if (s->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)nranks_) {
        s->arrived.store(0, std::memory_order_relaxed);
        s->gen.store(g + 1, std::memory_order_release);
        return GOL_OK;
    }
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    int n = 0;
    while (s->gen.load(std::memory_order_acquire) == g) {
        if (s->abort.load(std::memory_order_acquire))
            return gol_set_error(GOL_ECOMM, "IPC ranks: another rank gave up waiting");
        if ((n & 255) == 255 && std::chrono::steady_clock::now() > deadline) {
            s->abort.store(1, std::memory_order_release);
            return gol_set_error(GOL_ECOMM, "IPC ranks: rank %d waited %lld ms for the others at a collective", rank_,
                                 (long long)timeout_ms_);
        }
        backoff(n);
    }
    return GOL_OK;
}

template <typename T, typename Op>
int gol_ipc::allreduce(T *dev, int64_t n, hipStream_t st, Op op)
{
    if (n <= 0) return GOL_OK;
    std::vector<T> v((size_t)n);
    hipError_t he = hipStreamSynchronize(st);
    if (he == hipSuccess) he = hipMemcpy(v.data(), dev, (size_t)n * sizeof(T), hipMemcpyDeviceToHost);
    if (he != hipSuccess) return gol_set_error(GOL_EHIP, "IPC all-reduce readback: %s", hipGetErrorString(he));
    const int64_t per = IPC_REDUCE_WORDS * (int64_t)sizeof(uint64_t) / (int64_t)sizeof(T);
    for (int64_t i0 = 0; i0 < n; i0 += per) {
        const int64_t m = std::min(per, n - i0);
        memcpy(seg_->slot[rank_].data, v.data() + i0, (size_t)m * sizeof(T));
        int rc = host_barrier();
        if (rc) return rc;
        for (int r = 0; r < nranks_; ++r) {
            if (r == rank_) continue;
            const T *src = reinterpret_cast<const T *>(seg_->slot[r].data);
            for (int64_t j = 0; j < m; ++j) v[i0 + j] = op(v[i0 + j], src[j]);
        }
        rc = host_barrier();  // every rank has read this round's contributions
        if (rc) return rc;
    }
    he = hipMemcpy(dev, v.data(), (size_t)n * sizeof(T), hipMemcpyHostToDevice);
    return he == hipSuccess ? GOL_OK : gol_set_error(GOL_EHIP, "IPC all-reduce: %s", hipGetErrorString(he));
}

int gol_ipc::allreduce_max_u32(uint32_t *dev, int64_t n, hipStream_t st)
{
    return allreduce(dev, n, st, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
}

int gol_ipc::allreduce_sum_u64(uint64_t *dev, int64_t n, hipStream_t st)
{
    return allreduce(dev, n, st, [](uint64_t a, uint64_t b) { return a + b; });
}

int gol_ipc::barrier(uint32_t *, hipStream_t st)
{
    const hipError_t he = hipStreamSynchronize(st);
    if (he != hipSuccess) return gol_set_error(GOL_EHIP, "barrier: %s", hipGetErrorString(he));
    return host_barrier();
}

uint32_t *gol_ipc::peer_buf(int rank, int i) const
{
    for (const Peer &p : peers_)
        if (p.rank == rank) return p.buf[i];
    return nullptr;
}

int gol_ipc::signal(hipStream_t st, int which, uint32_t seq)
{
    const hipError_t he = golk_ipc_signal(flags_ + which, seq, st);
    return he == hipSuccess ? GOL_OK : gol_set_error(GOL_EHIP, "IPC signal: %s", hipGetErrorString(he));
}

int gol_ipc::wait(hipStream_t st, const std::vector<int> &ranks, int which, uint32_t seq, uint32_t *err)
{
    const uint32_t *f[GOLK_IPC_MAX_WAIT];
    int n = 0;
    for (int r : ranks)
        for (const Peer &p : peers_)
            if (p.rank == r) {
                if (n == GOLK_IPC_MAX_WAIT) return gol_set_error(GOL_EINVAL, "IPC wait: too many ranks");
                f[n++] = p.flags + which;
            }
    if (n == 0) return GOL_OK;
    const uint64_t ticks = (uint64_t)timeout_ms_ * 100000ull;  // s_memrealtime: 100 MHz
    const hipError_t he = golk_ipc_wait(f, n, seq, ticks, err, st);
    return he == hipSuccess ? GOL_OK : gol_set_error(GOL_EHIP, "IPC wait: %s", hipGetErrorString(he));
}

static int hip_fail(hipError_t e, const char *what)
{
    return gol_set_error(e == hipErrorOutOfMemory ? GOL_ENOMEM : GOL_EHIP, "%s: %s", what, hipGetErrorString(e));
}

// GOL_IPC_TRACE=1: every step of the join on stderr (a rank that hangs in the HIP runtime shows
// where: the host collectives time out by themselves, runtime calls do not)
static bool ipc_trace()
{
    static const bool on = getenv("GOL_IPC_TRACE") && atoi(getenv("GOL_IPC_TRACE")) > 0;
    return on;
}
#define IPC_TRACE(...)                                                                                  \
    do {                                                                                                \
        if (ipc_trace()) {                                                                              \
            fprintf(stderr, "[golhip ipc r%d %.3f] ", rank,                                             \
                    std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count()); \
            fprintf(stderr, __VA_ARGS__);                                                               \
            fputc('\n', stderr);                                                                        \
        }                                                                                               \
    } while (0)

// Ranks open their peers' handles one rank at a time (a host barrier between turns): 4 ranks
// importing each other's 2 GiB buffers at once hung inside the runtime (config 4's board over 4
// ranks on one GPU, round 4); 2 ranks and small buffers did not.
#ifndef GOL_IPC_SERIAL_OPEN
#define GOL_IPC_SERIAL_OPEN 1
#endif

int gol_ipc::open(const uint8_t *id, int nranks, int rank, int device, int64_t H, int64_t W, int kx, uint32_t *const bufs[2],
                  const std::vector<int> &peers, gol_ipc **out)
{
    *out = nullptr;
    if (!id || memcmp(id, IPC_MAGIC, sizeof IPC_MAGIC) != 0)
        return gol_set_error(GOL_EINVAL, "not an IPC id (make it with gol_ipc_unique_id)");
    if (nranks < 1 || nranks > GOL_IPC_MAX_RANKS || rank < 0 || rank >= nranks)
        return gol_set_error(GOL_EINVAL, "IPC transport: rank %d of %d (at most %d ranks)", rank, nranks, GOL_IPC_MAX_RANKS);
    char name[64];
    seg_name(id, name);
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) return gol_set_error(GOL_ECOMM, "shm_open(%s) failed", name);
    if (ftruncate(fd, sizeof(gol_ipc_seg)) != 0) {
        close(fd);
        shm_unlink(name);
        return gol_set_error(GOL_ECOMM, "cannot size the IPC segment %s", name);
    }
    void *m = mmap(nullptr, sizeof(gol_ipc_seg), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        shm_unlink(name);
        return gol_set_error(GOL_ECOMM, "cannot map the IPC segment %s", name);
    }
    gol_ipc *c = new gol_ipc();
    c->seg_ = static_cast<gol_ipc_seg *>(m);  // a new segment is zero-filled: every atomic starts at 0
    c->nranks_ = nranks;
    c->rank_ = rank;
    c->device_ = device;
    c->timeout_ms_ = ipc_timeout_ms();
    int rc = GOL_OK;
    gol_ipc_seg *s = c->seg_;
    auto fail = [&](int r) {
        // the other ranks fail at their next host barrier instead of waiting out the timeout (or,
        // past the joins, stalling at their first collective or halo wait)
        s->abort.store(1, std::memory_order_release);
        shm_unlink(name);  // (ENOENT once another rank has removed it)
        delete c;
        return r;
    };
    // every rank of one board agrees on its shape and on kx (the rows per exchange, which fixes
    // the halo plans the ranks pair their sends and receives by)
    const uint64_t key = (((uint64_t)nranks * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)H * 0xBF58476D1CE4E5B9ull) ^
                          ((uint64_t)W * 0x94D049BB133111EBull) ^ ((uint64_t)(uint32_t)kx * 0xD6E8FEB86659FD93ull)) | 1ull;
    uint64_t seen = 0;
    if (!s->key.compare_exchange_strong(seen, key) && seen != key)
        return fail(gol_set_error(GOL_EINVAL, "IPC ranks disagree on the board or the rank count"));
    uint32_t unclaimed = 0;
    if (!s->slot[rank].claimed.compare_exchange_strong(unclaimed, 1u))
        return fail(gol_set_error(GOL_EINVAL, "IPC rank %d joined twice", rank));

    IPC_TRACE("joined the segment %s", name);
    hipError_t he = hipMalloc(&c->flags_, GOL_IPC_FLAG_WORDS * sizeof(uint32_t));
    if (he == hipSuccess) he = hipMemset(c->flags_, 0, GOL_IPC_FLAG_WORDS * sizeof(uint32_t));
    if (he == hipSuccess) he = hipDeviceSynchronize();
    if (he != hipSuccess) return fail(hip_fail(he, "IPC flag words"));
    IPC_TRACE("flag words allocated");
    gol_ipc_slot &me = s->slot[rank];
    me.pid = (int32_t)getpid();
    me.device = device;
    for (int i = 0; i < 2 && he == hipSuccess; ++i)
        if (bufs[i]) he = hipIpcGetMemHandle(&me.buf[i], bufs[i]);
    if (he == hipSuccess) he = hipIpcGetMemHandle(&me.flags, c->flags_);
    if (he != hipSuccess) return fail(hip_fail(he, "hipIpcGetMemHandle"));
    me.published.store(1, std::memory_order_release);
    IPC_TRACE("handles published");

    rc = c->host_barrier();  // every rank has published its handles
    if (rc) return fail(rc);
    if (rank == 0) shm_unlink(name);  // mapped by every rank: the name is no longer needed
    IPC_TRACE("all ranks published");

    auto open_peers = [&]() -> int {
        for (int r : peers) {
            if (r == rank || r < 0 || r >= nranks) continue;
            const gol_ipc_slot &ps = s->slot[r];
            if (!ps.published.load(std::memory_order_acquire)) return gol_set_error(GOL_ECOMM, "IPC rank %d has no handles", r);
            if (ps.device != device) {  // (ranks on distinct GPUs: peer access for the pulls and the flag polls)
                (void)hipDeviceEnablePeerAccess(ps.device, 0);
                (void)hipGetLastError();
            }
            Peer p;
            p.rank = r;
            void *q = nullptr;
            for (int i = 0; i < 2 && he == hipSuccess; ++i) {
                if (!bufs[i]) continue;
                IPC_TRACE("opening rank %d's buffer %d", r, i);
                he = hipIpcOpenMemHandle(&q, ps.buf[i], hipIpcMemLazyEnablePeerAccess);
                if (he == hipSuccess) p.buf[i] = static_cast<uint32_t *>(q);
            }
            IPC_TRACE("opening rank %d's flag words", r);
            if (he == hipSuccess) he = hipIpcOpenMemHandle(&q, ps.flags, hipIpcMemLazyEnablePeerAccess);
            if (he == hipSuccess) p.flags = static_cast<uint32_t *>(q);
            c->peers_.push_back(p);
            if (he != hipSuccess) return hip_fail(he, "hipIpcOpenMemHandle");
        }
        return GOL_OK;
    };
    if (GOL_IPC_SERIAL_OPEN) {
        int orc = GOL_OK;  // (a rank whose opens failed still takes part in every turn's barrier)
        for (int turn = 0; turn < nranks && rc == GOL_OK; ++turn) {
            if (turn == rank) orc = open_peers();
            rc = c->host_barrier();
        }
        if (rc == GOL_OK) rc = orc;
    } else {
        rc = open_peers();
    }
    // every rank learns whether any rank's opens failed: a final barrier after which a failed rank
    // has set abort (fail() below) before any rank returns success
    if (rc) return fail(rc);
    rc = c->host_barrier();
    if (rc == GOL_OK && s->abort.load(std::memory_order_acquire))
        rc = gol_set_error(GOL_ECOMM, "IPC ranks: another rank failed to join");
    if (rc) return fail(rc);
    IPC_TRACE("peers opened");
    *out = c;
    return GOL_OK;
}

gol_ipc::~gol_ipc()
{
    (void)hipSetDevice(device_);
    for (Peer &p : peers_) {
        for (uint32_t *b : p.buf)
            if (b) (void)hipIpcCloseMemHandle(b);
        if (p.flags) (void)hipIpcCloseMemHandle(p.flags);
    }
    if (flags_) (void)hipFree(flags_);
    if (seg_) munmap(seg_, sizeof(gol_ipc_seg));
}
