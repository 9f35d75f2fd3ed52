// gol_comm.h -- collectives and the IPC halo transport of a several-process engine (private).
//
// gol_engine_create_rank builds one of two transports (include/golhip.h):
//  * RCCL (production, one process per GPU): the halo rows travel by ncclSend/ncclRecv in
//    gol_engine.cpp's exchange(), the collectives below are ncclAllReduce on the shard's stream;
//  * IPC (ranks of one node, possibly sharing a GPU): each rank maps its ring neighbours' two
//    bit buffers and their flag words through HIP IPC handles and pulls its ghost rows out of
//    their HBM; the collectives run on the host through a POSIX shared-memory segment.
// Every whole-board collective of the engine (error words in sync_all, counted-step series,
// the nonbinary and whitespace verdicts of a load, the PGM barriers, the step-state agreement)
// goes through gol_comm, so both transports run the same call sequence.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <vector>

struct gol_comm {
    virtual ~gol_comm() = default;
    // max / sum over the ranks of n words of device memory, in place, ordered on `st` after the
    // stream's earlier work (the result is ready for the stream's later work)
    virtual int allreduce_max_u32(uint32_t *dev, int64_t n, hipStream_t st) = 0;
    virtual int allreduce_sum_u64(uint64_t *dev, int64_t n, hipStream_t st) = 0;
    // returns when every rank's work on its `st` up to this call is done (scratch: 1 device word)
    virtual int barrier(uint32_t *scratch, hipStream_t st) = 0;
};

// RCCL collectives over an existing communicator (not owned: the shard destroys it).
gol_comm *gol_comm_rccl(ncclComm_t c);

// Flag words of an IPC rank (its own device memory, read by its neighbours through IPC):
// READY = the last exchange whose send rows this rank has written into its send buffer (its
// peers may pull them).  A sequence number, compared wrap-safe.  (Until round 5 a PULLED word
// also ordered board writes behind the peers' pulls; since the peers read only the send buffer,
// that order is implied by READY, gol_engine.cpp exchange_ipc.)
enum { GOL_IPC_READY = 0, GOL_IPC_FLAG_WORDS = 16 };

struct gol_ipc_seg;

class gol_ipc final : public gol_comm {
public:
    // Join the ranks named by `id` (gol_ipc_unique_id): publish this rank's exported allocations
    // (bufs: the engine passes its halo send buffer; nullptr entries are skipped) and flag words,
    // wait until all nranks have joined, map the buffers of `peers` (global ranks, this one
    // excluded).  Collective; every rank must pass the same (nranks, H, W, kx).  A rank whose
    // join fails marks the segment aborted, so the others fail at their next barrier instead of
    // waiting out GOL_IPC_TIMEOUT_MS.
    static int open(const uint8_t *id, int nranks, int rank, int device, int64_t H, int64_t W, int kx, uint32_t *const bufs[2],
                    const std::vector<int> &peers, gol_ipc **out);
    ~gol_ipc() override;

    int allreduce_max_u32(uint32_t *dev, int64_t n, hipStream_t st) override;
    int allreduce_sum_u64(uint64_t *dev, int64_t n, hipStream_t st) override;
    int barrier(uint32_t *scratch, hipStream_t st) override;

    // Peer `rank`'s bit allocation i mapped into this process (nullptr: not a mapped peer).
    uint32_t *peer_buf(int rank, int i) const;
    // Enqueue on st: set this rank's flag `which` to seq (after the stream's earlier work).
    int signal(hipStream_t st, int which, uint32_t seq);
    // Enqueue on st: wait until flag `which` of every rank in `ranks` has reached seq; a wait
    // that times out ORs GOLK_ERR_IPC into err and lets the stream go on.
    int wait(hipStream_t st, const std::vector<int> &ranks, int which, uint32_t seq, uint32_t *err);

private:
    gol_ipc() = default;
    int host_barrier();
    template <typename T, typename Op>
    int allreduce(T *dev, int64_t n, hipStream_t st, Op op);

    gol_ipc_seg *seg_ = nullptr;
    int nranks_ = 0, rank_ = 0, device_ = 0;
    uint32_t *flags_ = nullptr;  // this rank's GOL_IPC_FLAG_WORDS (device)
    struct Peer {
        int rank = -1;
        uint32_t *buf[2] = {nullptr, nullptr};
        uint32_t *flags = nullptr;
    };
    std::vector<Peer> peers_;
    int64_t timeout_ms_ = 0;
};
