// gol_host.cpp -- C++ host mirror of the reference's RPC services on top of the
// engine, plus their C ABI wrappers (gol_broker_*, gol_worker_update).
//
// The reference's host side is Go (net/rpc + gob); no Go toolchain exists in
// this image, so the service objects are restated here in C++ with the same
// names, field names and argument meaning:
//   stubs.Request / stubs.Response          stubs.go:20-38
//   util.Cell{X, Y}                          util/cell.go:4-5
//   Operations.{Run, Quit, SuperQuit, Pause, RetrieveCurrentData}   broker.go:62-277
//   GameOfLifeOperations.{Update, WorkerQuit}                      worker.go:77-86
// A Go drop-in registers the same service/method names and
// forwards each call to the C wrappers at the bottom of this file.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <vector>

#include "golhip.h"
#include "gol_internal.h"

namespace util {
struct Cell {  // util/cell.go:4-5
    int64_t X, Y;
};
}  // namespace util

namespace stubs {
struct Request {  // stubs.go:20-29 (World as a borrowed H x W byte view)
    const uint8_t *World = nullptr;
    int64_t WorldStride = 0;
    int64_t Turns = 0, ImageHeight = 0, ImageWidth = 0, Threads = 0, EndY = 0, StartY = 0, Worker = 0;
};
struct Response {  // stubs.go:31-38 (World / WorkSlice / Alive as caller-provided buffers)
    int32_t *Alive = nullptr;
    int64_t AliveCap = 0, AliveLen = 0;
    int64_t AliveCount = 0, TurnsCompleted = 0;
    uint8_t *World = nullptr;
    int64_t WorldStride = 0;
    uint8_t *WorkSlice = nullptr;
    int64_t WorkStride = 0;
    int64_t Worker = 0;
};
}  // namespace stubs

// ------------------------------------------------------------------ worker
// worker.go:73-86.  Stateless: Update computes one turn of rows [StartY, EndY).
struct GameOfLifeOperations {
    int Update(const stubs::Request &req, stubs::Response *res)
    {
        if (!req.World || !res || !res->WorkSlice)
            return gol_set_error(GOL_EINVAL, "Update needs World and a WorkSlice buffer");
        res->Worker = req.Worker;
        return gol_next_state_slab(req.World, req.ImageHeight, req.ImageWidth,
                                   req.WorldStride ? req.WorldStride : req.ImageWidth, req.StartY, req.EndY,
                                   res->WorkSlice, res->WorkStride ? res->WorkStride : req.ImageWidth);
    }
};

// ------------------------------------------------------------------ broker
// broker.go:22-36 globals become members: mt -> mu, cTurn, cWorld (the engine's
// resident board), the unbuffered channels `waiting` / `quitting` / `superQuit`
// become counters consumed by the turn loop between steps.
struct Operations {
    gol_config cfg{};
    std::mutex mu;
    std::condition_variable cv;
    gol_engine *eng = nullptr;
    int64_t H = 0, W = 0;
    int64_t cTurn = 0;
    bool have_world = false;  // cWorld allocated by a Run (broker.go:67-70)
    bool running = false;
    int pending_pause = 0, pending_quit = 0;
    bool paused = false, shut_down = false;
    // Callers other than the turn loop announce themselves here before locking `mu`;
    // the loop yields the lock between chunks while any are waiting, so queries and
    // control calls are served within one chunk (std::mutex alone is not fair).
    std::atomic<int> waiters{0};

    struct Access {  // RAII: announce, lock, and on exit release + wake the turn loop
        Operations &o;
        std::unique_lock<std::mutex> lk;
        explicit Access(Operations &op) : o(op), lk((op.waiters.fetch_add(1), op.mu)) {}
        ~Access()
        {
            o.waiters.fetch_sub(1);
            lk.unlock();
            o.cv.notify_all();
        }
    };

    ~Operations()
    {
        if (eng) gol_engine_destroy(eng);
    }

    // The board of a Run: row-sharded over cfg.shards GPUs (broker.go:135-206's split applied
    // to GPUs) when configured and the board allows it (W % 64 == 0, at least one row per
    // shard), else on one GPU (a byte board, GOL_LAYOUT_BYTES, always: it does not shard).
    int ensure_engine(int64_t h, int64_t w)
    {
        if (eng && H == h && W == w) return GOL_OK;
        if (eng) gol_engine_destroy(eng);
        eng = nullptr;
        H = h;
        W = w;
        gol_config c = cfg;
        if (c.shards > 1 && (w % 64 != 0 || h < c.shards || c.layout == GOL_LAYOUT_BYTES)) c.shards = 1;
        if (c.shards <= 1) c.transport = GOL_TRANSPORT_AUTO;
        return gol_engine_create(h, w, &c, &eng);
    }

    // Turn-loop control point (broker.go:79-88 / 122-130), checked between steps.
    // Returns true when the loop must stop (Quit / SuperQuit).
    bool control(std::unique_lock<std::mutex> &lk)
    {
        if (pending_quit) {
            pending_quit--;
            return true;
        }
        if (pending_pause) {
            pending_pause--;
            paused = true;  // "State paused": block until the second Pause
            cv.wait(lk, [&] { return pending_pause > 0 || pending_quit > 0 || shut_down; });
            if (pending_pause) pending_pause--;
            paused = false;  // "Loop resumed"
            if (pending_quit) {
                pending_quit--;
                return true;
            }
        }
        return shut_down;
    }

    int fill_board(stubs::Response *res)
    {
        int rc = GOL_OK;
        if (res->World) rc = gol_engine_store_bytes(eng, res->World, res->WorldStride ? res->WorldStride : W);
        if (rc == GOL_OK && (res->Alive || res->AliveCap == 0)) {
            int64_t n = 0;
            rc = gol_engine_alive_cells(eng, res->Alive, res->Alive ? res->AliveCap : 0, &n);
            res->AliveLen = n;
        }
        return rc;
    }

    // broker.go:62-234
    int Run(const stubs::Request &req, stubs::Response *res)
    {
        if (!res || !req.World || req.ImageHeight <= 0 || req.ImageWidth <= 0 || req.Turns < 0 || req.Threads < 1)
            return gol_set_error(GOL_EINVAL, "Run needs World, ImageHeight/Width > 0, Turns >= 0, Threads >= 1");
        std::unique_lock<std::mutex> lk(mu);
        if (shut_down) return gol_set_error(GOL_EQUIT, "broker has shut down (SuperQuit)");
        if (running) return gol_set_error(GOL_ESTATE, "a Run is already in progress");
        int rc = ensure_engine(req.ImageHeight, req.ImageWidth);
        if (rc == GOL_OK)
            rc = gol_engine_load_bytes(eng, req.World, req.WorldStride ? req.WorldStride : req.ImageWidth);
        if (rc != GOL_OK) return rc;
        cTurn = 0;  // broker.go:64
        have_world = true;
        running = true;
        // Threads only chose the slab split across workers (broker.go:135-206); results
        // do not depend on it.  Here the board stays resident and is stepped in chunks
        // sized so that Retrieve / Pause / Quit are served within ~10 ms.  The first chunk is
        // ~2^31 cell-updates (~1 ms on a launch-bound small board, ~0.1 ms on a large one) instead
        // of one turn, so a short Run does not ramp up through a synchronised step per doubling.
        int64_t chunk = 1;
        while (chunk < 1024 && chunk * 2 * req.ImageHeight * req.ImageWidth <= (int64_t(1) << 31)) chunk *= 2;
        while (cTurn < req.Turns && rc == GOL_OK) {
            if (control(lk)) break;
            const int64_t n = std::min(chunk, req.Turns - cTurn);
            const auto t0 = std::chrono::steady_clock::now();
            rc = gol_engine_step(eng, n);
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (rc != GOL_OK) break;
            cTurn += n;  // the (turn, board) pair is updated atomically under mu
            if (ms < 5.0 && chunk < (1LL << 20)) chunk *= 2;
            else if (ms > 20.0 && chunk > 1) chunk /= 2;
            // let Retrieve / Pause / Quit in before the next chunk
            cv.wait(lk, [&] { return waiters.load() == 0; });
        }
        if (rc == GOL_OK) {
            res->TurnsCompleted = cTurn;  // broker.go:228-230
            rc = fill_board(res);
            res->AliveCount = res->AliveLen;
        }
        running = false;
        cv.notify_all();
        return rc;
    }

    // broker.go:256-277
    int RetrieveCurrentData(const stubs::Request &req, stubs::Response *res)
    {
        if (!res) return gol_set_error(GOL_EINVAL, "res is NULL");
        Access acc(*this);
        if (!have_world) return gol_set_error(GOL_ESTATE, "no board: Operations.Run has not been called");
        if ((req.ImageHeight && req.ImageHeight != H) || (req.ImageWidth && req.ImageWidth != W))
            return gol_set_error(GOL_EINVAL, "request size %lldx%lld does not match the board %lldx%lld",
                                 (long long)req.ImageWidth, (long long)req.ImageHeight, (long long)W, (long long)H);
        res->TurnsCompleted = cTurn;
        if (cTurn == 0) {
            // cWorld is all-zero until the first turn completes (broker.go:67-70, 96-105)
            if (res->World)
                for (int64_t y = 0; y < H; ++y) memset(res->World + y * (res->WorldStride ? res->WorldStride : W), 0, W);
            res->AliveLen = 0;
            res->AliveCount = 0;
            return GOL_OK;
        }
        int rc = GOL_OK;
        if (res->World || res->Alive) rc = fill_board(res);
        if (rc == GOL_OK) {
            uint64_t c = 0;
            rc = gol_engine_alive_count(eng, &c);  // len(calculateAliveCells(...)), broker.go:273
            res->AliveCount = (int64_t)c;
            if (!res->Alive) res->AliveLen = (int64_t)c;
        }
        return rc;
    }

    int Pause()  // broker.go:251-254
    {
        Access acc(*this);
        if (shut_down) return gol_set_error(GOL_EQUIT, "broker has shut down");
        pending_pause++;
        cv.notify_all();
        return GOL_OK;
    }

    int Quit()  // broker.go:236-239
    {
        Access acc(*this);
        if (shut_down) return gol_set_error(GOL_EQUIT, "broker has shut down");
        pending_quit++;
        cv.notify_all();
        return GOL_OK;
    }

    int SuperQuit()  // broker.go:241-249: stop the loop, the workers and the listener
    {
        Access acc(*this);
        if (running) pending_quit++;
        shut_down = true;
        cv.notify_all();
        return GOL_OK;
    }
};

struct gol_broker {
    Operations ops;
};

// ------------------------------------------------------------------ C ABI wrappers
static stubs::Request to_req(const gol_request *r)
{
    stubs::Request q;
    if (!r) return q;
    q.World = r->World;
    q.WorldStride = r->world_stride;
    q.Turns = r->Turns;
    q.ImageHeight = r->ImageHeight;
    q.ImageWidth = r->ImageWidth;
    q.Threads = r->Threads;
    q.EndY = r->EndY;
    q.StartY = r->StartY;
    q.Worker = r->Worker;
    return q;
}

static stubs::Response to_res(const gol_response *r)
{
    stubs::Response s;
    s.Alive = r->Alive;
    s.AliveCap = r->alive_cap;
    s.World = r->World;
    s.WorldStride = r->world_stride;
    s.WorkSlice = r->WorkSlice;
    s.WorkStride = r->work_stride;
    return s;
}

static void from_res(const stubs::Response &s, gol_response *r)
{
    r->alive_len = s.AliveLen;
    r->AliveCount = s.AliveCount;
    r->TurnsCompleted = s.TurnsCompleted;
    r->Worker = s.Worker;
}

extern "C" int gol_broker_create(const gol_config *cfg, gol_broker **out)
{
    if (!out) return gol_set_error(GOL_EINVAL, "out is NULL");
    gol_broker *b = new gol_broker();
    if (cfg) b->ops.cfg = *cfg;
    else b->ops.cfg.device = -1;
    *out = b;
    return GOL_OK;
}

extern "C" void gol_broker_destroy(gol_broker *b) { delete b; }

extern "C" int gol_broker_run(gol_broker *b, const gol_request *req, gol_response *res)
{
    if (!b || !req || !res) return gol_set_error(GOL_EINVAL, "NULL argument");
    stubs::Response r = to_res(res);
    int rc = b->ops.Run(to_req(req), &r);
    from_res(r, res);
    return rc;
}

extern "C" int gol_broker_retrieve(gol_broker *b, const gol_request *req, gol_response *res)
{
    if (!b || !res) return gol_set_error(GOL_EINVAL, "NULL argument");
    stubs::Response r = to_res(res);
    int rc = b->ops.RetrieveCurrentData(to_req(req), &r);
    from_res(r, res);
    return rc;
}

extern "C" int gol_broker_pause(gol_broker *b) { return b ? b->ops.Pause() : gol_set_error(GOL_EINVAL, "NULL"); }
extern "C" int gol_broker_quit(gol_broker *b) { return b ? b->ops.Quit() : gol_set_error(GOL_EINVAL, "NULL"); }
extern "C" int gol_broker_superquit(gol_broker *b)
{
    return b ? b->ops.SuperQuit() : gol_set_error(GOL_EINVAL, "NULL");
}

extern "C" int gol_broker_paused(gol_broker *b, int32_t *paused)
{
    if (!b || !paused) return gol_set_error(GOL_EINVAL, "NULL argument");
    Operations::Access acc(b->ops);
    *paused = b->ops.paused ? 1 : 0;
    return GOL_OK;
}

extern "C" int gol_worker_update(const gol_request *req, gol_response *res)
{
    if (!req || !res) return gol_set_error(GOL_EINVAL, "NULL argument");
    GameOfLifeOperations w;
    stubs::Response r = to_res(res);
    int rc = w.Update(to_req(req), &r);
    from_res(r, res);
    return rc;
}
