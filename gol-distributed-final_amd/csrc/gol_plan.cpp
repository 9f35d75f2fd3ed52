// gol_plan.cpp -- the schedule of a row-sharded step, as data (include/golhip.h, "plans").
//
// The reference partitions rows per turn and ships the whole board to every worker
// (broker.go:135-206, 143-157).  The sharded engine applies the same partition once and, per
// k-turn step, exchanges kx halo rows with the ring neighbours.  What a shard sends and
// receives (gol_halo_plan) and which launches make up a step (gol_step_plan) are computed
// here, in plain host code: the engine (gol_engine.cpp exchange() / launch_k()) executes
// exactly these plans, and so does the Python mirror (golhip.sharded) that the multi-process
// gloo tests drive on the CPU, so both run one schedule.
#include <stdint.h>

#include "golhip.h"
#include "gol_internal.h"

extern "C" int gol_halo_plan(int64_t H, int32_t nranks, int32_t rank, int32_t k, gol_halo_op *ops, int32_t cap,
                             int32_t *n)
{
    if (!n || nranks < 1 || rank < 0 || rank >= nranks || k < 1 || H < nranks || (cap > 0 && !ops) || cap < 0)
        return gol_set_error(GOL_EINVAL, "bad halo plan arguments (H %lld, rank %d of %d, k %d)", (long long)H, rank,
                             nranks, k);
    int64_t y0 = 0, y1 = 0;
    int rc = gol_partition_rows(H, nranks, rank, &y0, &y1);
    if (rc) return rc;
    const int64_t R = y1 - y0;
    if (k > H / nranks) return gol_set_error(GOL_EINVAL, "k %d exceeds the smallest shard (%lld rows)", k, (long long)(H / nranks));
    const int32_t prev = (rank + nranks - 1) % nranks, next = (rank + 1) % nranks;
    // Issue order.  ncclSend/ncclRecv (and torch's P2P ops) match the sends of one rank to
    // another with that rank's receives from it in issue order.  For nranks = 2 both
    // neighbours are one peer: my first send (top rows) meets the peer's first receive (its
    // bottom ghost rows, the rows below its last row on the torus), my second send (bottom
    // rows) its second receive (top ghost rows).  nranks = 1 sends to itself: the torus wrap.
    const gol_halo_op plan[4] = {
        {GOL_HALO_SEND, prev, 0, k},      // my first k rows -> the rank above (its bottom ghosts)
        {GOL_HALO_RECV, next, R, k},      // ghost rows [R, R+k) <- the first k rows of the rank below
        {GOL_HALO_SEND, next, R - k, k},  // my last k rows -> the rank below (its top ghosts)
        {GOL_HALO_RECV, prev, -k, k},     // ghost rows [-k, 0) <- the last k rows of the rank above
    };
    for (int i = 0; i < 4 && i < cap; ++i) ops[i] = plan[i];
    *n = 4;
    return GOL_OK;
}

extern "C" int gol_step_plan(int64_t R, int32_t k, int32_t kx, int32_t flags, gol_launch *out, int32_t cap,
                             int32_t *n)
{
    if (!n || R < 1 || k < 1 || kx < k || kx > R || cap < 0 || (cap > 0 && !out))
        return gol_set_error(GOL_EINVAL, "bad step plan arguments (R %lld, k %d, kx %d)", (long long)R, k, kx);
    gol_launch plan[3];
    int m = 0;
    const bool split = !(flags & GOL_STEP_SERIAL) && (flags & (GOL_STEP_OVERLAP | GOL_STEP_EDGE_FIRST)) &&
                       R >= 3 * (int64_t)kx;
    if (!split) {
        // one launch over every row, once the halo is in; the next exchange waits for it
        plan[m++] = {GOL_LAUNCH_MAIN, 1, 0, R};
    } else {
        // the rows the next exchange sends (and that need this step's halo) first -- on the edge
        // stream (OVERLAP) or ahead of the interior on the compute stream (EDGE_FIRST); the
        // interior [kx, R - kx) reads no ghost row and runs beside the next exchange
        const int32_t st = (flags & GOL_STEP_OVERLAP) ? GOL_LAUNCH_EDGE : GOL_LAUNCH_MAIN;
        plan[m++] = {st, 1, 0, kx};
        plan[m++] = {st, 1, R - kx, kx};
        plan[m++] = {GOL_LAUNCH_MAIN, 0, kx, R - 2 * (int64_t)kx};
    }
    for (int i = 0; i < m && i < cap; ++i) out[i] = plan[i];
    *n = m;
    return GOL_OK;
}
