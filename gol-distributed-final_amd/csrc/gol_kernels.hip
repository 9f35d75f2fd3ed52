// gol_kernels.hip -- gfx950 (MI355X) kernels of the Game-of-Life hot path.
//
// Replaces the reference's per-cell Go loops:
//   worker.go:15-42 calculateNextState, worker.go:44-70 calculateSurroundings
//   broker.go:47-58 calculateAliveCells (count part)
// with two board representations:
//   * bit board  : 32 cells per uint32 (64 per uint64, LSB = lowest x).  A lane
//                  owns DW consecutive words of a row and slides down a strip
//                  of rows; K generations are pipelined in registers (temporal
//                  blocking), so a launch reads and writes the board once for K
//                  turns.  Stepped in the column-band layout (bit b of word w =
//                  cell b*Wd + w, shift-free generations) when W % 1024 == 0.
//   * byte board : one byte per cell (exact reference semantics incl. bytes
//                  that are neither 0 nor 255), SWAR on 4 cells per VGPR.
// One compiled path per kernel family; the variants measured and dropped in
// round 1 (vertical-first stages, barrier-synchronised split pipeline, centred
// standard-layout stages, per-role profiling builds) are recorded in DESIGN.md
// and live in git history (commit 297b13e).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <set>
#include <type_traits>
#include <utility>

#include "gol_kernels.h"

// Polls of a pipeline flag before a wave gives up (sets GOLK_ERR_SPIN in the launch's error
// word and leaves; the host turns that into GOL_EHIP).  A test build sets 0 to force the path.
#ifndef GOL_SPIN_LIMIT
#define GOL_SPIN_LIMIT (1 << 22)
#endif
// s_sleep argument between two polls of a pipeline flag (units of 64 shader cycles): 0 (the
// poll's own LDS round trip paces it) measured +1 % on 65536^2, +0.3 % on 16384^2 bytes, equal on
// the weak board, over 1; 2 was slower (same box, tools/ab.py)
#ifndef GOL_BYTES_SPIN_SLEEP
#define GOL_BYTES_SPIN_SLEEP 0  // (the byte pipeline's polls, spin_until_ge<true>)
#endif
#ifndef GOL_SPIN_SLEEP
#define GOL_SPIN_SLEEP 0
#endif

namespace golk {

// ------------------------------------------------------------------ helpers
// v_bitop3_b32 truth tables: operand 0 -> 0xF0, operand 1 -> 0xCC, operand 2 -> 0xAA.
constexpr unsigned TT_XOR3 = 0x96;  // a ^ b ^ c
constexpr unsigned TT_MAJ = 0xE8;   // majority(a, b, c)
// The rule tail (tools/rule_search.c, tests/test_rule_circuit_cpu.py): with T = t0 + 2(k0 + u +
// 2v) the 3x3 sum including the cell, alive' = (T == 3) | (cell & T == 4)
//   = (t0 | cell) & G2,  G2 = TT_G2(u, v, G1),  G1 = TT_G1(t0, k0, v)  (exactly one of t0, k0, v).
// Three gates instead of the four of t0 ? [S == 1] : cell & [S == 2]: an exhaustive search over
// 3-gate circuits finds them only when it may use that the centre row's horizontal sum includes
// the cell (a centre sum of 0 means a dead cell, 3 a live one), which holds in every kernel here.
constexpr unsigned TT_G1 = 0x16;    // exactly one of a, b, c
constexpr unsigned TT_G2 = 0x29;    // (~a & ~b & ~c) | (~a & b & c) | (a & ~b & c)
constexpr unsigned TT_OUT = 0xA8;   // (a | b) & c

template <unsigned TT>
__device__ __forceinline__ uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}
// lane i receives lane i-1's value (lane 0 receives 0)
__device__ __forceinline__ uint32_t from_lower_lane(uint32_t v)
{
    return __builtin_amdgcn_mov_dpp(v, 0x138 /* wave_shr:1 */, 0xf, 0xf, true);
}
// lane i receives lane i+1's value (lane 63 receives 0)
__device__ __forceinline__ uint32_t from_upper_lane(uint32_t v)
{
    return __builtin_amdgcn_mov_dpp(v, 0x130 /* wave_shl:1 */, 0xf, 0xf, true);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// One atomic per wave into one of GOL_COUNT_SLOTS slots (64 B apart).
__device__ __forceinline__ void slot_add(uint64_t *slots, uint64_t v)
{
    v = wave_sum_u64(v);
    if ((threadIdx.x & 63) == 0 && v) {
        unsigned wave = (blockIdx.x + blockIdx.y * gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
        atomicAdd((unsigned long long *)&slots[(wave % GOL_COUNT_SLOTS) * 8], (unsigned long long)v);
    }
}

// Error word of a launch: flags ORed by lane 0 of a failing wave (a vector global atomic).
__device__ __forceinline__ void raise_error(uint32_t *err, uint32_t flag)
{
    if ((threadIdx.x & 63) == 0) atomicOr(err, flag);
}

template <int DW> struct VecT;
template <> struct VecT<1> { typedef uint32_t type; };
template <> struct VecT<2> { typedef uint2 type; };
template <> struct VecT<4> { typedef uint4 type; };

template <int DW>
__device__ __forceinline__ void load_words(const uint32_t *p, uint32_t (&w)[DW])
{
    typedef typename VecT<DW>::type V;
    V v = *reinterpret_cast<const V *>(p);
    if constexpr (DW == 1) { w[0] = v; }
    if constexpr (DW == 2) { w[0] = v.x; w[1] = v.y; }
    if constexpr (DW == 4) { w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w; }
}
template <int DW>
__device__ __forceinline__ void store_words(uint32_t *p, const uint32_t (&w)[DW])
{
    typedef typename VecT<DW>::type V;
    V v;
    if constexpr (DW == 1) { v = w[0]; }
    if constexpr (DW == 2) { v.x = w[0]; v.y = w[1]; }
    if constexpr (DW == 4) { v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3]; }
    *reinterpret_cast<V *>(p) = v;
}

// B3/S23 from three horizontal sums (rows above/middle/below, value = h0 + 2*h1 in 0..3 per
// cell; the middle one includes the cell) and the middle cell.  T = sum of the 3x3 block
// including the cell = t0 + 2*(k0 + u + 2v); alive' = (T == 3) | (cell & T == 4): 7 gates.
__device__ __forceinline__ uint32_t rule(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1,
                                         uint32_t c0, uint32_t c1, uint32_t cell)
{
    const uint32_t t0 = bitop3<TT_XOR3>(a0, b0, c0);
    const uint32_t k0 = bitop3<TT_MAJ>(a0, b0, c0);
    const uint32_t u = bitop3<TT_XOR3>(a1, b1, c1);
    const uint32_t v = bitop3<TT_MAJ>(a1, b1, c1);
    const uint32_t g1 = bitop3<TT_G1>(t0, k0, v);
    const uint32_t g2 = bitop3<TT_G2>(u, v, g1);
    return bitop3<TT_OUT>(t0, cell, g2);
}

// ------------------------------------------------------------------ register pipeline
// State of stage g (generation g+1): a ring of 3 rows of horizontal sums plus the cells of
// those rows.  Slot s = step % 3 holds the row received at this step; the stage emits the
// next state of the row received one step ago.
template <int K, int DW>
struct Pipe {
    uint32_t h0[K][3][DW];
    uint32_t h1[K][3][DW];
    uint32_t cc[K][3][DW];
};

template <int K, int DW>
__device__ __forceinline__ void pipe_init(Pipe<K, DW> &p)
{
#pragma unroll
    for (int g = 0; g < K; ++g)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < DW; ++j) { p.h0[g][s][j] = 0; p.h1[g][s][j] = 0; p.cc[g][s][j] = 0; }
}

// Standard layout, shifted frame: the horizontal 3-sum is formed from the cell and its two
// LEFT neighbours, S'[p] = c[p] + c[p-1] + c[p-2] = the 3-sum centred on p-1, so a stage
// needs one DPP (left word) instead of two and the centre cell is c << 1.  Every
// generation moves the frame one bit to the left; after K generations one funnel shift
// with the right neighbour word realigns the row.
template <int DW>
__device__ __forceinline__ void hsum_left(const uint32_t (&c)[DW], uint32_t (&h0)[DW], uint32_t (&h1)[DW],
                                          uint32_t (&ctr)[DW])
{
    const uint32_t left_in = from_lower_lane(c[DW - 1]);
#pragma unroll
    for (int j = 0; j < DW; ++j) {
        const uint32_t wl = (j == 0) ? left_in : c[j - 1];
        const uint32_t L1 = __builtin_amdgcn_alignbit(c[j], wl, 31);  // c[p-1] at bit p
        const uint32_t L2 = __builtin_amdgcn_alignbit(c[j], wl, 30);  // c[p-2] at bit p
        h0[j] = bitop3<TT_XOR3>(L1, c[j], L2);
        h1[j] = bitop3<TT_MAJ>(L1, c[j], L2);
        ctr[j] = L1;
    }
}

// One shifted-frame stage (generation g+1) of one row step S, in place on `cur`.
template <int K, int DW, int S>
__device__ __forceinline__ void sstage(Pipe<K, DW> &p, const int g, uint32_t (&cur)[DW])
{
    constexpr int SA = (S + 1) % 3, SM = (S + 2) % 3;
    hsum_left<DW>(cur, p.h0[g][S], p.h1[g][S], p.cc[g][S]);
#pragma unroll
    for (int j = 0; j < DW; ++j)
        cur[j] = rule(p.h0[g][SA][j], p.h1[g][SA][j], p.h0[g][SM][j], p.h1[g][SM][j], p.h0[g][S][j],
                      p.h1[g][S][j], p.cc[g][SM][j]);
}

// Step W of a 3-row wavefront over K shifted-frame stages, one word per lane: row r (ring slot
// r) is at stage W - r.  The three rows' stages are independent within a step, and each op is
// written for all active rows before the next (a one-word stage is a dependent chain of 13
// ops; row after row, the compiler kept the chains apart and one wave issued at the
// dependent-op latency).
template <int K, int NSTG, int W>
__device__ __forceinline__ void sstage_wave3(Pipe<K, 1> &p, uint32_t (&c)[3])
{
    static_assert(NSTG <= K, "stages of the pipe state");
    constexpr bool on[3] = {W < NSTG, W >= 1 && W - 1 < NSTG, W >= 2 && W - 2 < NSTG};
    constexpr int g[3] = {on[0] ? W : 0, on[1] ? W - 1 : 0, on[2] ? W - 2 : 0};
    uint32_t wl[3], L1[3], L2[3], t0[3], k0[3], u[3], v[3], e1[3], e2[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) if (on[r]) wl[r] = from_lower_lane(c[r]);
#pragma unroll
    for (int r = 0; r < 3; ++r) if (on[r]) L1[r] = __builtin_amdgcn_alignbit(c[r], wl[r], 31);
#pragma unroll
    for (int r = 0; r < 3; ++r) if (on[r]) L2[r] = __builtin_amdgcn_alignbit(c[r], wl[r], 30);
#pragma unroll
    for (int r = 0; r < 3; ++r) if (on[r]) p.h0[g[r]][r][0] = bitop3<TT_XOR3>(L1[r], c[r], L2[r]);
#pragma unroll
    for (int r = 0; r < 3; ++r) if (on[r]) p.h1[g[r]][r][0] = bitop3<TT_MAJ>(L1[r], c[r], L2[r]);
#pragma unroll
    for (int r = 0; r < 3; ++r) if (on[r]) p.cc[g[r]][r][0] = L1[r];
#define GOL_ROWS3(expr) _Pragma("unroll") for (int r = 0; r < 3; ++r) if (on[r]) { const int A = (r + 1) % 3, M = (r + 2) % 3; (void)A; (void)M; expr; }
    GOL_ROWS3(k0[r] = bitop3<TT_MAJ>(p.h0[g[r]][A][0], p.h0[g[r]][M][0], p.h0[g[r]][r][0]))
    GOL_ROWS3(u[r] = bitop3<TT_XOR3>(p.h1[g[r]][A][0], p.h1[g[r]][M][0], p.h1[g[r]][r][0]))
    GOL_ROWS3(v[r] = bitop3<TT_MAJ>(p.h1[g[r]][A][0], p.h1[g[r]][M][0], p.h1[g[r]][r][0]))
    GOL_ROWS3(t0[r] = bitop3<TT_XOR3>(p.h0[g[r]][A][0], p.h0[g[r]][M][0], p.h0[g[r]][r][0]))
    GOL_ROWS3(e1[r] = bitop3<TT_G1>(t0[r], k0[r], v[r]))
    GOL_ROWS3(e2[r] = bitop3<TT_G2>(u[r], v[r], e1[r]))
    GOL_ROWS3(c[r] = bitop3<TT_OUT>(t0[r], p.cc[g[r]][M][0], e2[r]))
#undef GOL_ROWS3
}
// All NSTG stages of one 3-row block (steps 0 .. NSTG + 1).
template <int K, int NSTG, int... W>
__device__ __forceinline__ void sstage_waves3(Pipe<K, 1> &p, uint32_t (&c)[3], std::integer_sequence<int, W...>)
{
    (sstage_wave3<K, NSTG, W>(p, c), ...);
}

// Work items of the pipelined kernels (one workgroup = one column group x one strip of rows).
// ranked = 0: equal strips of `strip` rows, workgroup l -> XCD-remapped item.  ranked = 1 (a
// launch of exactly one round, cus x per_cu workgroups): the dispatcher deals workgroup l to CU
// l % cus as the (l / cus)-th arrival there, and a SIMD issues to its oldest ready wave first,
// so the CU's workgroups run at different speeds (one round of equal strips ended them at 247 /
// 298 / 388 / 482 us, tools/timeline.py); each CU then takes one column group x `period` rows
// and splits the rows by arrival rank: rank r gets len[r] rows at off[r].
// Paired ranks (dir != 0): two workgroups of a CU share one row range [off, off + len) and
// walk it from both ends (dir +1 down from its top, dir -1 up from its bottom), claiming input
// blocks from a counter of the pair (claims: 16 words per (CU, pair slot): [0] blocks claimed,
// [1] pipelines done; the second to finish zeroes both for the next launch).  3 * (claimed
// blocks of both) = len + 4K exactly, so their outputs meet without overlap wherever the
// faster one got to: no rank waits for a slower one at the end of the launch.
// Tail (ranked = 0, launches of many rounds): workgroups l >= tail_l, the last dispatched,
// take strips of tail_strip rows from row tail_row on, so the launch ends on short strips
// instead of a partial round of full ones.
struct StripMap {
    int32_t ranked, cus, per_cu, period;
    int32_t len[4], off[4];
    int32_t dir[4], pslot[4];
    uint32_t *claims;
    int32_t chunk;  // blocks per claim
    int32_t tail_l, tail_row, tail_strip;
};

struct BitsArgs {
    const uint32_t *top, *mid, *bot;
    uint32_t *dst;
    int64_t R, Wd, pitch, row0, rows;
    int32_t strip, ngroups;
    uint64_t *slots;
    uint32_t *err;
    uint32_t *cu_slots;  // band pipeline: per-CU masks of the workgroup slots in use (GOL_CU_SLOT_WORDS)
    StripMap sm;
};

// Column group, strip [s0, s1) and a per-CU rotation index of workgroup l (1-D grid); false:
// the workgroup has no rows.
__device__ __forceinline__ bool work_item(const StripMap &sm, int ngroups, int64_t row0, int64_t rows, int strip, int l,
                                          int &group, int &s0, int &s1, int &rot)
{
    const int end = (int)(row0 + rows);
    if (!sm.ranked && sm.tail_l && l >= sm.tail_l) {
        const int i = l - sm.tail_l;
        group = i % ngroups;
        const int t = i / ngroups;
        s0 = (int)row0 + sm.tail_row + t * sm.tail_strip;
        s1 = min(s0 + sm.tail_strip, end);
        rot = group + t;
    } else if (!sm.ranked) {
        // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs (L2 per XCD), so
        // consecutive ids are remapped to let each XCD walk its own contiguous run of column groups
        // of a strip: the lateral halo columns two neighbouring groups both read then meet in one L2.
        const int n = sm.tail_l ? sm.tail_l : (int)gridDim.x, per = n / 8;
        const int m = l < per * 8 ? (l % 8) * per + l / 8 : l;
        group = m % ngroups;
        const int by = m / ngroups;
        s0 = (int)row0 + by * strip;
        s1 = min(s0 + strip, sm.tail_l ? (int)row0 + sm.tail_row : end);
        rot = group + by;
    } else {
        const int rank = l / sm.cus, c = l % sm.cus;
        const int c2 = (c % 8) * (sm.cus / 8) + c / 8;  // contiguous CUs per XCD (cus % 8 == 0)
        group = c2 % ngroups;
        const int t = c2 / ngroups;
        s0 = (int)row0 + t * sm.period + sm.off[rank];
        s1 = min(s0 + sm.len[rank], end);
        rot = rank;
    }
    return s0 < s1;
}
// Direction and claim counter of workgroup l (0 / nullptr: a static strip).
__device__ __forceinline__ int work_dir(const StripMap &sm, int l, uint32_t *&ctr)
{
    ctr = nullptr;
    if (!sm.ranked) return 0;
    const int rank = l / sm.cus, c = l % sm.cus;
    if (!sm.dir[rank]) return 0;
    ctr = sm.claims + ((int64_t)c * 2 + sm.pslot[rank]) * 16;
    return sm.dir[rank];
}

// ------------------------------------------------------------------ bit-board step, standard layout
// grid.x: groups of 4 waves along the row; grid.y: strips of output rows.
// Wave = one column group of 62*DW output words (+1 halo lane each side).
template <int K, int DW>
__global__ void __launch_bounds__(256) bits_step_kernel(BitsArgs a)
{
    const int lane = threadIdx.x & 63;
    const int group = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (group >= a.ngroups) return;  // whole wave exits; no barriers in this kernel

    // column (in words) of this lane's first word, torus-wrapped
    const int64_t col_raw = (int64_t)group * (62 * DW) + (int64_t)(lane - 1) * DW;
    const int64_t col = ((col_raw % a.Wd) + a.Wd) % a.Wd;
    const bool writer = lane >= 1 && lane <= 62 && col_raw < a.Wd;

    // Row indices are wave-uniform 32-bit values (rows < 2^31), kept in SGPRs.
    const int R = (int)a.R;
    const int s0 = (int)a.row0 + (int)blockIdx.y * a.strip;  // first output row
    const int s1 = min(s0 + a.strip, (int)(a.row0 + a.rows)); // end output row
    const int first_in = s0 - K;                              // first input row
    const int last_in = s1 + K - 1;                           // last input row
    const int nblk = ((s1 - s0) + 2 * K + 2) / 3;

    // Input row y lives at base(y) + y*pitch with base = top + k*pitch (y < 0), mid
    // (0 <= y < R) or bot - R*pitch (y >= R): a scalar row pointer plus a 32-bit per-lane
    // byte offset (global_load ... saddr form).
    const uint32_t *top_adj = a.top + K * a.pitch;
    const uint32_t *bot_adj = a.bot - a.R * a.pitch;
    const uint32_t lane_off = (uint32_t)col * 4u;  // bytes
    auto row_ptr = [&](int y) -> const uint32_t * {
        y = y > last_in ? last_in : y;  // steps past the end re-read the last row; never stored
        const uint32_t *base = y < 0 ? top_adj : (y >= R ? bot_adj : a.mid);
        const char *rb = reinterpret_cast<const char *>(base + (int64_t)y * a.pitch);
        return reinterpret_cast<const uint32_t *>(rb + lane_off);
    };

    Pipe<K, DW> p;
    pipe_init(p);

    uint32_t buf[3][DW];
#pragma unroll
    for (int s = 0; s < 3; ++s) load_words<DW>(row_ptr(first_in + s), buf[s]);

    uint32_t alive = 0;  // < 2^32: strips are capped at 2^24 rows x 128 cells per lane
    for (int blk = 0; blk < nblk; ++blk) {
        const int t0 = blk * 3;
        uint32_t nxt[3][DW];
#pragma unroll
        for (int s = 0; s < 3; ++s) load_words<DW>(row_ptr(first_in + t0 + 3 + s), nxt[s]);

        // The three rows of this block run through the K stages as a wavefront (row S is
        // at stage w - S), so every instruction has two independent neighbours to issue
        // beside it and the DPP read-after-write hazards are covered without s_nop.
        uint32_t cur[3][DW];
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < DW; ++j) cur[s][j] = buf[s][j];
#pragma unroll
        for (int w = 0; w < K + 2; ++w) {
            if (w < K) sstage<K, DW, 0>(p, w, cur[0]);
            if (w >= 1 && w - 1 < K) sstage<K, DW, 1>(p, w - 1, cur[1]);
            if (w >= 2 && w - 2 < K) sstage<K, DW, 2>(p, w - 2, cur[2]);
        }
#pragma unroll
        for (int S = 0; S < 3; ++S) {
            uint32_t (&out)[DW] = cur[S];
            const int t = t0 + S;
            const int y = s0 + t - 2 * K;  // row emitted by the last stage
            if (t >= 2 * K && y < s1) {
                const uint32_t nx0 = from_upper_lane(out[0]);  // undo the K-bit frame shift
#pragma unroll
                for (int j = 0; j < DW; ++j) out[j] = __builtin_amdgcn_alignbit(j == DW - 1 ? nx0 : out[j + 1], out[j], K);
                if (writer) {
                    char *rb = reinterpret_cast<char *>(a.dst + (int64_t)y * a.pitch);
                    store_words<DW>(reinterpret_cast<uint32_t *>(rb + lane_off), out);
                    if (a.slots) {
#pragma unroll
                        for (int j = 0; j < DW; ++j) alive += __popc(out[j]);
                    }
                }
            }
        }
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < DW; ++j) buf[s][j] = nxt[s][j];
    }
    if (a.slots) slot_add(a.slots, alive);
}

// Store DW words at byte offset voff of a buffer [row, row + nbytes): out-of-range offsets
// (and nbytes = 0) are dropped by the hardware range check.  aux 2 = nt (streaming) stores.
template <int DW>
__device__ __forceinline__ void store_row_masked(char *row, uint32_t nbytes, uint32_t voff, const uint32_t (&w)[DW])
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, (int)nbytes, 0x00020000);
    if constexpr (DW == 4) {
        typedef __attribute__((ext_vector_type(4))) uint32_t v4u;
        __builtin_amdgcn_raw_buffer_store_b128(v4u{w[0], w[1], w[2], w[3]}, r, voff, 0, 2);
    } else if constexpr (DW == 2) {
        typedef __attribute__((ext_vector_type(2))) uint32_t v2u;
        __builtin_amdgcn_raw_buffer_store_b64(v2u{w[0], w[1]}, r, voff, 0, 0);
    } else {
        static_assert(DW == 4 || DW == 2, "band lanes hold 2 or 4 words");
    }
}

// ------------------------------------------------------------------ band-layout bit board
// Column-band layout: a row is Wd = W/32 words and bit b of word w is cell x = b*Wd + w (32
// bands of Wd columns, one per bit).  The horizontal neighbours of a cell are the SAME bit
// of the neighbouring words, so a generation is pure bitwise logic: no v_alignbit (which
// issues at half the rate of v_bitop3 on gfx950) and the centre cell is the
// word itself.  The column torus wraps band b's last column onto band b+1's first:
// band-space column c = q*Wd + r reads word r rotated right by q (one v_alignbit per word
// per LOAD, only in the waves that straddle the wrap).  Cost: the horizontal halo is k words
// (k columns) instead of one 32-cell word, so a wave of 64 lanes x DW words keeps
// 64 - 2*ceil(k/DW) lanes of output.
template <int DW>
__device__ __forceinline__ void hsum_band(const uint32_t (&c)[DW], uint32_t (&h0)[DW], uint32_t (&h1)[DW])
{
    const uint32_t left_in = from_lower_lane(c[DW - 1]);
    const uint32_t right_in = from_upper_lane(c[0]);
#pragma unroll
    for (int j = 0; j < DW; ++j) {
        const uint32_t L = (j == 0) ? left_in : c[j - 1];
        const uint32_t R = (j == DW - 1) ? right_in : c[j + 1];
        h0[j] = bitop3<TT_XOR3>(L, c[j], R);
        h1[j] = bitop3<TT_MAJ>(L, c[j], R);
    }
}

// The rule written op by op across the DW words (each op has DW-1 independent neighbours):
// per word the 8 ops form a dependent chain, and one wave issues a dependent VALU op ~1.7x
// slower than an independent one (MI355X_MICROARCH.md, constants table).
template <int K, int DW, int S>
__device__ __forceinline__ void bstage(Pipe<K, DW> &p, const int g, uint32_t (&cur)[DW])
{
    constexpr int SA = (S + 1) % 3, SM = (S + 2) % 3;
#pragma unroll
    for (int j = 0; j < DW; ++j) p.cc[g][S][j] = cur[j];
    hsum_band<DW>(p.cc[g][S], p.h0[g][S], p.h1[g][S]);
    const uint32_t (&a0)[DW] = p.h0[g][SA], (&a1)[DW] = p.h1[g][SA];
    const uint32_t (&b0)[DW] = p.h0[g][SM], (&b1)[DW] = p.h1[g][SM];
    const uint32_t (&c0)[DW] = p.h0[g][S], (&c1)[DW] = p.h1[g][S];
    uint32_t t0[DW], k0[DW], u[DW], v[DW], e1[DW], e2[DW];
#pragma unroll
    for (int j = 0; j < DW; ++j) k0[j] = bitop3<TT_MAJ>(a0[j], b0[j], c0[j]);
#pragma unroll
    for (int j = 0; j < DW; ++j) u[j] = bitop3<TT_XOR3>(a1[j], b1[j], c1[j]);
#pragma unroll
    for (int j = 0; j < DW; ++j) v[j] = bitop3<TT_MAJ>(a1[j], b1[j], c1[j]);
#pragma unroll
    for (int j = 0; j < DW; ++j) t0[j] = bitop3<TT_XOR3>(a0[j], b0[j], c0[j]);
#pragma unroll
    for (int j = 0; j < DW; ++j) e1[j] = bitop3<TT_G1>(t0[j], k0[j], v[j]);
#pragma unroll
    for (int j = 0; j < DW; ++j) e2[j] = bitop3<TT_G2>(u[j], v[j], e1[j]);
#pragma unroll
    for (int j = 0; j < DW; ++j) cur[j] = bitop3<TT_OUT>(t0[j], p.cc[g][SM][j], e2[j]);
}

// Same stage with the rule evaluated word by word (fewer live temporaries than bstage; at
// 4 waves per SIMD a dependent op issues as fast as an independent one).
template <int K, int DW, int S>
__device__ __forceinline__ void bstage_seq(Pipe<K, DW> &p, const int g, uint32_t (&cur)[DW])
{
    constexpr int SA = (S + 1) % 3, SM = (S + 2) % 3;
#pragma unroll
    for (int j = 0; j < DW; ++j) p.cc[g][S][j] = cur[j];
    hsum_band<DW>(p.cc[g][S], p.h0[g][S], p.h1[g][S]);
#pragma unroll
    for (int j = 0; j < DW; ++j)
        cur[j] = rule(p.h0[g][SA][j], p.h1[g][SA][j], p.h0[g][SM][j], p.h1[g][SM][j], p.h0[g][S][j],
                      p.h1[g][S][j], p.cc[g][SM][j]);
}

__host__ __device__ constexpr int band_halo_lanes(int k, int dw) { return (k + dw - 1) / dw; }
__host__ __device__ constexpr int band_useful_words(int k, int dw) { return (64 - 2 * band_halo_lanes(k, dw)) * dw; }

// One wave = all K stages (k = 1, 2, 4, 8; 16 with 2 words per lane).  Same row addressing,
// strips and fused count as bits_step_kernel; grid.x: groups of 4 waves along the row,
// grid.y: strips of output rows.
// CONTIG: top == mid - K*pitch and bot == mid + R*pitch (halo rows stored right above and
// below the shard), so input row y is simply mid + y*pitch: no per-row segment select.
template <int K, int DW, bool CONTIG>
__global__ void __launch_bounds__(256) band_step_kernel(BitsArgs a)
{
    constexpr int HL = band_halo_lanes(K, DW);
    constexpr int U = band_useful_words(K, DW);
    const int lane = threadIdx.x & 63;
    const int group = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (group >= a.ngroups) return;

    const int64_t col_raw = (int64_t)group * U + (int64_t)(lane - HL) * DW;
    const int64_t q = col_raw >= 0 ? col_raw / a.Wd : -((-col_raw + a.Wd - 1) / a.Wd);  // floor
    const int64_t col = col_raw - q * a.Wd;
    const uint32_t rot = (uint32_t)q & 31u;
    const bool wrap = __ballot(rot != 0) != 0;  // wave-uniform: any lane outside [0, Wd)
    const bool writer = lane >= HL && lane < 64 - HL && col_raw < a.Wd;

    const int R = (int)a.R;
    const int s0 = (int)a.row0 + (int)blockIdx.y * a.strip;
    const int s1 = min(s0 + a.strip, (int)(a.row0 + a.rows));
    const int first_in = s0 - K;
    const int last_in = s1 + K - 1;
    constexpr int NB = 2;  // blocks per loop trip: the ring below (one block loaded ahead)
    const int nblk = ((s1 - s0) + 2 * K + 2) / 3;
    const int nblk_r = (nblk + NB - 1) / NB * NB;  // trailing blocks re-read the last row, store nothing

    // Every row address is a.mid + (segment displacement + y * pitch): one pointer (the
    // compiler keeps it in the global address space, so the loads are global_load with exact
    // vmcnt waits) plus an integer select.  A select between pointer locals can become an
    // indexed private array (scratch loads in the loop); an integer-to-pointer cast becomes a
    // flat load (vmcnt(0) + lgkmcnt waits).
    const int pitch_b = (int)a.pitch * 4;
    const char *mid_b = reinterpret_cast<const char *>(a.mid);
    const int64_t top_d = (reinterpret_cast<const char *>(a.top) - mid_b) + (int64_t)K * pitch_b;
    const int64_t bot_d = (reinterpret_cast<const char *>(a.bot) - mid_b) - (int64_t)R * pitch_b;
    const uint32_t lane_off = (uint32_t)col * 4u;
    // Stores: buffer stores with the row as the buffer range, so rows that must not be
    // written (pipeline fill, past the strip) and halo lanes are dropped by the range check
    // instead of a branch (stores under a branch make the compiler's vmcnt waits for the NEXT
    // block's rows also wait for these stores).
    char *dst_b = reinterpret_cast<char *>(a.dst);
    const uint32_t row_bytes = (uint32_t)a.Wd * 4u;
    const uint32_t st_off = writer ? lane_off : 0x80000000u;
    const uint32_t st_mask = writer ? 0xFFFFFFFFu : 0u;
    auto load_row = [&](int y, uint32_t (&w)[DW]) {
        y = y > last_in ? last_in : y;
        const int64_t d = CONTIG ? 0 : (y < 0 ? top_d : (y >= R ? bot_d : 0));
        const char *rb = mid_b + (d + (int64_t)y * pitch_b);
        load_words<DW>(reinterpret_cast<const uint32_t *>(rb + lane_off), w);
    };
    auto unwrap = [&](uint32_t (&w)[DW]) {
        if (wrap) {
#pragma unroll
            for (int j = 0; j < DW; ++j) w[j] = __builtin_amdgcn_alignbit(w[j], w[j], rot);
        }
    };

    Pipe<K, DW> p;
    pipe_init(p);

    // Row blocks in flight: a ring of NB three-row buffers; block b lives in ring[b % NB] and
    // is loaded one block ahead of use.  The block loop is unrolled by NB so the ring index is
    // static: no register copies, and the loads are waited for just before their first use (a
    // copy at the loop end would also wait for that block's stores: gfx9 has one in-order
    // vmcnt for loads and stores).
    uint32_t ring[NB][3][DW];
#pragma unroll
    for (int s = 0; s < 3; ++s) load_row(first_in + s, ring[0][s]);
    // Three empty-range stores (dropped) so that the loop is entered with the same memory-
    // counter history as its back edge (loads, then a block's 3 stores): the compiler then
    // waits for the block's rows with vmcnt(6), not vmcnt(3).
#pragma unroll
    for (int s = 0; s < 3; ++s) store_row_masked<DW>(dst_b, 0u, st_off, ring[0][s]);

    uint32_t alive = 0;  // < 2^32: strips are capped at 2^24 rows x 128 cells per lane
    for (int blk0 = 0; blk0 < nblk_r; blk0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int t0 = (blk0 + u) * 3;
#pragma unroll
            for (int s = 0; s < 3; ++s) load_row(first_in + t0 + 3 + s, ring[(u + 1) % NB][s]);
            uint32_t (&cur)[3][DW] = ring[u];
#pragma unroll
            for (int s = 0; s < 3; ++s) unwrap(cur[s]);
#pragma unroll
            for (int w = 0; w < K + 2; ++w) {
                if (w < K) bstage<K, DW, 0>(p, w, cur[0]);
                if (w >= 1 && w - 1 < K) bstage<K, DW, 1>(p, w - 1, cur[1]);
                if (w >= 2 && w - 2 < K) bstage<K, DW, 2>(p, w - 2, cur[2]);
            }
#pragma unroll
            for (int S = 0; S < 3; ++S) {
                const int t = t0 + S;
                const int y = s0 + t - 2 * K;
                const bool row_ok = t >= 2 * K && y < s1;  // wave-uniform
                store_row_masked<DW>(dst_b + (int64_t)(row_ok ? y : s0) * pitch_b, row_ok ? row_bytes : 0u, st_off,
                                     cur[S]);
                if (a.slots) {
                    uint32_t c = 0;
#pragma unroll
                    for (int j = 0; j < DW; ++j) c += __popc(cur[S][j]);
                    alive += c & (row_ok ? st_mask : 0u);
                }
            }
        }
    }
    if (a.slots) slot_add(a.slots, alive);
}

// ------------------------------------------------------------------ LDS helpers of the pipelines
// LDS accesses of the pipelines are inline asm: the compiler treats a global_load_lds in
// flight as a pending LDS write and would put vmcnt(0) before every LDS access it can see
// (which, on the storing wave, also waits for its HBM stores).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
// ceil(a / d) for a >= 0 (else 0) and floor(a / d) for any a (d > 0)
__device__ __forceinline__ int div_ceil_nn(int a, int d) { return a > 0 ? (a + d - 1) / d : 0; }
__device__ __forceinline__ int div_floor(int a, int d) { return a >= 0 ? a / d : -((-a + d - 1) / d); }
typedef __attribute__((ext_vector_type(4))) uint32_t v4u32;
__device__ __forceinline__ v4u32 lds_rd128(const lds_u32 *p)
{
    v4u32 r;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    return r;
}
// Wait for a read with N younger LDS operations allowed in flight (LDS operations of a wave
// complete in order, and these kernels issue no scalar loads in the loop; the assembly check
// tools/check_lds_wait.py confirms the latter).  The value is an in-out operand, so every
// use of it is ordered after the wait.
template <int N>
__device__ __forceinline__ void lds_wait_n(v4u32 &r)
{
    if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r)::"memory");
    else asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(r)::"memory");
}
__device__ __forceinline__ void lds_wait1() { asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory"); }

// Wait until `r` (an issued read) has landed, N younger LDS operations left in flight: at a loop
// back edge, so that the compiler's copies of the loop-carried register read the landed value.
template <int N>
__device__ __forceinline__ void lds_settle(v4u32 &r) { asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(r) : "i"(N) : "memory"); }
// Immediate-offset forms (byte offsets < 64 KiB): ring slots and rows at compile-time offsets
// from one per-lane address register.
template <int OFF>
__device__ __forceinline__ v4u32 lds_rd128_issue_o(const lds_u32 *p)
{
    v4u32 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(p), "i"(OFF) : "memory");
    return r;
}
template <int OFF>
__device__ __forceinline__ void lds_wr128_o(lds_u32 *p, v4u32 v)
{
    asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(p), "v"(v), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ void lds_wr32_o(lds_u32 *p, uint32_t v)
{
    asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(p), "v"(v), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ uint32_t lds_rd32_issue_o(const lds_u32 *p)
{
    uint32_t r;
    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(p), "i"(OFF) : "memory");
    return r;
}
// Two-instruction forms (one asm statement: one conservative hazard s_nop after it, not two):
// the band pipeline's block reads, writes, settle and middle-wave flags through these measured
// weak 163.3 -> 165.2 TCUPS, 262144^2 +0.2 % (same box, profiles/r05/r05g_ab_lds_pairs.jsonl).
template <int OFF0, int OFF1>
__device__ __forceinline__ void lds_rd128x2_issue_o(const lds_u32 *p, v4u32 &a, v4u32 &b)
{
    asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4" : "=&v"(a), "=&v"(b) : "v"(p), "i"(OFF0), "i"(OFF1) : "memory");
}
template <int OFF0, int OFF1>
__device__ __forceinline__ void lds_wr128x2_o(lds_u32 *p, v4u32 a, v4u32 b)
{
    asm volatile("ds_write_b128 %0, %1 offset:%3\n\tds_write_b128 %0, %2 offset:%4" ::"v"(p), "v"(a), "v"(b), "i"(OFF0), "i"(OFF1) : "memory");
}
__device__ __forceinline__ void lds_settle2(v4u32 &a, v4u32 &b) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b)::"memory"); }
__device__ __forceinline__ void lds_flag_wr2(lds_u32 *p, int v, lds_u32 *q, int w)
{
    asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %2, %3" ::"v"(p), "v"(v), "v"(q), "v"(w) : "memory");
}
// Flag write without an exec mask: lane 0's address is the flag, the other lanes write their
// own scratch word (one ds_write, no saveexec / branch around it).
__device__ __forceinline__ void lds_flag_wr(lds_u32 *p, int v) { asm volatile("ds_write_b32 %0, %1" ::"v"(p), "v"(v) : "memory"); }
__device__ __forceinline__ int lds_rd32(const lds_u32 *p)
{
    int r;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    return r;
}
__device__ __forceinline__ void lds_wr32(lds_u32 *p, int v) { asm volatile("ds_write_b32 %0, %1" ::"v"(p), "v"(v) : "memory"); }
// Wait until flag f >= v; returns the value seen (callers cache it: a producer is usually
// several blocks ahead, so most blocks need no flag read), or -1 after GOL_SPIN_LIMIT polls.
// A wave that sees -1 leaves its loop, every wave waiting on it times out the same way, and
// each records GOLK_ERR_SPIN in the launch's error word on its way out (once, after the loop:
// an atomic inside the loop costs the pipeline registers), so the host reports the launch as
// failed (GOL_EHIP) instead of returning a board with unwritten strips.
// YIELD (the byte pipeline, whose waves run at priority 1): the polling wave drops to priority 0,
// so the computing waves of its SIMD win the issue arbitration (+1.5 % on 16384^2 bytes; the band
// pipeline measured 0 / -1 %, same box).
template <bool YIELD = false>
__device__ __forceinline__ int spin_until_ge(const lds_u32 *f, int v)
{
    if constexpr (YIELD) __builtin_amdgcn_s_setprio(0);
#pragma clang loop unroll(disable)
    for (int n = 0; n < GOL_SPIN_LIMIT; ++n) {
        const int x = __builtin_amdgcn_readfirstlane(lds_rd32(f));
        if (x >= v) {
            if constexpr (YIELD) __builtin_amdgcn_s_setprio(1);
            return x;
        }
        __builtin_amdgcn_s_sleep(YIELD ? GOL_BYTES_SPIN_SLEEP : GOL_SPIN_SLEEP);
    }
    if constexpr (YIELD) __builtin_amdgcn_s_setprio(1);
    return -1;
}

// ------------------------------------------------------------------ band layout, split pipeline
// Pair step of one stage.  The stage's input stream x_0, x_1, ... arrives in
// pairs (x_2m, x_2m+1) = (r0, r1); its state holds the horizontal 3-sums of x_2m-2 (a) and
// x_2m-1 (b) and the cells of x_2m-1 (cb).  It emits the next state of rows 2m-1 and 2m in
// place of r0, r1 (one row of delay per stage, as a row-by-row stage) and moves its state on by
// two rows.  The two outputs share the sum of their common rows P = b + c = p0 + 2 p1 + 4 p2
// (c = x_2m's 3-sums; 4 gates), then each takes a 4-gate tail over (P, the third row's sums, its
// cell) found by exhaustive search (tools/rule_search_pair.c; tests/test_rule_circuit_cpu.py
// checks it on every 4 x 3 neighbourhood): with the 2 gates of each row's horizontal sum a
// generation is 8 ops per 32 cells instead of 9.  The tail relies on the cell's row being one of
// the pair (the pair sum of a live cell is >= 1, of a dead one <= 5), which holds for both outputs.
constexpr unsigned TT_PG1 = 0x43;   // (p0, x0, cell)
constexpr unsigned TT_PG2 = 0x25;   // (p1, p2, x1)
constexpr unsigned TT_PG3 = 0x8D;   // (p2, cell, g1)
constexpr unsigned TT_POUT = 0x90;  // (g3, g1, g2)
__device__ __forceinline__ uint32_t pair_tail(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t x0, uint32_t x1,
                                              uint32_t cell)
{
    const uint32_t g1 = bitop3<TT_PG1>(p0, x0, cell);
    const uint32_t g2 = bitop3<TT_PG2>(p1, p2, x1);
    const uint32_t g3 = bitop3<TT_PG3>(p2, cell, g1);
    return bitop3<TT_POUT>(g3, g1, g2);
}
template <int DW>
struct PairState {
    uint32_t a0[DW], a1[DW], b0[DW], b1[DW], cb[DW];
};
template <int DW>
__device__ __forceinline__ void pstage(PairState<DW> &s, uint32_t (&r0)[DW], uint32_t (&r1)[DW])
{
    // word by word, so that few temporaries are live at once (the pipeline holds 5 KW DW state
    // registers beside this); the outputs go to o0 / o1 because a word's 3-sums need its
    // neighbour words' old values.  (Writing the lane's edge words first -- the next stage's DPP
    // moves read them, and a DPP move right after the VALU op that wrote its source waits on an
    // s_nop -- cut the s_nops per trip from 43 to 15 and measured equal, same box.)
    const uint32_t l0 = from_lower_lane(r0[DW - 1]), u0 = from_upper_lane(r0[0]);
    const uint32_t l1 = from_lower_lane(r1[DW - 1]), u1 = from_upper_lane(r1[0]);
    uint32_t o0[DW], o1[DW];
#pragma unroll
    for (int j = 0; j < DW; ++j) {
        const uint32_t x0 = r0[j], x1 = r1[j];
        const uint32_t w0 = j == 0 ? l0 : r0[j - 1], w1 = j == 0 ? l1 : r1[j - 1];
        const uint32_t n0 = j == DW - 1 ? u0 : r0[j + 1], n1 = j == DW - 1 ? u1 : r1[j + 1];
        const uint32_t c0 = bitop3<TT_XOR3>(w0, x0, n0), c1 = bitop3<TT_MAJ>(w0, x0, n0);
        const uint32_t d0 = bitop3<TT_XOR3>(w1, x1, n1), d1 = bitop3<TT_MAJ>(w1, x1, n1);
        const uint32_t k = s.b0[j] & c0;
        const uint32_t p0 = s.b0[j] ^ c0;
        const uint32_t p1 = bitop3<TT_XOR3>(s.b1[j], c1, k);
        const uint32_t p2 = bitop3<TT_MAJ>(s.b1[j], c1, k);
        o0[j] = pair_tail(p0, p1, p2, s.a0[j], s.a1[j], s.cb[j]);  // row 2m-1: above = x_2m-2
        o1[j] = pair_tail(p0, p1, p2, d0, d1, x0);                 // row 2m: below = x_2m+1
        s.a0[j] = c0;
        s.a1[j] = c1;
        s.b0[j] = d0;
        s.b1[j] = d1;
        s.cb[j] = x1;
    }
#pragma unroll
    for (int j = 0; j < DW; ++j) {
        r0[j] = o0[j];
        r1[j] = o1[j];
    }
}

// The K = KW*P stages split over the P waves of one workgroup: wave w runs stages
// [w*KW, (w+1)*KW) and hands every block of RPB = 2 rows (one pair step) to wave w+1 through an
// LDS ring of NS = 4 slots.  A wave then holds 5*KW*4 pipeline VGPRs instead of 5*K*4, which fits
// 4 waves per SIMD.  Wave 0 stages its input rows HBM -> LDS with global_load_lds (no VGPRs),
// wave P-1 stores to HBM.  Synchronisation is per ring, by LDS flags: ready[e] = blocks
// published into ring e, consumed[e] = blocks taken out of it; a producer fills slot b % NS
// once block b-NS is consumed.  Every spin is bounded (spin_until_ge).  1-D grid of work items
// (work_item).
// COUNT: the last wave adds the alive cells of the rows it stores to a.slots (branch-free: a
// per-row uniform select, no branch around the count as a null-slots check made it).
// Role placement (GOL_BAND_PLACE): a workgroup of the band pipeline claims a free slot q (0..3) in
// its CU's mask and each wave takes pipeline role (its SIMD + q) % 4, so that the (up to) four
// workgroups resident on a CU put one wave of every role on every SIMD.  (Roles by wave index +
// a per-workgroup rotation put two waves of one role on a SIMD for 64-75 % of the waves,
// tools/timeline.py, profiles/r03/r03h_tl_roles.jsonl.)  Vector atomics of lane 0.
#ifndef GOL_BAND_PLACE
#define GOL_BAND_PLACE 1
#endif
__device__ __forceinline__ uint32_t cu_slot_index()
{
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;  // XCC_ID
    return (xcc << 8) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 0xFu);
}
__device__ __forceinline__ int claim_cu_slot(uint32_t *m)
{
    uint32_t cur = __hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = 0; i < 8; ++i) {
        const uint32_t fr = ~cur & 0xFu;
        if (!fr) return -1;
        const int b = __ffs(fr) - 1;
        const uint32_t old = atomicCAS(m, cur, cur | (1u << b));
        if (old == cur) return b;
        cur = old;
    }
    return -1;
}

// Cache policy bits of the band pipeline's output stores (2 = nt, streaming) and input loads.
#ifndef GOL_BAND_STORE_AUX
#define GOL_BAND_STORE_AUX 2
#endif
#ifndef GOL_BAND_LOAD_AUX
#define GOL_BAND_LOAD_AUX 0
#endif
// Pipeline shape of k = 12: KW stages in each of P waves; blocks of GOL_BAND_RPB rows (one pair
// step), rings of GOL_BAND_NS slots (the role loops are unrolled over the slots).
#ifndef GOL_BAND_KW
#define GOL_BAND_KW 3
#endif
#define GOL_BAND_P 4
#define GOL_BAND_RPB 2
#define GOL_BAND_NS 4
// The loader issues block b + GOL_BAND_PREFETCH at block b (its in_ring slot was read at the start
// of block b + GOL_BAND_PREFETCH - NS, so up to NS) and waits for block b + 1 only.  Same box, 3
// reps: 3 against 2 weak 163.6-164.1 vs 163.1-163.7 TCUPS, 262144^2 +0.6 %, 65536^2 +1.2 %; 4 as 3
// (profiles/r05/r05d_ab_prefetch.jsonl).
#ifndef GOL_BAND_PREFETCH
#define GOL_BAND_PREFETCH 3
#endif
template <int KW, int P, bool CONTIG, bool COUNT>
__global__ void __launch_bounds__(64 * P)
__attribute__((amdgpu_waves_per_eu(KW >= 4 ? 3 : 4, 8)))  // 5 KW DW pipeline VGPRs
band_pipe_kernel(BitsArgs a)
{
    constexpr int DW = 4;
    constexpr int K = KW * P;
    constexpr int HL = band_halo_lanes(K, DW);
    constexpr int U = band_useful_words(K, DW);
    constexpr int ROW = 64 * DW;
    constexpr int RPB = GOL_BAND_RPB;  // rows per block: one pair step
    constexpr int NS = GOL_BAND_NS;    // (the loops below are unrolled over the NS slots)
    static_assert(RPB == 2, "a block is one pair step");
    __shared__ uint32_t in_ring[NS][RPB][ROW];
    __shared__ uint32_t ring_[P - 1][NS][RPB][ROW];  // ring e+1 in the text = ring[e] here
    __shared__ int ready_[P], consumed_[P];
    __shared__ int flag_scratch[64];  // dummy target of lanes 1..63's flag writes (never read; all waves share it)
    __shared__ int place_[P + 2];  // GOL_BAND_PLACE: SIMD of each wave, the CU slot, the mask index

    const int lane = threadIdx.x & 63;
    const int litem = (int)blockIdx.x;
    int group, s0, s1, rotv;
    const bool has_rows = work_item(a.sm, a.ngroups, a.row0, a.rows, a.strip, litem, group, s0, s1, rotv);
    uint32_t *ctr;
    const int dir = work_dir(a.sm, litem, ctr);  // 0: static strip, +1 / -1: paired (StripMap)
    // Pipeline position of this wave, rotated per workgroup (role placement below refines it)
    int wv = __builtin_amdgcn_readfirstlane(((threadIdx.x >> 6) + rotv) % P);
    constexpr bool PLACE = GOL_BAND_PLACE && P == 4;

    const int64_t col_raw = (int64_t)group * U + (int64_t)(lane - HL) * DW;
    const int64_t band_q = col_raw >= 0 ? col_raw / a.Wd : -((-col_raw + a.Wd - 1) / a.Wd);
    const int64_t col = col_raw - band_q * a.Wd;
    const uint32_t rot = (uint32_t)band_q & 31u;
    const bool wrap = __ballot(rot != 0) != 0;
    const bool writer = lane >= HL && lane < 64 - HL && col_raw < a.Wd;

    const int R = (int)a.R;
    const int first_in = s0 - K;
    const int last_in = s1 + K - 1;
    // the stream: input row first_in + t at stream step t (walking up, dir -1: s1e + K - 1 - t);
    // output row first_in + t - K (s1e - 1 + 2K - t), valid from step 2K on
    const int nblk = ((s1 - s0) + 2 * K + RPB - 1) / RPB;
    constexpr int TRIP = RPB * NS;  // rows per loop trip
    // a pair's range, stretched to s1e so that TRIP divides its len + 4K (whole loop trips); rows
    // past s1 are read clamped and never stored
    const int s1e = dir ? s0 + ((s1 - s0 + 4 * K + TRIP - 1) / TRIP) * TRIP - 4 * K : s1;
    const int nclaim = (s1e - s0 + 4 * K) / RPB;  // blocks of the pair (a multiple of NS)

    const int pitch_b = (int)a.pitch * 4;
    const char *mid_b = reinterpret_cast<const char *>(a.mid);
    const int64_t top_d = (reinterpret_cast<const char *>(a.top) - mid_b) + (int64_t)K * pitch_b;
    const int64_t bot_d = (reinterpret_cast<const char *>(a.bot) - mid_b) - (int64_t)R * pitch_b;
    const uint32_t lane_off = (uint32_t)col * 4u;
    char *dst_b = reinterpret_cast<char *>(a.dst);
    const uint32_t st_off = writer ? lane_off : 0x80000000u;

    // wave 0: block b -> in_ring[b % NS] (global_load_lds).  The slot is an argument: a lambda
    // that captures a __shared__ array silently loses the kernel's host-side stub.
    // Interior blocks (both rows inside [first_in, last_in] and, unless CONTIG, inside the shard's
    // own rows: every block but the first and last few of a strip) take the row address carried
    // from the previous block (uniform) plus the lane's offset; the others clamp and pick the row's
    // segment per row.  stage_in is called for blocks 0, 1, 2, ... in order.
    // The slot is an LDS-typed pointer (a generic one costs a null check per load: 4 SALU).  The
    // interior blocks are one range [ib_lo, ib_lo + ib_n) of block numbers, found here once.
    const int in_lo = CONTIG ? first_in : max(first_in, 0), in_hi = CONTIG ? last_in : min(last_in, R - 1);
    const int64_t row_step = dir >= 0 ? (int64_t)pitch_b : -(int64_t)pitch_b;
    const int y_first = dir >= 0 ? first_in : s1e + K - 1;  // first row of block 0
    const int ib_lo = dir >= 0 ? div_ceil_nn(in_lo - y_first, RPB) : div_ceil_nn(y_first - in_hi, RPB);
    const int ib_hi = dir >= 0 ? div_floor(in_hi - (RPB - 1) - y_first, RPB) : div_floor(y_first - (RPB - 1) - in_lo, RPB);
    const uint32_t ib_n = ib_hi >= ib_lo ? (uint32_t)(ib_hi - ib_lo + 1) : 0u;
    const char *st_row = mid_b + (int64_t)y_first * pitch_b;  // the next block's first row (used when interior)
    auto stage_in = [&](int b, lds_u32 *slot) {
        const char *g0 = st_row;
        st_row += RPB * row_step;
        if ((uint32_t)(b - ib_lo) < ib_n) {
            // The block's two rows as two LDS-DMA loads in the SGPR-base form (the row address in
            // an SGPR pair, the lane's 32-bit offset in a VGPR): the builtin's address computation
            // made the compiler use the 64-bit VGPR-address form here, one v_lshl_add_u64 and a
            // VGPR pair read per load.  Same box, 3 reps: weak +0.6-1.0 %, 262144^2 +-0
            // (profiles/r06/r06_ab_saddr.jsonl).  M0 (the LDS destination) is written and
            // restored inside the statement, one wait state before each load (the hazard scan of
            // tools/check_lds_wait.py checks it); s_nop 4 first covers an SGPR base that a VALU
            // (readfirstlane) may have written.
            static_assert(RPB == 2 && GOL_BAND_LOAD_AUX == 0, "two rows per block, default cache policy");
            uint32_t keep;
            const char *g1 = g0 + row_step;
            asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, %5\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(lane_off), "s"(slot), "s"(g0), "s"(slot + ROW), "s"(g1)
                         : "memory");
            return;
        }
#pragma unroll
        for (int s = 0; s < RPB; ++s) {
            const int t = RPB * b + s;  // stream position
            int y = dir >= 0 ? first_in + t : s1e + K - 1 - t;
            y = y > last_in ? last_in : (y < first_in ? first_in : y);
            const int64_t d = CONTIG ? 0 : (y < 0 ? top_d : (y >= R ? bot_d : 0));
            const char *g = mid_b + (d + (int64_t)y * pitch_b) + lane_off;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g), slot + s * ROW, 16, 0, GOL_BAND_LOAD_AUX);
        }
    };

    if (!has_rows) return;  // whole workgroup (no barrier after this point)
    if (threadIdx.x < P) { ready_[threadIdx.x] = 0; consumed_[threadIdx.x] = 0; }
    if constexpr (PLACE) {
        if (lane == 0) place_[threadIdx.x >> 6] = (int)((__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3u);
        if (threadIdx.x == 0) {
            const uint32_t idx = cu_slot_index();
            place_[P] = a.cu_slots ? claim_cu_slot(a.cu_slots + idx) : -1;
            place_[P + 1] = (int)idx;
        }
    }
    __syncthreads();
    if constexpr (PLACE) {
        const int q = place_[P];
        const int m = (1 << place_[0]) | (1 << place_[1]) | (1 << place_[2]) | (1 << place_[3]);
        if (q >= 0 && m == 0xF) wv = __builtin_amdgcn_readfirstlane((place_[threadIdx.x >> 6] + q) & 3);
    }
    lds_u32 *const ring_l = (lds_u32 *)&ring_[0][0][0][0];
    lds_u32 *const in_l = (lds_u32 *)&in_ring[0][0][0];
    lds_u32 *const ready_l = (lds_u32 *)&ready_[0];
    lds_u32 *const consumed_l = (lds_u32 *)&consumed_[0];
    constexpr int SLOT = RPB * ROW;  // uint32 per slot (one block)

    PairState<DW> st[KW];
#pragma unroll
    for (int g = 0; g < KW; ++g)
#pragma unroll
        for (int j = 0; j < DW; ++j) { st[g].a0[j] = 0; st[g].a1[j] = 0; st[g].b0[j] = 0; st[g].b1[j] = 0; st[g].cb[j] = 0; }
    uint32_t alive = 0;
    const uint32_t st_mask = writer ? 0xFFFFFFFFu : 0u;
    int seen_ready = 0, seen_free = 0;  // cached flag values (ring wv ready, ring wv+1 consumed)
    const uint32_t nrows = (uint32_t)(s1 - s0);
    // One loop per role (0 = loader, 1 = middle, 2 = last), unrolled over the NS ring slots so
    // every LDS address is a per-lane register plus an immediate offset and every wait count is
    // a constant.  Per block b (LDS operations of a wave complete in order):
    //  * wait for block b's two rows (read at the end of block b-1, the wave's youngest LDS
    //    operations: lgkmcnt(0), which also completes block b-1's row writes);
    //  * readers: write "block b consumed"; writers: publish "blocks < b ready";
    //  * compute the pair through the wave's KW stages;
    //  * writers: make sure slot b % NS is free, write the two rows; the last wave stores them
    //    to HBM;
    //  * readers: make sure block b+1 is published; the loader instead refills block b-2's slot
    //    with block b+2 (global_load_lds) and waits (vmcnt) for block b+1's; read block b+1's rows;
    //  * the block count is padded to a multiple of NS: padding blocks read clamped rows and
    //    their stores fall outside the strip's buffer range.
    //  (Reading the next rows before the compute instead holds 8 more VGPRs across it: the kernel
    //  then spills at 128.)
    const int nblkT = (nblk + NS - 1) / NS * NS;
    constexpr int SB = SLOT * 4, RB = ROW * 4;  // slot and row strides in bytes
    lds_u32 *const scratch = (lds_u32 *)&flag_scratch[0] + lane;
    lds_u32 *const rdy_addr = lane == 0 ? ready_l + wv + 1 : scratch;  // writer: ring wv+1 ready
    lds_u32 *const cns_addr = lane == 0 ? consumed_l + wv : scratch;   // reader: ring wv consumed
    lds_u32 *const in_base = in_l + lane * 4;
    lds_u32 *const rd_base = ring_l + (wv - 1) * NS * SLOT + lane * 4;  // ring wv (wv >= 1)
    lds_u32 *const wr_base = ring_l + wv * NS * SLOT + lane * 4;        // ring wv+1 (wv < P-1)
    auto unpack = [&](const v4u32 v, uint32_t (&cur)[DW]) { cur[0] = v.x; cur[1] = v.y; cur[2] = v.z; cur[3] = v.w; };
    auto pack = [&](const uint32_t (&cur)[DW]) { return v4u32{cur[0], cur[1], cur[2], cur[3]}; };
    // last wave: output row y = s0 + 2b + S - 2K, stored at voffset lane_off + (y - s0) * pitch
    // of a buffer spanning the strip's rows: rows before s0 (negative offsets, as unsigned
    // >= 2^32 - 2K * pitch) and from s1 on fall outside it, and so does a halo lane's 2^31.
    const __amdgpu_buffer_rsrc_t strip_rs = __builtin_amdgcn_make_buffer_rsrc(
        dst_b + (int64_t)s0 * pitch_b, (short)0, (int)(nrows * (uint32_t)pitch_b), 0x00020000);
    // (walking up, dir -1: output row y = s1e - 1 + 2K - 2b - S, offsets decreasing)
    // (readfirstlane: the compiler otherwise keeps this uniform row index in a VGPR and compares it
    // with a vector compare per row)
    int rrel = __builtin_amdgcn_readfirstlane(dir >= 0 ? -2 * K : s1e - 1 + 2 * K - s0);  // output row - s0
    const int rstep = dir >= 0 ? 1 : -1;
    uint32_t voff = st_off + (uint32_t)rrel * (uint32_t)pitch_b;
    const uint32_t vstep = (uint32_t)rstep * (uint32_t)pitch_b;
    // a row's cells onto the count: one accumulating v_bcnt per word, as one asm statement (the
    // compiler turns the same chain in C into bcnt pairs + v_add3).  Plain VALU reading VALU
    // results: no wait states inside (tools/check_lds_wait.py checks the pipeline kernels' asm for
    // the VALU hazards the compiler cannot see).
    auto count_row = [&](const uint32_t (&cur)[DW]) {
        uint32_t c = 0;
        asm("v_bcnt_u32_b32 %0, %1, 0\n\tv_bcnt_u32_b32 %0, %2, %0\n\tv_bcnt_u32_b32 %0, %3, %0\n\t"
            "v_bcnt_u32_b32 %0, %4, %0"
            : "=&v"(c)
            : "v"(cur[0]), "v"(cur[1]), "v"(cur[2]), "v"(cur[3]));
        return c;
    };
    auto count_rows2 = [&](const uint32_t (&x0)[DW], const uint32_t (&x1)[DW]) {
        asm("v_bcnt_u32_b32 %0, %1, %0\n\tv_bcnt_u32_b32 %0, %2, %0\n\tv_bcnt_u32_b32 %0, %3, %0\n\t"
            "v_bcnt_u32_b32 %0, %4, %0\n\tv_bcnt_u32_b32 %0, %5, %0\n\tv_bcnt_u32_b32 %0, %6, %0\n\t"
            "v_bcnt_u32_b32 %0, %7, %0\n\tv_bcnt_u32_b32 %0, %8, %0"
            : "+v"(alive)
            : "v"(x0[0]), "v"(x0[1]), "v"(x0[2]), "v"(x0[3]), "v"(x1[0]), "v"(x1[1]), "v"(x1[2]), "v"(x1[3]));
    };
    // the block's two output rows to HBM, and the fused count of the rows this strip stores (halo
    // lanes are masked once at the end): one v_bcnt chain of 8 words onto the count, and a block at
    // a strip's end (a row outside it: a uniform branch) takes the count of that row off again.
    // (Round 5's per-row select cost 15 VALU per block instead of 8: the count in bcnt pairs +
    // v_add3, a vector compare and a select per row.)
    auto emit2 = [&](const uint32_t (&x0)[DW], const uint32_t (&x1)[DW]) {
        __builtin_amdgcn_raw_buffer_store_b128(pack(x0), strip_rs, voff, 0, GOL_BAND_STORE_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(pack(x1), strip_rs, voff + vstep, 0, GOL_BAND_STORE_AUX);
        if constexpr (COUNT) {
            count_rows2(x0, x1);
            const bool in0 = (uint32_t)rrel < nrows, in1 = (uint32_t)(rrel + rstep) < nrows;  // wave-uniform
            if (!(in0 && in1)) alive -= (in0 ? 0u : count_row(x0)) + (in1 ? 0u : count_row(x1));
        }
        voff += 2 * vstep;
        rrel += 2 * rstep;
    };
    lds_u32 *const src_base = wv == 0 ? in_base : rd_base;
    // paired: the loader's claims, NS blocks (one loop trip) each, one in flight (issued at a
    // trip's first block, used at the next trip's start); the first before block 0's loads
    constexpr int FINAL = 1 << 30;  // ready flag = FINAL + blocks: the stream has ended
    // (lane 0 claims; the kernels are built without the atomic optimizer, which broadcast the
    // claim's return at once and so waited for it right there: an atomic round trip per trip)
    uint32_t pending = 0;
    if (wv == 0 && dir && lane == 0) pending = atomicAdd(ctr, (uint32_t)NS);
    // block 0's rows, read to completion here (the compiler copies the loop-carried registers
    // on loop entry, which must not happen while a read is in flight)
    constexpr int PF = GOL_BAND_PREFETCH;
    static_assert(PF >= 2 && PF <= NS, "blocks b+1 .. b+PF in flight in NS slots");
    if (wv == 0) {
        stage_in(0, in_l);
        stage_in(1, in_l + SLOT);
        if constexpr (PF > 2) stage_in(2, in_l + (2 % NS) * SLOT);
        if constexpr (PF > 3) stage_in(3, in_l + (3 % NS) * SLOT);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RPB * (PF - 1)) : "memory");  // block 0 (and the claim)
    } else if (seen_ready < 1) {
        seen_ready = spin_until_ge(ready_l + wv, 1);
        if (seen_ready < 0) {
            raise_error(a.err, GOLK_ERR_SPIN);
            return;
        }
    }
    v4u32 nx0 = lds_rd128_issue_o<0>(src_base);
    v4u32 nx1 = lds_rd128_issue_o<RB>(src_base);
    lds_wait_n<0>(nx0);
    lds_wait_n<0>(nx1);
    // readers: the block the loop is about to run exists (an empty paired stream ends at once)
    bool more = !(seen_ready >= FINAL && seen_ready - FINAL == 0);
    auto step = [&](int b, auto u_c, auto role_c, auto dyn_c, auto skip_c) -> bool {
        constexpr int US = decltype(u_c)::value;
        constexpr int ROLE = decltype(role_c)::value;
        constexpr bool DYN = decltype(dyn_c)::value;
        constexpr bool SKIP = decltype(skip_c)::value;  // a fill block: no rule (see run)
        constexpr bool LAST = ROLE == 2;
        constexpr int NXT = (US + 1) % NS;
        uint32_t r0[DW], r1[DW];
        // block b's rows, the youngest LDS operations of this wave: once they are in, so are
        // block b-1's row writes, and both flags can go out at once
        lds_settle2(nx0, nx1);
        unpack(nx0, r0);
        unpack(nx1, r1);
        if constexpr (ROLE == 1) lds_flag_wr2(cns_addr, b + 1, rdy_addr, b);
        else if constexpr (ROLE != 0) lds_flag_wr(cns_addr, b + 1);  // block b's slot is free
        else lds_flag_wr(rdy_addr, b);          // blocks < b are in ring wv+1
        if constexpr (ROLE == 0) {
            if (wrap) {
#pragma unroll
                for (int j = 0; j < DW; ++j) {
                    r0[j] = __builtin_amdgcn_alignbit(r0[j], r0[j], rot);
                    r1[j] = __builtin_amdgcn_alignbit(r1[j], r1[j], rot);
                }
            }
        }
        if constexpr (!SKIP) {
#pragma unroll
            for (int g = 0; g < KW; ++g) pstage<DW>(st[g], r0, r1);
        }
        if constexpr (LAST) {
            emit2(r0, r1);
        } else {
            if (seen_free < b + 1 - NS) {  // slot b % NS: block b - NS consumed
                seen_free = spin_until_ge(consumed_l + wv + 1, b + 1 - NS);
                if (seen_free < 0) return false;
            }
            lds_wr128x2_o<US * SB, US * SB + RB>(wr_base, pack(r0), pack(r1));
        }
        // block b+1's rows: read now, waited for at the next block's start (the compute of the
        // other waves of the SIMD covers the LDS latency)
        if constexpr (ROLE == 0) {
            stage_in(b + PF, in_l + ((US + PF) % NS) * SLOT);  // refills block b+PF-NS's slot (clamped past the end)
            // block b+1 landed, b+2 .. b+PF in flight (and, paired, at US 1 the claim issued at US 0)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RPB * (PF - 1) + (DYN && US == 1 ? 1 : 0)) : "memory");
            if constexpr (DYN && US == 0) {
                if (lane == 0) pending = atomicAdd(ctr, (uint32_t)NS);
            }
        } else {
            // the next block exists unless the writer's flag says the stream ended before it
            if (seen_ready < b + 2) {
                seen_ready = spin_until_ge(ready_l + wv, b + 2);
                if (seen_ready < 0) return false;
            }
            more = seen_ready < FINAL || b + 1 < seen_ready - FINAL;
        }
        lds_rd128x2_issue_o<NXT * SB, NXT * SB + RB>(src_base, nx0, nx1);  // (past the stream's end: a stale slot, unused)
        return true;
    };
    // blocks the loader has: nblkT, or (paired) the claims granted so far
    auto grant = [&](uint32_t c) { return c >= (uint32_t)nclaim ? 0 : NS; };
    auto trip = [&](int b, auto role_c, auto dyn_c, auto skip_c) -> bool {
        return step(b, std::integral_constant<int, 0>(), role_c, dyn_c, skip_c) &&
               step(b + 1, std::integral_constant<int, 1>(), role_c, dyn_c, skip_c) &&
               step(b + 2, std::integral_constant<int, 2>(), role_c, dyn_c, skip_c) &&
               step(b + 3, std::integral_constant<int, 3>(), role_c, dyn_c, skip_c);
    };
    static_assert(NS == 4, "trip() runs NS steps");
    auto run = [&](auto role_c, auto dyn_c) -> bool {
        constexpr int ROLE = decltype(role_c)::value;
        constexpr bool DYN = decltype(dyn_c)::value;
        int nb = DYN ? 0 : nblkT;
        int b = 0;
        // Fill blocks: stage g's input is valid from stream step 2g on, and a stage whose state
        // missed the steps before S emits garbage only up to step S + 1, which no later stage uses
        // if S <= 2g (stage g's outputs are read from step 2g + 2 on; the last stage's rows before
        // step 2K fall outside the strip).  A wave whose first stage is g0 = KW * wv therefore
        // passes the blocks before step 2 g0 (2b + 1 < 2 g0: b < g0) on without the rule -- whole
        // loop trips of them, in a loop of their own (a branch per block inside the main loop made
        // the compiler spill).
        if constexpr (ROLE != 0) {
            const int nskip = KW * wv;
            for (; b + NS <= nskip; b += NS) {
                if (!more) break;
                if (!trip(b, role_c, dyn_c, std::true_type())) return false;
            }
        }
        for (;; b += NS) {
            if constexpr (ROLE == 0) {
                if constexpr (DYN) nb += grant(__builtin_amdgcn_readfirstlane(pending));
                if (b >= nb) break;
            } else {
                if (!more) break;
            }
            if (!trip(b, role_c, dyn_c, std::false_type())) return false;
        }
        // the last block's reads of the next slot are still in flight: land them before their
        // registers are used for anything else
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (ROLE != 2) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            lds_flag_wr(rdy_addr, FINAL + b);
        }
        if constexpr (ROLE == 0 && DYN) {
            if (lane == 0 && atomicAdd(ctr + 1, 1u) == 1u) {  // both loaders' claims are over
                atomicExch(ctr, 0u);
                atomicExch(ctr + 1, 0u);
            }
        }
        return true;
    };
    // (paired or not changes only the loader's loop: the readers' loops are one instantiation,
    // 65 -> 44 KB of code per kernel; measured equal, same box: weak -0.5 %, 262144^2 +0.8 %,
    // 65536^2 -0.6 %, profiles/r05/r05b_ab_dedupe_bytes.jsonl)
    auto run_role = [&](auto role_c) -> bool {
        if constexpr (decltype(role_c)::value != 0) return run(role_c, std::false_type());
        else return dir ? run(role_c, std::true_type()) : run(role_c, std::false_type());
    };
    bool ok;
    if (wv == 0) ok = run_role(std::integral_constant<int, 0>());
    else if (wv == P - 1) ok = run_role(std::integral_constant<int, 2>());
    else ok = run_role(std::integral_constant<int, 1>());
    if (!ok) raise_error(a.err, GOLK_ERR_SPIN);
    alive &= st_mask;  // halo lanes' rows are not this group's
    if (wv == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (COUNT && wv == P - 1) slot_add(a.slots, alive);
    if constexpr (PLACE) {  // the last wave of the pipeline frees the workgroup's CU slot
        if (wv == P - 1 && lane == 0 && place_[P] >= 0) atomicAnd(a.cu_slots + place_[P + 1], ~(1u << place_[P]));
    }
}

#ifdef GOL_TU_BAND_PIPE
}  // namespace golk

// gol_band_pipe.hip: this file up to here, compiled on its own with the max-ILP machine
// scheduler (Makefile BANDFLAGS): band_pipe_kernel's instantiations, their host stubs and launch.
// The scheduler choice is per translation unit, and it is a per-kernel one: same box, 2 reps,
// max-ILP ran the band boards 1.0-1.9 % faster (weak 148.3 vs 146.8, 262144^2 151.5 vs 148.9,
// 65536^2 139.8 vs 137.2) and the byte pipeline 4.5 % slower (56.8 vs 59.4);
// profiles/r04/r04h_sched.jsonl.
using namespace golk;
const void *golk_band_pipe_fn(bool contig, bool count)
{
    constexpr int KW = GOL_BAND_KW, P = GOL_BAND_P;
    return contig ? (count ? (const void *)band_pipe_kernel<KW, P, true, true> : (const void *)band_pipe_kernel<KW, P, true, false>)
                  : (count ? (const void *)band_pipe_kernel<KW, P, false, true> : (const void *)band_pipe_kernel<KW, P, false, false>);
}
hipError_t golk_band_pipe_launch(bool contig, bool count, unsigned nwg, const BitsArgs &a, hipStream_t s)
{
    constexpr int KW = GOL_BAND_KW, P = GOL_BAND_P;
    const dim3 g(nwg), blk(64 * P);
    if (contig && count) hipLaunchKernelGGL((band_pipe_kernel<KW, P, true, true>), g, blk, 0, s, a);
    else if (contig) hipLaunchKernelGGL((band_pipe_kernel<KW, P, true, false>), g, blk, 0, s, a);
    else if (count) hipLaunchKernelGGL((band_pipe_kernel<KW, P, false, true>), g, blk, 0, s, a);
    else hipLaunchKernelGGL((band_pipe_kernel<KW, P, false, false>), g, blk, 0, s, a);
    return hipGetLastError();
}
#else  // the rest of the kernels and the host side

// 32 x 32 bit-matrix transpose in registers: afterwards x[i] bit b = (before) x[b] bit i.
__device__ __forceinline__ void transpose32(uint32_t (&x)[32])
{
    uint32_t m = 0x0000FFFFu;
#pragma unroll
    for (int j = 16; j != 0; j >>= 1) {
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if (k & j) continue;
            const uint32_t t = ((x[k] >> j) ^ x[k + j]) & m;
            x[k + j] ^= t;
            x[k] ^= t << j;
        }
        m ^= m << (j >> 1);
    }
}

// Standard bit rows (word s bit i = cell 32s + i) -> band rows, or back.  One lane per
// (row, m): the 32 standard words m, m + Wm, ..., m + 31*Wm (Wm = Wd/32) hold exactly the
// cells of band words 32m .. 32m+31, so the conversion is one 32x32 transpose.
template <bool TO_BAND>
__global__ void band_convert_kernel(const uint32_t *src, uint32_t *dst, int64_t rows, int64_t Wm, int64_t spitch,
                                    int64_t dpitch)
{
    const int64_t n = rows * Wm;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / Wm, m = i % Wm;
        uint32_t x[32];
        if (TO_BAND) {
            const uint32_t *s = src + y * spitch + m;
#pragma unroll
            for (int b = 0; b < 32; ++b) x[b] = s[b * Wm];
        } else {
            const uint4 *s = reinterpret_cast<const uint4 *>(src + y * spitch + 32 * m);
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const uint4 q = s[v];
                x[4 * v] = q.x; x[4 * v + 1] = q.y; x[4 * v + 2] = q.z; x[4 * v + 3] = q.w;
            }
        }
        transpose32(x);
        if (TO_BAND) {
            uint4 *d = reinterpret_cast<uint4 *>(dst + y * dpitch + 32 * m);
#pragma unroll
            for (int v = 0; v < 8; ++v) d[v] = make_uint4(x[4 * v], x[4 * v + 1], x[4 * v + 2], x[4 * v + 3]);
        } else {
            uint32_t *d = dst + y * dpitch + m;
#pragma unroll
            for (int b = 0; b < 32; ++b) d[b * Wm] = x[b];
        }
    }
}

// ------------------------------------------------------------------ byte-board step, k turns per launch
// For boards whose bytes are all 0 or 255 (every board after its first turn): each lane
// packs 32 bytes of a row into one 32-cell word (bit i = byte i & 1), runs the same K-stage
// shifted-frame register pipeline as the standard bit board and unpacks the result to 0/255
// bytes.  HBM traffic: 2 bytes per cell per K turns.
__device__ __forceinline__ uint32_t pack32(const uint4 lo, const uint4 hi)
{
    const uint32_t d[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)  // byte q of the word = cells 8q..8q+7
        b[q] = __builtin_amdgcn_udot4(d[2 * q] & 0x01010101u, 0x08040201u,
                                      __builtin_amdgcn_udot4(d[2 * q + 1] & 0x01010101u, 0x80402010u, 0u, false),
                                      false);
    return b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
}
// Same for bytes that are exactly 0x00 or 0xFF (-1 as int8): weights -2^i give +2^i per set byte.
// (Builtins, not inline asm: a v_dot4 result read by another VALU needs 3 wait states, which the
// compiler's hazard recognizer inserts only for instructions it can see.  The inline-asm VOP3P
// form measured +1.5 % and then +-0 on another box, and under the post-RA scheduler it read
// stale sums: profiles/r05/r05y_ab_bytes_sched.jsonl.)
__device__ __forceinline__ uint32_t pack32_ff(const uint4 lo, const uint4 hi)
{
    const uint32_t d[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        b[q] = (uint32_t)__builtin_amdgcn_sdot4((int)d[2 * q], (int)0xF8FCFEFFu,
                                               __builtin_amdgcn_sdot4((int)d[2 * q + 1], (int)0x80C0E0F0u, 0, false), false);
    return b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
}

__device__ __forceinline__ void unpack32(const uint32_t w, uint4 &lo, uint4 &hi)
{
    uint32_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const uint32_t n = (w >> (4 * q)) & 0xFu;
        const uint32_t sp = __umul24(n, 0x00204081u) & 0x01010101u;  // bit i -> byte i
        o[q] = (sp << 8) - sp;                                       // 0x01 -> 0xFF
    }
    lo = make_uint4(o[0], o[1], o[2], o[3]);
    hi = make_uint4(o[4], o[5], o[6], o[7]);
}

struct BytesKArgs {
    const uint8_t *top, *mid, *bot;
    uint8_t *dst;
    int64_t R, Wd, pitch, row0, rows;  // Wd = W / 32 words, pitch in bytes
    int32_t strip, ngroups;
    uint64_t *slots;
    uint32_t *err;
    StripMap sm;
};

// Byte rows of one lane: 32 bytes = two 16-byte loads, packed to a word at use.
struct Raw32 {
    uint4 lo, hi;
};

// One wave = all K stages (k = 1..16), 62 column words per wave.
template <int K>
__global__ void __launch_bounds__(256) bytes_blocked_kernel(BytesKArgs a)
{
    const int lane = threadIdx.x & 63;
    const int group = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (group >= a.ngroups) return;
    const int64_t col_raw = (int64_t)group * 62 + (lane - 1);
    const int64_t col = ((col_raw % a.Wd) + a.Wd) % a.Wd;
    const bool writer = lane >= 1 && lane <= 62 && col_raw < a.Wd;
    const int R = (int)a.R;
    const int s0 = (int)a.row0 + (int)blockIdx.y * a.strip;
    const int s1 = min(s0 + a.strip, (int)(a.row0 + a.rows));
    const int first_in = s0 - K, last_in = s1 + K - 1;
    constexpr int NB = 2;  // blocks per loop trip: one block loaded ahead
    const int nblk = ((s1 - s0) + 2 * K + 2) / 3;
    const int nblk_r = (nblk + NB - 1) / NB * NB;  // trailing blocks store nothing
    // row addresses: a.mid + (segment displacement + y * pitch) (see band_step_kernel)
    const int pitch = (int)a.pitch;
    const char *mid_b = reinterpret_cast<const char *>(a.mid);
    const int64_t top_d = (reinterpret_cast<const char *>(a.top) - mid_b) + (int64_t)K * pitch;
    const int64_t bot_d = (reinterpret_cast<const char *>(a.bot) - mid_b) - (int64_t)R * pitch;
    const uint32_t lane_off = (uint32_t)(col * 32);
    auto load = [&](int y, Raw32 &r) {
        y = y > last_in ? last_in : y;
        const int64_t d = y < 0 ? top_d : (y >= R ? bot_d : 0);
        const uint4 *q = reinterpret_cast<const uint4 *>(mid_b + (d + (int64_t)y * pitch) + lane_off);
        r.lo = q[0];
        r.hi = q[1];
    };
    // range-checked stores (dropped for halo lanes and rows outside the strip)
    char *dst_b = reinterpret_cast<char *>(a.dst);
    const uint32_t row_bytes = (uint32_t)a.Wd * 32u;
    const uint32_t st_off = writer ? lane_off : 0x80000000u;
    const uint32_t st_mask = writer ? 0xFFFFFFFFu : 0u;
    auto store = [&](char *row, uint32_t nbytes, const uint32_t w) {
        uint4 lo, hi;
        unpack32(w, lo, hi);
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, (int)nbytes, 0x00020000);
        typedef __attribute__((ext_vector_type(4))) uint32_t v4u;
        __builtin_amdgcn_raw_buffer_store_b128(v4u{lo.x, lo.y, lo.z, lo.w}, r, st_off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v4u{hi.x, hi.y, hi.z, hi.w}, r, st_off + 16u, 0, 0);
    };
    Pipe<K, 1> p;
    pipe_init(p);
    Raw32 ring[NB][3];
#pragma unroll
    for (int s = 0; s < 3; ++s) load(first_in + s, ring[0][s]);
    // same memory-counter history on loop entry as on the back edge (3 rows x 2 stores)
#pragma unroll
    for (int s = 0; s < 3; ++s) store(dst_b, 0u, 0u);
    uint32_t alive = 0;  // strips are capped at 2^24 rows x 32 cells per lane
    for (int blk0 = 0; blk0 < nblk_r; blk0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int t0 = (blk0 + u) * 3;
#pragma unroll
            for (int s = 0; s < 3; ++s) load(first_in + t0 + 3 + s, ring[(u + 1) % NB][s]);
            uint32_t cur[3][1];
#pragma unroll
            for (int s = 0; s < 3; ++s) cur[s][0] = pack32(ring[u][s].lo, ring[u][s].hi);
#pragma unroll
            for (int w = 0; w < K + 2; ++w) {
                if (w < K) sstage<K, 1, 0>(p, w, cur[0]);
                if (w >= 1 && w - 1 < K) sstage<K, 1, 1>(p, w - 1, cur[1]);
                if (w >= 2 && w - 2 < K) sstage<K, 1, 2>(p, w - 2, cur[2]);
            }
#pragma unroll
            for (int S = 0; S < 3; ++S) {
                const int t = t0 + S;
                const int y = s0 + t - 2 * K;
                const bool row_ok = t >= 2 * K && y < s1;  // wave-uniform
                const uint32_t o = __builtin_amdgcn_alignbit(from_upper_lane(cur[S][0]), cur[S][0], K);
                store(dst_b + (int64_t)(row_ok ? y : s0) * pitch, row_ok ? row_bytes : 0u, o);
                if (a.slots) alive += (uint32_t)__popc(o) & (row_ok ? st_mask : 0u);
            }
        }
    }
    if (a.slots) slot_add(a.slots, alive);
}

// f(integral_constant<0>), .., f(integral_constant<N-1>), unrolled
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (I < N) {
        f(std::integral_constant<int, I>());
        static_for<N, I + 1>(f);
    }
}

// Byte board, split pipeline: K = KW * P turns per launch, P waves per workgroup on one
// column group of 62 words (32 cells per lane, standard bit layout in registers, shifted
// frame), KW stages per wave, blocks of 4 rows (two pair steps, as band_pipe_kernel's, run as a
// wavefront: the second pair one stage behind the first, two independent pair steps in flight
// per stage step -- one 32-cell word per lane is otherwise one dependent chain) handed on
// through LDS rings of NS slots (256 B per row) with band_pipe_kernel's flag protocol and loop
// shape: one loop per role, unrolled over the NS slots (every LDS address a register plus an
// immediate, no slot arithmetic, no per-block branch for the fill blocks).  Wave 0 stages its
// input blocks HBM -> LDS with global_load_lds and packs 32 bytes per lane into one word with
// v_dot4_i32_i8; wave P-1 realigns (after 32 stages the frame shift is exactly one word),
// unpacks through a 2 KiB LDS table (byte -> 8 bytes of 0x00 / 0xFF) and stores the strip
// through one buffer descriptor with a running offset.  One 32-cell word per lane covers K <= 32
// columns of halo, so K = 32 costs no more lanes than K = 16.
// (Round 4's form -- 3-row blocks, one block per loop trip with running slot indices and a
// per-block fill branch -- spent 0.44 scalar instructions per VALU: DESIGN.md §4.4.)
//
// Shifted-frame pair step: pstage's circuit on this frame.  A row's 3-sum at bit p is
// c[p] + c[p-1] + c[p-2] (centred on p-1: the neighbour from the lower lane by one DPP, two
// v_alignbit), the cell is c[p-1]; every stage moves the frame one bit to the left.
__device__ __forceinline__ void spstage(PairState<1> &s, uint32_t &r0, uint32_t &r1)
{
    const uint32_t w0 = from_lower_lane(r0), w1 = from_lower_lane(r1);
    const uint32_t l0 = __builtin_amdgcn_alignbit(r0, w0, 31), m0 = __builtin_amdgcn_alignbit(r0, w0, 30);
    const uint32_t l1 = __builtin_amdgcn_alignbit(r1, w1, 31), m1 = __builtin_amdgcn_alignbit(r1, w1, 30);
    const uint32_t c0 = bitop3<TT_XOR3>(l0, r0, m0), c1 = bitop3<TT_MAJ>(l0, r0, m0);
    const uint32_t d0 = bitop3<TT_XOR3>(l1, r1, m1), d1 = bitop3<TT_MAJ>(l1, r1, m1);
    const uint32_t k = s.b0[0] & c0;
    const uint32_t p0 = s.b0[0] ^ c0;
    const uint32_t p1 = bitop3<TT_XOR3>(s.b1[0], c1, k);
    const uint32_t p2 = bitop3<TT_MAJ>(s.b1[0], c1, k);
    r0 = pair_tail(p0, p1, p2, s.a0[0], s.a1[0], s.cb[0]);  // row 2m-1: its cell = c[p-1] of x_2m-1
    r1 = pair_tail(p0, p1, p2, d0, d1, l0);                 // row 2m: its cell = c[p-1] of x_2m
    s.a0[0] = c0;
    s.a1[0] = c1;
    s.b0[0] = d0;
    s.b1[0] = d1;
    s.cb[0] = l1;
}

#ifndef GOL_BYTES_PER_CU
#define GOL_BYTES_PER_CU 3  // workgroups per CU of a one-round launch
#endif
// Ring slots of the byte pipeline: NS hand-off slots of 4 rows between the waves, NSI input slots
// of the first wave (2 blocks in flight); the role loops are unrolled over NS (NSI divides it)
#ifndef GOL_BYTES_NS
#define GOL_BYTES_NS 3
#endif
#ifndef GOL_BYTES_NSI
#define GOL_BYTES_NSI 3
#endif
// Cache policy bits of the byte pipeline's output stores (0: default)
#ifndef GOL_BYTES_STORE_AUX
#define GOL_BYTES_STORE_AUX 0
#endif
template <int KW, int P, bool COUNT>
__global__ void __launch_bounds__(64 * P) __attribute__((amdgpu_waves_per_eu(6, 8))) bytes_pipe_kernel(BytesKArgs a)
{
    constexpr int K = KW * P;
    static_assert(K <= 32, "one 32-cell halo word per side");
    constexpr int RPB = 4;            // rows per block: two pair steps
    constexpr int NS = GOL_BYTES_NS;  // (the loops below are unrolled over the NS slots)
    constexpr int NSI = GOL_BYTES_NSI;
    static_assert(NS % NSI == 0 && NSI >= 3, "input slots: 2 blocks in flight, one being read");
    constexpr int ROW = 64;  // uint32 per ring row
    __shared__ uint32_t ring[P - 1][NS][RPB][ROW];
    __shared__ uint32_t in_ring[NSI][RPB][2][256];  // byte rows: [half][lane][16 bytes]
    __shared__ uint2 lut[256];
    __shared__ int ready[P], consumed[P];
    __shared__ int flag_scratch[64];  // dummy target of lanes 1..63's flag writes (lds_flag_wr; never read)

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int group, s0, s1, rotv;
    if (!work_item(a.sm, a.ngroups, a.row0, a.rows, a.strip, blockIdx.x, group, s0, s1, rotv)) return;
    uint32_t *ctr;
    const int dir = work_dir(a.sm, blockIdx.x, ctr);  // 0: static strip, +1 / -1: paired
    const int64_t col_raw = (int64_t)group * 62 + (lane - 1);
    const int64_t col = ((col_raw % a.Wd) + a.Wd) % a.Wd;
    const bool writer = lane >= 1 && lane <= 62 && col_raw < a.Wd;
    const int R = (int)a.R;
    const int first_in = s0 - K, last_in = s1 + K - 1;
    const int nblk = ((s1 - s0) + 2 * K + RPB - 1) / RPB;
    constexpr int TRIP = RPB * NS;  // rows per loop trip
    // a pair's range, stretched to s1e so that TRIP divides its len + 4K (rows past s1 are read
    // clamped and never stored: they only feed outputs past s1)
    const int s1e = dir ? s0 + ((s1 - s0 + 4 * K + TRIP - 1) / TRIP) * TRIP - 4 * K : s1;
    const int nclaim = (s1e - s0 + 4 * K) / RPB;  // blocks of the pair (a multiple of NS)
    const int pitch = (int)a.pitch;
    const char *mid_b = reinterpret_cast<const char *>(a.mid);
    const int64_t top_d = (reinterpret_cast<const char *>(a.top) - mid_b) + (int64_t)K * pitch;
    const int64_t bot_d = (reinterpret_cast<const char *>(a.bot) - mid_b) - (int64_t)R * pitch;
    const uint32_t lane_off = (uint32_t)(col * 32);
    char *dst_b = reinterpret_cast<char *>(a.dst);
    const uint32_t st_off = writer ? lane_off : 0x80000000u;
    const uint32_t st_mask = writer ? 0xFFFFFFFFu : 0u;

    // stream position t -> input row (walking up, dir -1: from s1e + K - 1)
    auto in_row = [&](int t) { return dir >= 0 ? first_in + t : s1e + K - 1 - t; };
    // wave 0: block b -> an in_ring slot (the slot is an argument: a lambda that captures a
    // __shared__ array loses the kernel's host-side stub).  Interior blocks (both rows inside the
    // shard and inside [first_in, last_in]: every block but the first and last few of a strip) take
    // one row address, carried from block to block and stepped by a pitch; the others clamp and
    // pick the row's segment per row (round 4: +2.4 % on 16384^2 bytes over per-row addresses).
    // The slot is an LDS-typed pointer (a generic one costs a null check per load: 4 SALU) and the
    // interior blocks are one range [ib_lo, ib_lo + ib_n) of block numbers, found here once.  (The
    // load's immediate offset moves its LDS destination too: the second 16 bytes of a lane's 32
    // take their own address.)
    const int in_lo = max(first_in, 0), in_hi = min(last_in, R - 1);
    const int64_t row_step = dir >= 0 ? (int64_t)pitch : -(int64_t)pitch;
    const int y_first = in_row(0);
    const int ib_lo = dir >= 0 ? div_ceil_nn(in_lo - y_first, RPB) : div_ceil_nn(y_first - in_hi, RPB);
    const int ib_hi = dir >= 0 ? div_floor(in_hi - (RPB - 1) - y_first, RPB) : div_floor(y_first - (RPB - 1) - in_lo, RPB);
    const uint32_t ib_n = ib_hi >= ib_lo ? (uint32_t)(ib_hi - ib_lo + 1) : 0u;
    const char *st_u = mid_b + (int64_t)y_first * pitch;  // the next block's first row (wave-uniform)
    constexpr int IROW = 2 * 256;  // uint32 per input row in LDS (two 16-byte halves of 64 lanes)
    auto stage_in = [&](int b, lds_u32 *slot) {
        const char *gu = st_u;
        st_u += RPB * row_step;
        if ((uint32_t)(b - ib_lo) < ib_n) {
            // The block's 8 LDS-DMA loads in the SGPR-base form, as the band loader's (row address
            // in an SGPR pair, the lane's 32-bit offset -- and +16 for a row's second half -- in a
            // VGPR; M0 set and restored inside, a wait state before each load): the builtin made
            // the compiler compute a 64-bit VGPR address per load.  Same box, 3 reps: 16384^2
            // bytes 63.0 -> 63.7 TCUPS (profiles/r06/r06_ab_bsaddr.jsonl).
            static_assert(RPB == 4, "four rows per block");
            // row bases, wave-uniform: readfirstlane makes that explicit for builds whose control
            // flow hides it (GOL_SPIN_LIMIT=0: the "s" operands below would get VGPRs); it folds
            // away where the compiler already keeps them in SGPRs
            auto uni = [](const char *q) {
                const uint64_t v = reinterpret_cast<uint64_t>(q);
                const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
                const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
                return reinterpret_cast<const char *>(lo | (hi << 32));
            };
            const char *r0 = uni(gu), *r1 = uni(r0 + row_step), *r2 = uni(r1 + row_step), *r3 = uni(r2 + row_step);
            uint32_t keep;
            asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\t"
                         "s_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %7\n\t"
                         "s_add_u32 m0, %3, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %7\n\t"
                         "s_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %8\n\t"
                         "s_add_u32 m0, %4, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %8\n\t"
                         "s_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %9\n\t"
                         "s_add_u32 m0, %5, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %9\n\t"
                         "s_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %10\n\t"
                         "s_add_u32 m0, %6, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %10\n\t"
                         "s_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(lane_off), "v"(lane_off + 16u), "s"(slot), "s"(slot + IROW), "s"(slot + 2 * IROW),
                           "s"(slot + 3 * IROW), "s"(r0), "s"(r1), "s"(r2), "s"(r3)
                         : "memory", "scc");
            return;
        }
#pragma unroll
        for (int S = 0; S < RPB; ++S) {
            int y = in_row(RPB * b + S);
            y = y > last_in ? last_in : (y < first_in ? first_in : y);  // past the end: clamped, never stored
            const int64_t d = y < 0 ? top_d : (y >= R ? bot_d : 0);
            const char *gg = mid_b + (d + (int64_t)y * pitch) + lane_off;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(gg), slot + S * IROW, 16, 0, 0);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(gg + 16), slot + S * IROW + 256, 16, 0, 0);
        }
    };
    __builtin_amdgcn_s_setprio(1);  // polls drop to 0 (spin_until_ge<true>)
    for (int i = threadIdx.x; i < 256; i += 64 * P) {
        uint32_t o[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t sp = __umul24((i >> (4 * h)) & 0xF, 0x00204081u) & 0x01010101u;
            o[h] = (sp << 8) - sp;
        }
        lut[i] = make_uint2(o[0], o[1]);
    }
    if (threadIdx.x < P) { ready[threadIdx.x] = 0; consumed[threadIdx.x] = 0; }
    __syncthreads();
    lds_u32 *const ring_l = (lds_u32 *)&ring[0][0][0][0];
    lds_u32 *const in_l = (lds_u32 *)&in_ring[0][0][0][0];
    lds_u32 *const ready_l = (lds_u32 *)&ready[0];
    lds_u32 *const consumed_l = (lds_u32 *)&consumed[0];
    constexpr int SLOT = RPB * ROW;        // uint32 per hand-off slot
    constexpr int ISLOT = RPB * 2 * 256;   // uint32 per input slot
    constexpr int SB = SLOT * 4, RB = ROW * 4, ISB = ISLOT * 4;
    lds_u32 *const scratch = (lds_u32 *)&flag_scratch[0] + lane;
    lds_u32 *const rdy_addr = lane == 0 ? ready_l + wv + 1 : scratch;  // ring wv+1 ready
    lds_u32 *const cns_addr = lane == 0 ? consumed_l + wv : scratch;   // ring wv consumed
    lds_u32 *const in_base = in_l + lane * 4;
    lds_u32 *const rd_base = ring_l + (wv - 1) * NS * SLOT + lane;  // ring wv (wv >= 1)
    lds_u32 *const wr_base = ring_l + wv * NS * SLOT + lane;        // ring wv+1 (wv < P-1)

    PairState<1> st[KW];
#pragma unroll
    for (int g = 0; g < KW; ++g) { st[g].a0[0] = 0; st[g].a1[0] = 0; st[g].b0[0] = 0; st[g].b1[0] = 0; st[g].cb[0] = 0; }
    uint32_t alive = 0;
    const uint32_t nrows = (uint32_t)(s1 - s0);
    // last wave: output row y stored at voffset st_off + (y - s0) * pitch of ONE buffer spanning
    // the strip's rows (the host keeps rows x pitch < 2^31): rows before s0 (negative offsets, as
    // unsigned >= 2^32 - 2K * pitch), from s1 on, and a halo lane's 2^31 fall outside it
    const __amdgpu_buffer_rsrc_t strip_rs = __builtin_amdgcn_make_buffer_rsrc(
        dst_b + (int64_t)s0 * pitch, (short)0, (int)(nrows * (uint32_t)pitch), 0x00020000);
    int rrel = dir >= 0 ? -2 * K : s1e - 1 + 2 * K - s0;  // output row - s0 of the next row (wave-uniform)
    const int rstep = dir >= 0 ? 1 : -1;
    uint32_t voff = st_off + (uint32_t)rrel * (uint32_t)pitch;
    const uint32_t vstep = (uint32_t)rstep * (uint32_t)pitch;
    // undo the K-bit frame shift (K = 32: exactly the next lane's word; alignbit takes its shift
    // mod 32), unpack through the LUT, store, count
    auto emit = [&](uint32_t w) {
        const uint32_t nxw = from_upper_lane(w);
        const uint32_t o = K % 32 ? __builtin_amdgcn_alignbit(nxw, w, K % 32) : nxw;
        uint2 e[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) e[q] = lut[(o >> (8 * q)) & 0xFF];
        __builtin_amdgcn_raw_buffer_store_b128(v4u32{e[0].x, e[0].y, e[1].x, e[1].y}, strip_rs, voff, 0, GOL_BYTES_STORE_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(v4u32{e[2].x, e[2].y, e[3].x, e[3].y}, strip_rs, voff + 16u, 0, GOL_BYTES_STORE_AUX);
        if constexpr (COUNT) {
            const uint32_t c = __popc(o) + alive;
            alive = (uint32_t)rrel < nrows ? c : alive;
        }
        voff += vstep;
        rrel += rstep;
    };
    constexpr int FINAL = 1 << 30;  // ready flag = FINAL + blocks: the stream has ended
    uint32_t pending = 0;  // the loader's claim in flight (paired)
    if (wv == 0 && dir && lane == 0) pending = atomicAdd(ctr, (uint32_t)NS);
    // block 0's rows read to completion here (the compiler copies loop-carried registers on loop
    // entry, which must not happen while a read is in flight).  A reader's next block (RPB words)
    // is read at the end of a block; the loader reads its block's 2 RPB 16-byte halves at the
    // block's start (32 VGPRs held across the compute would spill at 6 waves per SIMD).
    v4u32 nb[2 * RPB];  // loader
    uint32_t nw[RPB];   // readers
    int seen_ready = 0, seen_free = 0;
    auto read_in = [&](auto off_c) {  // the loader's reads of one input slot
        constexpr int OFF = decltype(off_c)::value;
        static_assert(RPB == 4, "eight half-row reads");
        nb[0] = lds_rd128_issue_o<OFF>(in_base);
        nb[1] = lds_rd128_issue_o<OFF + 1024>(in_base);
        nb[2] = lds_rd128_issue_o<OFF + 2048>(in_base);
        nb[3] = lds_rd128_issue_o<OFF + 3072>(in_base);
        nb[4] = lds_rd128_issue_o<OFF + 4096>(in_base);
        nb[5] = lds_rd128_issue_o<OFF + 5120>(in_base);
        nb[6] = lds_rd128_issue_o<OFF + 6144>(in_base);
        nb[7] = lds_rd128_issue_o<OFF + 7168>(in_base);
    };
    auto read_ring = [&](auto off_c) {  // a reader's reads of one ring slot
        constexpr int OFF = decltype(off_c)::value;
        static_assert(RPB == 4, "four row reads");
        nw[0] = lds_rd32_issue_o<OFF>(rd_base);
        nw[1] = lds_rd32_issue_o<OFF + 256>(rd_base);
        nw[2] = lds_rd32_issue_o<OFF + 512>(rd_base);
        nw[3] = lds_rd32_issue_o<OFF + 768>(rd_base);
    };
    auto settle_in = [&]() {
#pragma unroll
        for (int h = 0; h < 2 * RPB; ++h) lds_settle<0>(nb[h]);
    };
    if (wv == 0) {
        stage_in(0, in_l);
        stage_in(1, in_l + ISLOT);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * RPB) : "memory");  // block 0 landed (the claim before it too)
#pragma unroll
        for (int S = 0; S < RPB; ++S) nw[S] = 0;
    } else {
        seen_ready = spin_until_ge<true>(ready_l + wv, 1);
        if (seen_ready < 0) {
            raise_error(a.err, GOLK_ERR_SPIN);
            return;
        }
        read_ring(std::integral_constant<int, 0>());
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nw[0]), "+v"(nw[1]), "+v"(nw[2]), "+v"(nw[3])::"memory");
    }
    bool more = !(seen_ready >= FINAL && seen_ready - FINAL == 0);
    // Fill blocks (band_pipe_kernel's rule): a wave whose first stage is g0 = KW * wv passes the
    // blocks that end before step 2 g0 (RPB b + RPB <= 2 g0) on without the rule -- a uniform
    // branch per block here (the byte pipeline has registers to spare; a loop of its own per role
    // doubled the role's code)
    const int nskip = 2 * KW * wv / RPB;
    auto step = [&](int b, auto u_c, auto role_c, auto dyn_c) -> bool {
        constexpr int US = decltype(u_c)::value;
        constexpr int ROLE = decltype(role_c)::value;
        constexpr bool DYN = decltype(dyn_c)::value;
        constexpr bool LAST = ROLE == 2;
        constexpr int NXT = (US + 1) % NS;
        uint32_t r[RPB];
        // block b's rows, the youngest LDS operations of this wave: once they are in, so are
        // block b-1's row writes, and both flags can go out at once
        if constexpr (ROLE == 0) {
            read_in(std::integral_constant<int, US % NSI * ISB>());
            settle_in();
#pragma unroll
            for (int S = 0; S < RPB; ++S)
                r[S] = pack32_ff(uint4{nb[2 * S].x, nb[2 * S].y, nb[2 * S].z, nb[2 * S].w},
                                 uint4{nb[2 * S + 1].x, nb[2 * S + 1].y, nb[2 * S + 1].z, nb[2 * S + 1].w});
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nw[0]), "+v"(nw[1]), "+v"(nw[2]), "+v"(nw[3])::"memory");
#pragma unroll
            for (int S = 0; S < RPB; ++S) r[S] = nw[S];
            lds_flag_wr(cns_addr, b + 1);  // block b's slot is free
        }
        if constexpr (!LAST) lds_flag_wr(rdy_addr, b);  // blocks < b are in ring wv+1
        if (ROLE == 0 || b >= nskip) {
            // stage step w: the first pair at stage w, the second at stage w-1 (each stage takes
            // its pairs in stream order)
#pragma unroll
            for (int w = 0; w <= KW; ++w) {
                if (w < KW) spstage(st[w], r[0], r[1]);
                if (w >= 1) spstage(st[w - 1], r[2], r[3]);
            }
        }
        if constexpr (LAST) {
#pragma unroll
            for (int S = 0; S < RPB; ++S) emit(r[S]);
        } else {
            if (seen_free < b + 1 - NS) {  // slot b % NS: block b - NS consumed
                seen_free = spin_until_ge<true>(consumed_l + wv + 1, b + 1 - NS);
                if (seen_free < 0) return false;
            }
            static_assert(RPB == 4, "four row writes");
            lds_wr32_o<US * SB>(wr_base, r[0]);
            lds_wr32_o<US * SB + RB>(wr_base, r[1]);
            lds_wr32_o<US * SB + 2 * RB>(wr_base, r[2]);
            lds_wr32_o<US * SB + 3 * RB>(wr_base, r[3]);
        }
        // block b+1's rows: read now, waited for at the next block's start
        if constexpr (ROLE == 0) {
            stage_in(b + 2, in_l + ((US + 2) % NSI) * ISLOT);  // refills block b+2-NSI's slot (clamped past the end)
            // block b+1 landed, b+2 in flight (2 RPB loads; and, paired, at US 1 the claim issued at US 0)
            if constexpr (DYN && US == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * RPB + 1) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * RPB) : "memory");
            if constexpr (DYN && US == 0) {
                if (lane == 0) pending = atomicAdd(ctr, (uint32_t)NS);
            }
        } else {
            // the next block exists unless the writer's flag says the stream ended before it
            if (seen_ready < b + 2) {
                seen_ready = spin_until_ge<true>(ready_l + wv, b + 2);
                if (seen_ready < 0) return false;
            }
            more = seen_ready < FINAL || b + 1 < seen_ready - FINAL;
            read_ring(std::integral_constant<int, NXT * SB>());
        }
        return true;
    };
    auto grant = [&](uint32_t c) { return c >= (uint32_t)nclaim ? 0 : NS; };

    auto trip = [&](int b, auto role_c, auto dyn_c) -> bool {
        bool ok = true;
        static_for<NS>([&](auto u_c) {
            if (ok) ok = step(b + decltype(u_c)::value, u_c, role_c, dyn_c);
        });
        return ok;
    };
    auto run = [&](auto role_c, auto dyn_c) -> bool {
        constexpr int ROLE = decltype(role_c)::value;
        constexpr bool DYN = decltype(dyn_c)::value;
        int nb = DYN ? 0 : (nblk + NS - 1) / NS * NS;
        int b = 0;
        for (;; b += NS) {
            if constexpr (ROLE == 0) {
                if constexpr (DYN) nb += grant(__builtin_amdgcn_readfirstlane(pending));
                if (b >= nb) break;
            } else {
                if (!more) break;
            }
            if (!trip(b, role_c, dyn_c)) return false;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last block's reads of the next slot
        if constexpr (ROLE != 2) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            lds_flag_wr(rdy_addr, FINAL + b);
        }
        if constexpr (ROLE == 0 && DYN) {
            if (lane == 0 && atomicAdd(ctr + 1, 1u) == 1u) {  // both loaders' claims are over
                atomicExch(ctr, 0u);
                atomicExch(ctr + 1, 0u);
            }
        }
        return true;
    };
    // (paired or not changes only the loader's loop: the readers' loops are one instantiation,
    // which halves their code -- the I-cache holds 64 KiB for two CUs)
    auto run_role = [&](auto role_c) -> bool {
        if constexpr (decltype(role_c)::value != 0) return run(role_c, std::false_type());
        else return dir ? run(role_c, std::true_type()) : run(role_c, std::false_type());
    };
    bool ok;
    if (wv == 0) ok = run_role(std::integral_constant<int, 0>());
    else if (wv == P - 1) ok = run_role(std::integral_constant<int, 2>());
    else ok = run_role(std::integral_constant<int, 1>());
    if (wv == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // input blocks staged past the end
    if (!ok) raise_error(a.err, GOLK_ERR_SPIN);
    alive &= st_mask;  // halo lanes' rows are not this group's
    if (COUNT && wv == P - 1) slot_add(a.slots, alive);
}

#ifndef GOL_BYTES_PIPE_KW
#define GOL_BYTES_PIPE_KW 4
#define GOL_BYTES_PIPE_P 8
#endif
#define BYTES_PIPE(count) (bytes_pipe_kernel<GOL_BYTES_PIPE_KW, GOL_BYTES_PIPE_P, count>)



#ifdef GOL_TU_BYTES_PIPE
}  // namespace golk

// gol_bytes_pipe.hip: this file up to here, compiled on its own with the max-memory-clause
// machine scheduler, bottom-up, and no post-RA scheduler (Makefile BYTEFLAGS): bytes_pipe_kernel's
// instantiations and launch.  Same box, 3 reps each: 59.4 -> 60.4 TCUPS on 16384^2 bytes, then
// 60.2 -> 60.6 without the post-RA pass, 60.7 -> 61.2 bottom-up; under max-ILP (the band
// pipeline's) 56.8 (profiles/r04/r04h_sched.jsonl).
using namespace golk;
const void *golk_bytes_pipe_fn(bool count)
{
    return count ? (const void *)BYTES_PIPE(true) : (const void *)BYTES_PIPE(false);
}
hipError_t golk_bytes_pipe_launch(bool count, unsigned nwg, const BytesKArgs &a, hipStream_t s)
{
    if (count) hipLaunchKernelGGL(BYTES_PIPE(true), dim3(nwg), dim3(64 * GOL_BYTES_PIPE_P), 0, s, a);
    else hipLaunchKernelGGL(BYTES_PIPE(false), dim3(nwg), dim3(64 * GOL_BYTES_PIPE_P), 0, s, a);
    return hipGetLastError();
}
#else  // the rest of the kernels and the host side

// ------------------------------------------------------------------ byte-board step (exact semantics)
// SWAR on 4 cells per uint32.  A = (byte == 255), Z = (byte == 0), as 0x01 per byte.
__device__ __forceinline__ uint32_t bytes_eq_ff(uint32_t d)
{
    const uint32_t x = ~d;
    const uint32_t nz = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;  // bit7 set where x byte != 0
    return (~nz >> 7) & 0x01010101u;
}
__device__ __forceinline__ uint32_t bytes_eq_00(uint32_t d)
{
    const uint32_t nz = ((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d;
    return (~nz >> 7) & 0x01010101u;
}

struct ByteRow {
    uint32_t a[4];  // (byte == 255) flags
    uint32_t z[4];  // (byte == 0) flags
    uint32_t hs[4]; // horizontal 3-sums of the a flags (0..3 per byte)
};

__device__ __forceinline__ void byte_row(const uint4 v, ByteRow &r)
{
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) { r.a[j] = bytes_eq_ff(d[j]); r.z[j] = bytes_eq_00(d[j]); }
    const uint32_t left_in = from_lower_lane(r.a[3]);
    const uint32_t right_in = from_upper_lane(r.a[0]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t wl = j == 0 ? left_in : r.a[j - 1];
        const uint32_t wr = j == 3 ? right_in : r.a[j + 1];
        const uint32_t L = __builtin_amdgcn_alignbyte(r.a[j], wl, 3);  // byte x-1 at byte x
        const uint32_t R = __builtin_amdgcn_alignbyte(wr, r.a[j], 1);  // byte x+1 at byte x
        r.hs[j] = L + r.a[j] + R;
    }
}

__device__ __forceinline__ uint32_t byte_rule(uint32_t hs_up, uint32_t hs_mid, uint32_t hs_dn, uint32_t a,
                                              uint32_t z)
{
    const uint32_t n = hs_up + hs_mid + hs_dn - a;                                   // neighbours, 0..8
    const uint32_t ne3 = ((n ^ 0x03030303u) + 0x7F7F7F7Fu) & 0x80808080u;           // n != 3
    const uint32_t ne23 = (((n | 0x01010101u) ^ 0x03030303u) + 0x7F7F7F7Fu) & 0x80808080u;  // n not in {2,3}
    const uint32_t born = z & ~(ne3 >> 7);
    const uint32_t surv = a & ~(ne23 >> 7);
    const uint32_t r = born | surv;  // 0x01 per byte
    return (r << 8) - r;             // 0xFF per byte
}

struct BytesArgs {
    const uint8_t *world;
    uint8_t *out;
    int64_t H, W, stride, out_stride, y0, y1;
    int32_t strip, ngroups;
};

// Wave = 62 lanes x 16 bytes of output per row; lanes 0/63 are halo.
__global__ void __launch_bounds__(256) bytes_step_kernel(BytesArgs a)
{
    const int lane = threadIdx.x & 63;
    const int group = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (group >= a.ngroups) return;
    const int64_t col_raw = (int64_t)group * (62 * 16) + (int64_t)(lane - 1) * 16;
    const int64_t col = ((col_raw % a.W) + a.W) % a.W;
    const bool writer = lane >= 1 && lane <= 62 && col_raw < a.W;

    const int64_t s0 = a.y0 + (int64_t)blockIdx.y * a.strip;
    const int64_t s1 = min(s0 + (int64_t)a.strip, a.y1);
    auto load = [&](int64_t y) -> uint4 {
        y = ((y % a.H) + a.H) % a.H;
        return *reinterpret_cast<const uint4 *>(a.world + y * a.stride + col);
    };
    ByteRow up, mid, dn;
    byte_row(load(s0 - 1), up);
    byte_row(load(s0), mid);
    uint4 nxt = load(s0 + 1);
    for (int64_t y = s0; y < s1; ++y) {
        byte_row(nxt, dn);
        nxt = load(y + 2);  // prefetch (wraps harmlessly past the strip)
        if (writer) {
            uint4 o;
            o.x = byte_rule(up.hs[0], mid.hs[0], dn.hs[0], mid.a[0], mid.z[0]);
            o.y = byte_rule(up.hs[1], mid.hs[1], dn.hs[1], mid.a[1], mid.z[1]);
            o.z = byte_rule(up.hs[2], mid.hs[2], dn.hs[2], mid.a[2], mid.z[2]);
            o.w = byte_rule(up.hs[3], mid.hs[3], dn.hs[3], mid.a[3], mid.z[3]);
            *reinterpret_cast<uint4 *>(a.out + (y - a.y0) * a.out_stride + col) = o;
        }
        up = mid;
        mid = dn;
    }
}

// Widths that are not a multiple of 16 (one thread per cell), a literal restatement of
// worker.go:26-37 / 44-70.
__global__ void bytes_step_scalar_kernel(BytesArgs a)
{
    const int64_t n = (a.y1 - a.y0) * a.W;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = a.y0 + i / a.W, x = i % a.W;
        const int64_t ya = (y + a.H - 1) % a.H, yb = (y + 1) % a.H;
        const int64_t xl = (x + a.W - 1) % a.W, xr = (x + 1) % a.W;
        const uint8_t *w = a.world;
        const int64_t s = a.stride;
        int cnt = (w[ya * s + xl] == 255) + (w[ya * s + x] == 255) + (w[ya * s + xr] == 255) +
                  (w[y * s + xl] == 255) + (w[y * s + xr] == 255) + (w[yb * s + xl] == 255) +
                  (w[yb * s + x] == 255) + (w[yb * s + xr] == 255);
        const uint8_t c = w[y * s + x];
        uint8_t o = 0;
        if (c == 0 && cnt == 3) o = 255;
        if (c == 255 && (cnt == 2 || cnt == 3)) o = 255;
        a.out[(y - a.y0) * a.out_stride + x] = o;
    }
}

// ------------------------------------------------------------------ board utilities
// Synthetic board: 64-bit word (y, w) = splitmix64(seed ^ (y*Ww + w)).
__global__ void random_fill_kernel(uint32_t *dst, int64_t rows, int64_t grow0, int64_t Ww, int64_t pitch,
                                   uint64_t seed)
{
    const int64_t n = rows * Ww;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / Ww, w = i % Ww;
        const uint64_t v = splitmix64(seed ^ (uint64_t)((grow0 + y) * Ww + w));
        *reinterpret_cast<uint2 *>(dst + y * pitch + 2 * w) = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
    }
}

__global__ void popcount_kernel(const uint32_t *src, int64_t rows, int64_t Wd, int64_t pitch, uint64_t *slots)
{
    uint64_t c = 0;
    const int64_t n = rows * Wd;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / Wd, w = i % Wd;
        c += __popc(src[y * pitch + w]);
    }
    slot_add(slots, c);
}

// Sum the GOL_COUNT_SLOTS slots of `n` consecutive slot arrays into out[0..n) (one wave each).
__global__ void slots_reduce_kernel(uint64_t *slots, int64_t n, uint64_t *out)
{
    const int lane = threadIdx.x & 63;
    const int64_t i = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (i >= n) return;
    uint64_t s = 0;
    for (int j = lane; j < GOL_COUNT_SLOTS; j += 64) {
        uint64_t *p = &slots[(i * GOL_COUNT_SLOTS + j) * 8];
        s += *p;
        *p = 0;  // left zeroed: the next counted launch needs no memset (gol_engine.cpp slots_zero)
    }
    s = wave_sum_u64(s);
    if (lane == 0) out[i] = s;
}

__global__ void hash_kernel(const uint32_t *src, int64_t rows, int64_t grow0, int64_t Ww, int64_t pitch,
                            uint64_t *slots)
{
    uint64_t h = 0;
    const int64_t n = rows * Ww;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / Ww, w = i % Ww;
        const uint2 v = *reinterpret_cast<const uint2 *>(src + y * pitch + 2 * w);
        const uint64_t word = (uint64_t)v.x | ((uint64_t)v.y << 32);
        h += splitmix64(word ^ splitmix64((uint64_t)((grow0 + y) * Ww + w)));
    }
    slot_add(slots, h);
}

__global__ void count_nonzero_bytes_kernel(const uint8_t *src, int64_t rows, int64_t W, int64_t stride,
                                           uint64_t *slots)
{
    uint64_t c = 0;
    const int64_t n = rows * W;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / W, x = i % W;
        c += src[y * stride + x] != 0;
    }
    slot_add(slots, c);
}

// flag |= 1 if any byte of the rows x W board is neither 0 nor 255
__global__ void nonbinary_kernel(const uint8_t *bytes, int64_t rows, int64_t W, int64_t stride, uint32_t *flag)
{
    const int64_t n = rows * W;
    uint32_t bad = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t c = bytes[(i / W) * stride + i % W];
        bad |= (c != 0 && c != 255);
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

// bytes -> bits: one thread per 32-cell word
__global__ void pack_kernel(const uint8_t *bytes, int64_t rows, int64_t W, int64_t stride, uint32_t *bits,
                            int64_t pitch, uint32_t *nonbinary)
{
    const int64_t Wd = W / 32;
    const int64_t n = rows * Wd;
    uint32_t bad = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / Wd, w = i % Wd;
        const uint8_t *p = bytes + y * stride + 32 * w;
        uint32_t v = 0;
#pragma unroll 8
        for (int b = 0; b < 32; ++b) {
            const uint8_t c = p[b];
            v |= (uint32_t)(c == 255) << b;
            bad |= (c != 0 && c != 255);
        }
        bits[y * pitch + w] = v;
    }
    if (nonbinary && bad) atomicOr(nonbinary, 1u);
}

// bits -> bytes (0/255): one thread per 32-cell word, two 16-byte stores
__global__ void unpack_kernel(const uint32_t *bits, int64_t rows, int64_t W, int64_t pitch, uint8_t *bytes,
                              int64_t stride)
{
    const int64_t Wd = W / 32;
    const int64_t n = rows * Wd;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / Wd, w = i % Wd;
        const uint32_t v = bits[y * pitch + w];
        uint32_t o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t nib = (v >> (4 * q)) & 0xF;
            // spread 4 bits to 4 bytes, then 0x01 -> 0xFF
            const uint32_t s = (nib & 1) | ((nib & 2) << 7) | ((nib & 4) << 14) | ((nib & 8) << 21);
            o[q] = (s << 8) - s;
        }
        uint8_t *dst = bytes + y * stride + 32 * w;
        if (((uintptr_t)dst & 15) == 0) {
            reinterpret_cast<uint4 *>(dst)[0] = make_uint4(o[0], o[1], o[2], o[3]);
            reinterpret_cast<uint4 *>(dst)[1] = make_uint4(o[4], o[5], o[6], o[7]);
        } else {
            for (int q = 0; q < 8; ++q)
                for (int b = 0; b < 4; ++b) dst[4 * q + b] = (uint8_t)(o[q] >> (8 * b));
        }
    }
}

// Alive-cell list, row-major (broker.go:47-58): one wave per row, ballot + mbcnt prefix over
// 64 cells at a time.  offs[y] = first output index of row y.  With `prev` the listed cells
// are those that differ from `prev` (the CellFlipped events of one turn,
// gol/event.go:50-60): the same kernels over bits ^ prev.  y0 is the global row of row 0.
__global__ void alive_list_bits_kernel(const uint32_t *bits, const uint32_t *prev, int64_t rows, int64_t Wd,
                                       int64_t pitch, const int64_t *offs, int32_t *xy, int64_t cap, int64_t y0)
{
    const int lane = threadIdx.x & 63;
    const int64_t y = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (y >= rows) return;
    int64_t base = offs[y];
    for (int64_t w0 = 0; w0 < Wd; w0 += 64) {
        const int64_t w = w0 + lane;
        const uint32_t v = w < Wd ? bits[y * pitch + w] ^ (prev ? prev[y * pitch + w] : 0u) : 0u;
        const uint32_t c = __popc(v);
        // exclusive prefix of c over the wave
        uint32_t incl = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(incl, off, 64);
            if (lane >= off) incl += t;
        }
        int64_t o = base + (incl - c);
        uint32_t m = v;
        while (m) {
            const int b = __ffs(m) - 1;
            m &= m - 1;
            if (o < cap) { xy[2 * o] = (int32_t)(32 * w + b); xy[2 * o + 1] = (int32_t)(y0 + y); }
            ++o;
        }
        base += __shfl(incl, 63, 64);
    }
}

// bytes: a cell is alive when != 0 (broker.go:50-55); with `prev`, listed when its alive state
// differs from prev's.
__device__ __forceinline__ bool byte_listed(const uint8_t *bytes, const uint8_t *prev, int64_t i)
{
    return (bytes[i] != 0) != (prev ? prev[i] != 0 : false);
}

__global__ void alive_list_bytes_kernel(const uint8_t *bytes, const uint8_t *prev, int64_t rows, int64_t W,
                                        int64_t stride, const int64_t *offs, int32_t *xy, int64_t cap, int64_t y0)
{
    const int lane = threadIdx.x & 63;
    const int64_t y = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (y >= rows) return;
    int64_t base = offs[y];
    for (int64_t x0 = 0; x0 < W; x0 += 64) {
        const int64_t x = x0 + lane;
        const bool alive = x < W && byte_listed(bytes, prev, y * stride + x);
        const uint64_t m = __ballot(alive);
        if (alive) {
            const int64_t o = base + __popcll(m & ((1ULL << lane) - 1));
            if (o < cap) { xy[2 * o] = (int32_t)x; xy[2 * o + 1] = (int32_t)(y0 + y); }
        }
        base += __popcll(m);
    }
}

__global__ void row_counts_bits_kernel(const uint32_t *bits, const uint32_t *prev, int64_t rows, int64_t Wd,
                                       int64_t pitch, int64_t *out)
{
    const int lane = threadIdx.x & 63;
    const int64_t y = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (y >= rows) return;
    uint64_t c = 0;
    for (int64_t w = lane; w < Wd; w += 64) c += __popc(bits[y * pitch + w] ^ (prev ? prev[y * pitch + w] : 0u));
    c = wave_sum_u64(c);
    if (lane == 0) out[y] = (int64_t)c;
}

__global__ void row_counts_bytes_kernel(const uint8_t *bytes, const uint8_t *prev, int64_t rows, int64_t W,
                                        int64_t stride, int64_t *out)
{
    const int lane = threadIdx.x & 63;
    const int64_t y = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (y >= rows) return;
    uint64_t c = 0;
    for (int64_t x = lane; x < W; x += 64) c += byte_listed(bytes, prev, y * stride + x);
    c = wave_sum_u64(c);
    if (lane == 0) out[y] = (int64_t)c;
}

}  // namespace golk

// ------------------------------------------------------------------ IPC sequence flags
// The IPC halo transport (gol_ipc.cpp): a rank's flag words live in its own HBM and are polled by
// its ring neighbours' kernels through IPC mappings (other processes, the same or another GPU).
// Stream order puts a signal after the launches whose rows it announces (their end-of-kernel
// release has written them back), and the copy after the wait that acquired the flag.
__global__ void ipc_signal_kernel(uint32_t *flag, uint32_t value)
{
    if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct IpcWaitArgs {
    const uint32_t *f0, *f1, *f2, *f3;
    int32_t n;
    uint32_t want;
    uint64_t timeout;
    uint32_t *err;
};

// Lane i < n polls flag i (a bounded wait: every lane leaves, with or without the flag).
__global__ void ipc_wait_kernel(IpcWaitArgs a)
{
    const int lane = threadIdx.x;
    bool ok = true;
    if (lane < a.n) {
        const uint32_t *f = lane == 0 ? a.f0 : (lane == 1 ? a.f1 : (lane == 2 ? a.f2 : a.f3));
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            const uint32_t v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((int32_t)(v - a.want) >= 0) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
    }
    if (!ok) atomicOr(a.err, GOLK_ERR_IPC);
}

// ------------------------------------------------------------------ launchers
using namespace golk;

// Rows per wave strip are capped so a lane's 32-bit alive count cannot overflow.
constexpr int GOL_MAX_STRIP = 1 << 24;

static inline int grid_for(int64_t n, int block = 256, int64_t cap = 256 * 16)
{
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// Per-device error word used when a launcher is called without one (gol_dev_* launchers).
uint32_t *golk_device_err_word(int device)
{
    static std::mutex mu;
    static std::map<int, uint32_t *> words;
    std::lock_guard<std::mutex> lock(mu);
    auto it = words.find(device);
    if (it != words.end()) return it->second;
    int prev = 0;
    uint32_t *w = nullptr;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return nullptr;
    // zeroed and synchronised: launches on non-blocking streams are not ordered after the null stream
    if (hipMalloc(&w, sizeof(uint32_t)) != hipSuccess || hipMemset(w, 0, sizeof(uint32_t)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)
        w = nullptr;
    (void)hipSetDevice(prev);
    if (w) words[device] = w;
    return w;
}

// Per-device CU slot masks of the band pipeline (GOL_BAND_PLACE; zeroed once, every workgroup
// frees its slot on exit).
uint32_t *golk_cu_slots(int device)
{
    static std::mutex mu;
    static std::map<int, uint32_t *> tabs;
    std::lock_guard<std::mutex> lock(mu);
    auto it = tabs.find(device);
    if (it != tabs.end()) return it->second;
    int prev = 0;
    uint32_t *w = nullptr;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return nullptr;
    if (hipMalloc(&w, GOL_CU_SLOT_WORDS * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(w, 0, GOL_CU_SLOT_WORDS * sizeof(uint32_t)) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        w = nullptr;
    (void)hipSetDevice(prev);
    if (w) tabs[device] = w;
    return w;
}

hipError_t golk_reset_cu_slots(int device, hipStream_t s)
{
    uint32_t *w = golk_cu_slots(device);
    return w ? hipMemsetAsync(w, 0, GOL_CU_SLOT_WORDS * sizeof(uint32_t), s) : hipErrorOutOfMemory;
}

static uint32_t *err_or_default(uint32_t *err)
{
    if (err) return err;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    return golk_device_err_word(dev);
}

template <int K, int DW>
static hipError_t launch_bits(const BitsArgs &a, hipStream_t s)
{
    const int nstrips = (int)((a.rows + a.strip - 1) / a.strip);
    dim3 grid((a.ngroups + 3) / 4, nstrips);
    hipLaunchKernelGGL((bits_step_kernel<K, DW>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

template <int DW>
static hipError_t launch_bits_k(int k, const BitsArgs &a, hipStream_t s)
{
    switch (k) {
    case 1: return launch_bits<1, DW>(a, s);
    case 2: return launch_bits<2, DW>(a, s);
    case 4: return launch_bits<4, DW>(a, s);
    case 8: return launch_bits<8, DW>(a, s);
    case 16: if constexpr (DW <= 2) return launch_bits<16, DW>(a, s);
             return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
    }
}

int golk_auto_strip(int64_t rows, int64_t ngroups, int k)
{
    // aim for >= ~8192 waves (32 per CU) but no longer than 64*k rows: the 2k halo rows then
    // cost <= 1/32 (measured best on the 2^17 x 2^20 torus: 512 rows at k = 8, 1024 at k = 16)
    int64_t strip = rows * ngroups / 8192;
    const int64_t hi = 64 * (int64_t)k;
    if (strip > hi) strip = hi;
    int64_t lo = 8 * (int64_t)k;
    if (lo < 32) lo = 32;
    // a board too small for ~512 strips of lo rows (the reference's images: 512^2 is one column
    // group) is latency-bound: a launch lasts one wave's serial walk over strip + 2k rows, so
    // ~512 short strips win (512^2, k = 8: strip 1-2 -> 2.3 us per turn, 64 -> 5.8;
    // profiles/r03/r03q_small.jsonl)
    if (rows * ngroups < lo * 512) lo = std::max<int64_t>(1, rows * ngroups / 512);
    if (strip < lo) strip = lo;
    if (strip > rows) strip = rows;
    if (strip < 1) strip = 1;
    return (int)strip;
}

// Workgroups of `kernel` (block threads) resident on the whole device at once (cached).
static int64_t resident_workgroups(const void *kernel, int block)
{
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, int64_t> cache;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({kernel, dev});
    if (it != cache.end()) return it->second;
    int64_t n = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0) == hipSuccess)
        n = (int64_t)cus * per_cu;
    cache[{kernel, dev}] = n;
    return n;
}

// Strip length for a one-workgroup-per-(column group, strip) kernel on a board that fills the
// device only a few times over: the strip count is a multiple of the strips that fit in one
// round of resident workgroups, so the last round is not a small remainder (e.g. 65536^2 at
// k = 12: 9 groups x 228 strips = 2052 workgroups was 2 rounds + 4 workgroups).  Boards of
// many rounds keep `fallback` (their tail is a small fraction already).
static int64_t round_tiled_strip(int64_t rows, int64_t ngroups, int64_t slots, int64_t min_rows, int64_t cap,
                                 int64_t fallback)
{
    if (slots <= 0 || rows <= 0) return fallback;
    const int64_t per_round = std::max<int64_t>(1, slots / ngroups);
    const int64_t rounds = (rows + per_round * cap - 1) / (per_round * cap);
    if (rounds > 4) return fallback;
    const int64_t nstrips = per_round * rounds;
    const int64_t strip = (rows + nstrips - 1) / nstrips;
    return std::min(rows, std::max(strip, min_rows));
}

hipError_t golk_bits_step(const uint32_t *top, const uint32_t *mid, const uint32_t *bot, uint32_t *dst,
                          int64_t R, int64_t Wd, int64_t pitch, int64_t row0, int64_t rows, int k, int dw,
                          int strip, uint64_t *slots, hipStream_t s)
{
    BitsArgs a;
    a.top = top; a.mid = mid; a.bot = bot; a.dst = dst;
    a.R = R; a.Wd = Wd; a.pitch = pitch; a.row0 = row0; a.rows = rows;
    a.ngroups = (int)((Wd + 62 * dw - 1) / (62 * dw));
    a.strip = strip > 0 ? std::min(strip, GOL_MAX_STRIP) : golk_auto_strip(rows, a.ngroups, k);
    a.slots = slots;
    a.sm = StripMap{};
    a.err = nullptr;  // no flag waits in this kernel
    a.cu_slots = nullptr;
    if (rows <= 0) return hipSuccess;
    switch (dw) {
    case 1: return launch_bits_k<1>(k, a, s);
    case 2: return launch_bits_k<2>(k, a, s);
    case 4: return launch_bits_k<4>(k, a, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DW, bool C>
static hipError_t launch_band(int k, dim3 grid, const BitsArgs &a, hipStream_t s)
{
    switch (k) {
    case 1: hipLaunchKernelGGL((band_step_kernel<1, DW, C>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((band_step_kernel<2, DW, C>), grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL((band_step_kernel<4, DW, C>), grid, dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL((band_step_kernel<8, DW, C>), grid, dim3(256), 0, s, a); break;
    case 12: if constexpr (DW <= 2) { hipLaunchKernelGGL((band_step_kernel<12, DW, C>), grid, dim3(256), 0, s, a); break; }
             return hipErrorInvalidValue;
    case 16: if constexpr (DW <= 2) { hipLaunchKernelGGL((band_step_kernel<16, DW, C>), grid, dim3(256), 0, s, a); break; }
             return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

static int device_cus()
{
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    return cus;
}

// Rank-weighted strips for a launch of exactly one round (StripMap): every CU takes one column
// group x `period` rows and its per_cu workgroups split them in proportion to `weight[rank]`,
// the measured relative speed of the rank-th arrival on a CU.  Used when the strips of one
// column group can be spread over the CUs with little waste (ngroups x strips per group >= 94 %
// of the CUs) and every rank still gets >= min_rows rows; else false (equal strips).
// Claim counters of the paired ranks (StripMap), one zeroed buffer per stream: launches on one
// stream run in order and leave their counters zeroed; launches on different streams may run
// at once and must not share counters.  The buffer is zeroed ON that stream (stream-ordered
// before the launch that asks for it): a null-stream hipMemset is not ordered before work on a
// non-blocking stream, and a first launch that raced it counted rows twice (overlapping claims;
// tests/test_gpu_engine.py::test_band_paired_narrow_board).  A launch that faults (a pipeline
// wave timed out) can leave counters set: golk_reset_claims zeroes a device's buffers again.
static std::mutex claims_mu;
static std::map<std::pair<hipStream_t, int>, uint32_t *> claims_bufs;
static size_t claims_bytes(int cus) { return (size_t)cus * 2 * 16 * sizeof(uint32_t); }
static uint32_t *claim_counters(hipStream_t s, int cus)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(claims_mu);
    auto it = claims_bufs.find({s, dev});
    if (it != claims_bufs.end()) return it->second;
    uint32_t *c = nullptr;
    if (hipMalloc(&c, claims_bytes(cus)) != hipSuccess) return nullptr;
    if (hipMemsetAsync(c, 0, claims_bytes(cus), s) != hipSuccess) {
        (void)hipFree(c);
        return nullptr;
    }
    claims_bufs[{s, dev}] = c;
    return c;
}

static std::set<hipStream_t> engine_streams;  // streams owned by an engine (golk_own_stream)

hipError_t golk_reset_claims(hipStream_t s)
{
    std::lock_guard<std::mutex> lock(claims_mu);
    hipError_t e = hipSuccess;
    for (auto &kv : claims_bufs) {
        if (kv.first.first != s) continue;
        int cus = 0;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, kv.first.second);
        if (e == hipSuccess) e = hipMemsetAsync(kv.second, 0, claims_bytes(cus), s);  // before any later launch on s
        if (e != hipSuccess) break;
    }
    return e;
}

void golk_release_claims(hipStream_t s)
{
    std::lock_guard<std::mutex> lock(claims_mu);
    for (auto it = claims_bufs.begin(); it != claims_bufs.end();) {
        if (it->first.first == s) {
            (void)hipFree(it->second);
            it = claims_bufs.erase(it);
        } else {
            ++it;
        }
    }
    engine_streams.erase(s);
}

void golk_own_stream(hipStream_t s)
{
    std::lock_guard<std::mutex> lock(claims_mu);
    engine_streams.insert(s);
}

hipError_t golk_reset_claims_device(int device)
{
    // Synchronous, on the null stream between two device-wide synchronisations: a caller's stream
    // that owns a buffer here may have been destroyed since (its handle is not used), and the
    // second synchronisation orders the zeroing before any later launch on a non-blocking stream.
    std::lock_guard<std::mutex> lock(claims_mu);
    int cus = 0, prev = 0;
    hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e == hipSuccess) e = hipGetDevice(&prev);
    if (e == hipSuccess) e = hipSetDevice(device);
    if (e != hipSuccess) return e;
    e = hipDeviceSynchronize();
    for (auto &kv : claims_bufs) {
        if (e != hipSuccess) break;
        if (kv.first.second != device || engine_streams.count(kv.first.first)) continue;
        e = hipMemset(kv.second, 0, claims_bytes(cus));
    }
    if (e == hipSuccess) {
        uint32_t *w = golk_cu_slots(device);  // (placement only: a timed-out workgroup kept its slot)
        if (w) e = hipMemset(w, 0, GOL_CU_SLOT_WORDS * sizeof(uint32_t));
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    (void)hipSetDevice(prev);
    return e;
}

static bool rank_split(int64_t rows, int64_t ngroups, int cus, int per_cu, const double *weight, int64_t min_rows,
                       int64_t max_strip, StripMap &sm, bool paired, uint32_t *claims = nullptr, int chunk = 0,
                       int max_rounds = 2)
{
    if (cus <= 0 || cus % 8 || per_cu < 1 || per_cu > 4 || ngroups > cus || rows <= 0) return false;
    // only boards that fill the device at most max_rounds times with strips of max_strip rows: on
    // bigger boards workgroups refill the CUs as they finish, and only the last round has the tail
    if (ngroups * ((rows + max_strip - 1) / max_strip) > max_rounds * (int64_t)cus * per_cu) return false;
    const int64_t t = cus / ngroups;  // strips per column group, one CU each
    if (t * ngroups * 100 < (int64_t)cus * 94) return false;
    const int64_t period = (rows + t - 1) / t;
    double wsum = 0;
    for (int r = 0; r < per_cu; ++r) wsum += weight[r];
    StripMap m{};
    m.ranked = 1;
    m.cus = cus;
    m.per_cu = per_cu;
    m.period = (int32_t)period;
    if (paired && per_cu >= 2) {
        // pairs walking one range from both ends: per_cu 2: (0, 1); 3: (0, 2) + rank 1 alone;
        // 4: (0, 3) + (1, 2).  A pair's range gets the sum of its ranks' weights.
        static const int pa[4][2] = {{0, 0}, {0, 0}, {0, 1}, {0, 2}};
        int ga[2][2];
        int ng = 0;
        if (per_cu == 4) { ga[0][0] = 0; ga[0][1] = 3; ga[1][0] = 1; ga[1][1] = 2; ng = 2; }
        else { ga[0][0] = pa[per_cu][0]; ga[0][1] = pa[per_cu][1]; ng = 1; }
        m.claims = claims;
        m.chunk = chunk;
        int64_t off = 0;
        double wused = 0;
        for (int g = 0; g < ng; ++g) {
            const double w = weight[ga[g][0]] + weight[ga[g][1]];
            wused += w;
            const int64_t len = (g == ng - 1 && per_cu != 3) ? period - off : (int64_t)(period * wused / wsum + 0.5) - off;
            if (len < min_rows) return false;
            for (int j = 0; j < 2; ++j) {
                const int r = ga[g][j];
                m.off[r] = (int32_t)off;
                m.len[r] = (int32_t)len;
                m.dir[r] = j == 0 ? 1 : -1;
                m.pslot[r] = g;
            }
            off += len;
        }
        if (per_cu == 3) {  // rank 1: the rest, a static strip
            if (period - off < min_rows) return false;
            m.off[1] = (int32_t)off;
            m.len[1] = (int32_t)(period - off);
        }
        sm = m;
        return true;
    }
    int64_t off = 0;
    for (int r = 0; r < per_cu; ++r) {
        const int64_t len = r == per_cu - 1 ? period - off : (int64_t)(period * weight[r] / wsum + 0.5);
        if (len < min_rows) return false;
        m.len[r] = (int32_t)len;
        m.off[r] = (int32_t)off;
        off += len;
    }
    sm = m;
    return true;
}

// Rows per arrival rank, from measurements (tools/timeline.py, same-box A/B with tools/ab.py):
// one round of equal strips ended the ranks' workgroups at T_r (band 247 / 298 / 388 / 482 us,
// bytes 96 / 136 / 174 us), so the static split gives rank r a share ~ 1 / T_r, refined by
// re-measuring (w_r <- w_r T_mean / T_r).  With paired ranks (StripMap) only the sum over a
// pair matters: band pairs (0, 3) and (1, 2) ran at equal speed (65536^2: 0.54 / 0.46 ended
// them at 425 / 360 us; 50 / 50: 110.3 TCUPS vs 106.2 for the static split, same box); bytes
// pair (0, 2) with rank 1 alone on 0.31 of the rows.
#ifndef GOL_BAND_RANK_W
#define GOL_BAND_RANK_W 0.25, 0.25, 0.25, 0.25
#endif
#ifndef GOL_BYTES_RANK_W
#define GOL_BYTES_RANK_W 0.4457, 0.33, 0.2449, 0.0  // lone rank 1: 0.31 -> 0.33 after the fill skip (+1.3 %)
#endif
static const double BAND_PIPE_RANK_W[4] = {GOL_BAND_RANK_W};
static const double BYTES_PIPE_RANK_W[4] = {GOL_BYTES_RANK_W};

// Rounds of short tail strips (StripMap.tail_*), 1 / GOL_BAND_TAIL_DIV of a strip's rows each.
// Round 3, half-length strips, same box, 2^17 x 2^20: none 137.2 TCUPS, 0.5 round 138.8, 1.0
// 138.8, 1.5 138.6; 262144^2: 132.2 / 133.6 / 133.2 / 133.0.  Round 6, weak board, two boxes, 3 + 4
// reps against half-length strips for 0.5 round: quarter-length strips for 1 round +0.5 / +0.6 %,
// for 0.5 round +0.1 %, 0.25 round -1.1 %, 1.5 rounds -0.4 %; third-length -0.3 %, eighth-length
// -0.1 % (profiles/r06/r06_ab_tail.log).
#ifndef GOL_BAND_TAIL
#define GOL_BAND_TAIL 1.0
#endif
#ifndef GOL_BAND_TAIL_DIV
#define GOL_BAND_TAIL_DIV 4
#endif
#ifndef GOL_BAND_PAIRED
#define GOL_BAND_PAIRED 1
#endif
#ifndef GOL_BYTES_PAIRED
#define GOL_BYTES_PAIRED 1
#endif
// bytes_pipe_kernel lives in its own translation unit (gol_bytes_pipe.hip: another scheduler)
const void *golk_bytes_pipe_fn(bool count);
hipError_t golk_bytes_pipe_launch(bool count, unsigned nwg, const BytesKArgs &a, hipStream_t s);
// Rows per strip of the band pipeline's launches of many rounds (same box, weak board, 3 reps:
// 1024 148.4 TCUPS, 2048 148.3, 4096 147.0; profiles/r04/r04d_ab_rounds.jsonl)
#ifndef GOL_BAND_STRIP
#define GOL_BAND_STRIP 1024
#endif
// Band launches of up to this many rounds of strips run as one round of rank-weighted, paired
// ranges instead, when their column groups spread over the CUs (rank_split).  Same box, 3 reps
// each: config 4's N = 4 share 65536 x 262144 (2.95 rounds of 781-row strips) 134.2 -> 148.3
// TCUPS at 4 rounds; at 16 rounds the N = 2 share 131072 x 262144 (4.5 rounds) 142.0 -> 150.2
// and the whole 262144^2 board (9 rounds) 145.3 -> 149.4 (profiles/r04/r04d_ab_*.jsonl).  The
// weak board's 133 column groups spread over 256 CUs only one per CU (52 %): strips.
#ifndef GOL_BAND_RANK_ROUNDS
#define GOL_BAND_RANK_ROUNDS 16
#endif
static constexpr int BAND_RANK_ROUNDS = GOL_BAND_RANK_ROUNDS;
static constexpr int BYTES_PIPE_P = GOL_BYTES_PIPE_P;

// The band pipeline's one-round launch (rank_split) of `rows` rows, when it applies; claims:
// the paired ranks' counters (null: only ask whether it applies).
static bool band_rank_map(int64_t rows, int64_t ngroups, int64_t pitch, int cus, int64_t slots, uint32_t *claims,
                          StripMap &sm)
{
    constexpr int KW = GOL_BAND_KW, P = GOL_BAND_P;
    if (cus <= 0 || slots <= 0) return false;
    StripMap m{};
    if (!rank_split(rows, ngroups, cus, (int)(slots / cus), BAND_PIPE_RANK_W, 8 * KW * P, 1024, m, GOL_BAND_PAIRED,
                    claims, GOL_BAND_NS, BAND_RANK_ROUNDS))
        return false;
    if ((int64_t)m.period * pitch * 4 >= (int64_t(1) << 31)) return false;  // a range's stores: one 32-bit buffer
    sm = m;
    return true;
}

// band_pipe_kernel lives in its own translation unit (gol_band_pipe.hip: another scheduler)
const void *golk_band_pipe_fn(bool contig, bool count);
hipError_t golk_band_pipe_launch(bool contig, bool count, unsigned nwg, const BitsArgs &a, hipStream_t s);

// k = 12 on the band layout: 4 waves x 3 stages (band_pipe_kernel).
static hipError_t launch_band_pipe(bool contig, BitsArgs a, hipStream_t s, bool auto_strip)
{
    constexpr int KW = GOL_BAND_KW, P = GOL_BAND_P;
    const bool count = a.slots != nullptr;
    const void *kf = golk_band_pipe_fn(contig, count);
    int64_t nwg = 0;
    const int cus = device_cus();
    const int64_t slots = resident_workgroups(kf, 64 * P);
    uint32_t *claims = auto_strip && GOL_BAND_PAIRED && cus > 0 ? claim_counters(s, cus) : nullptr;
    if (auto_strip && (claims || !GOL_BAND_PAIRED) && band_rank_map(a.rows, a.ngroups, a.pitch, cus, slots, claims, a.sm)) {
        nwg = (int64_t)cus * a.sm.per_cu;
    } else {
        if (auto_strip) a.strip = (int)round_tiled_strip(a.rows, a.ngroups, slots, 8 * KW * P, 1024, a.strip);
        nwg = (int64_t)a.ngroups * ((a.rows + a.strip - 1) / a.strip);
        if (auto_strip && GOL_BAND_TAIL > 0 && slots > 0 && nwg > 4 * slots) {
            // the last ~GOL_BAND_TAIL rounds of workgroups run strips of 1 / GOL_BAND_TAIL_DIV of the rows
            const int64_t ts = std::max<int64_t>(8 * KW * P, a.strip / GOL_BAND_TAIL_DIV);
            const int64_t nt = (int64_t)(GOL_BAND_TAIL * (double)slots / a.ngroups + 0.999);  // tail strips per group
            const int64_t tail_rows = std::min<int64_t>(a.rows / 2, nt * ts);
            const int64_t big = a.rows - tail_rows;
            const int64_t nbig = (big + a.strip - 1) / a.strip;
            a.sm.tail_l = (int32_t)(a.ngroups * nbig);
            a.sm.tail_row = (int32_t)big;
            a.sm.tail_strip = (int32_t)ts;
            nwg = a.sm.tail_l + a.ngroups * ((tail_rows + ts - 1) / ts);
        }
    }
    return golk_band_pipe_launch(contig, count, (unsigned)nwg, a, s);
}

hipError_t golk_band_step(const uint32_t *top, const uint32_t *mid, const uint32_t *bot, uint32_t *dst, int64_t R,
                          int64_t Wd, int64_t pitch, int64_t row0, int64_t rows, int k, int dw, int strip,
                          uint64_t *slots, uint32_t *err, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    BitsArgs a;
    a.top = top; a.mid = mid; a.bot = bot; a.dst = dst;
    a.R = R; a.Wd = Wd; a.pitch = pitch; a.row0 = row0; a.rows = rows;
    a.slots = slots;
    a.sm = StripMap{};
    a.err = err_or_default(err);
    if (!a.err) return hipErrorOutOfMemory;
    a.cu_slots = nullptr;
    if (GOL_BAND_PLACE) {
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess) a.cu_slots = golk_cu_slots(dev);
    }
    const bool contig = top + (int64_t)k * pitch == mid && bot == mid + R * pitch;
    const int U = band_useful_words(k, dw);
    a.ngroups = (int)((Wd + U - 1) / U);
    if (dw == 4 && k == GOL_BAND_KW * GOL_BAND_P) {
        // one workgroup per (column group, strip): strips up to 1024 rows (measured best at k = 12)
        // Boards with fewer than ~256 tiles of 8k rows are latency-bound (a launch lasts one
        // pipeline's walk over strip + 2k rows): ~512 tiles of >= 2 rows instead, without the
        // one-round rank split (1024^2: 2.6 us per turn vs 5.1 at 96 rows; 4096^2: 3.0 vs 5.2;
        // 8192^2: 4.1 vs 5.3; 16384^2 keeps the rank split: 6.0 vs 6.4 with 96-row tiles;
        // profiles/r03/r03q_small.jsonl)
        const int64_t work = rows * a.ngroups;
        const bool small = strip <= 0 && work < (int64_t)8 * k * 256;
        if (small)
            a.strip = (int)std::min<int64_t>(rows, std::max<int64_t>(2, work / 512));
        else
            a.strip = strip > 0 ? std::min(strip, GOL_MAX_STRIP)
                                : (int)std::min<int64_t>(rows, std::max<int64_t>(8 * k, std::min<int64_t>(GOL_BAND_STRIP, rows * a.ngroups / 2048)));
        // the pipe kernel's stores address a strip as one buffer (32-bit range)
        a.strip = (int)std::max<int64_t>(1, std::min<int64_t>(a.strip, (int64_t(1) << 30) / (pitch * 4)));
        return launch_band_pipe(contig, a, s, strip <= 0 && !small);
    }
    a.strip = strip > 0 ? std::min(strip, GOL_MAX_STRIP) : golk_auto_strip(rows, a.ngroups, k);
    dim3 grid((a.ngroups + 3) / 4, (int)((rows + a.strip - 1) / a.strip));
    if (dw == 2) return contig ? launch_band<2, true>(k, grid, a, s) : launch_band<2, false>(k, grid, a, s);
    if (dw == 4) return contig ? launch_band<4, true>(k, grid, a, s) : launch_band<4, false>(k, grid, a, s);
    return hipErrorInvalidValue;
}

int golk_band_useful_words(int k, int dw) { return band_useful_words(k, dw); }

double golk_step_rounds(bool band, int64_t rows, int64_t Wd, int64_t pitch, int k, int dw, int strip)
{
    if (!band || dw != 4 || k != GOL_BAND_KW * GOL_BAND_P || rows <= 0) return 1e9;
    const int64_t ngroups = (Wd + band_useful_words(k, dw) - 1) / band_useful_words(k, dw);
    const int64_t slots = resident_workgroups(golk_band_pipe_fn(true, true), 64 * GOL_BAND_P);
    if (slots <= 0) return 1e9;
    StripMap sm{};
    if (strip <= 0 && band_rank_map(rows, ngroups, pitch, device_cus(), slots, nullptr, sm)) return 1.0;
    const int64_t st = strip > 0 ? strip : GOL_BAND_STRIP;  // launch_band_pipe's strips
    return (double)(ngroups * ((rows + st - 1) / st)) / (double)slots;
}

hipError_t golk_band_convert(bool to_band, const uint32_t *src, uint32_t *dst, int64_t rows, int64_t Wd,
                             int64_t spitch, int64_t dpitch, hipStream_t s)
{
    const int64_t Wm = Wd / 32;
    if (rows <= 0) return hipSuccess;
    const dim3 g(grid_for(rows * Wm, 256, 256 * 64));
    if (to_band)
        hipLaunchKernelGGL(band_convert_kernel<true>, g, dim3(256), 0, s, src, dst, rows, Wm, spitch, dpitch);
    else
        hipLaunchKernelGGL(band_convert_kernel<false>, g, dim3(256), 0, s, src, dst, rows, Wm, spitch, dpitch);
    return hipGetLastError();
}

hipError_t golk_bytes_step(const uint8_t *world, int64_t H, int64_t W, int64_t stride, int64_t y0, int64_t y1,
                           uint8_t *out, int64_t out_stride, hipStream_t s)
{
    BytesArgs a;
    a.world = world; a.out = out; a.H = H; a.W = W; a.stride = stride; a.out_stride = out_stride;
    a.y0 = y0; a.y1 = y1;
    if (y1 <= y0) return hipSuccess;
    const bool vec = (W % 16 == 0) && (stride % 16 == 0) && (out_stride % 16 == 0) &&
                     (((uintptr_t)world & 15) == 0) && (((uintptr_t)out & 15) == 0);
    if (vec) {
        a.ngroups = (int)((W + 62 * 16 - 1) / (62 * 16));
        const int64_t rows = y1 - y0;
        int64_t strip = rows * a.ngroups / 8192;
        if (strip < 16) strip = 16;
        if (strip > 256) strip = 256;
        if (strip > rows) strip = rows;
        a.strip = (int)strip;
        dim3 grid((a.ngroups + 3) / 4, (int)((rows + strip - 1) / strip));
        hipLaunchKernelGGL(bytes_step_kernel, grid, dim3(256), 0, s, a);
    } else {
        a.ngroups = 0; a.strip = 0;
        hipLaunchKernelGGL(bytes_step_scalar_kernel, dim3(grid_for((y1 - y0) * W)), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t golk_bytes_blocked(const uint8_t *top, const uint8_t *mid, const uint8_t *bot, uint8_t *dst, int64_t R,
                              int64_t W, int64_t pitch, int64_t row0, int64_t rows, int k, int strip, uint64_t *slots,
                              uint32_t *err, hipStream_t s)
{
    BytesKArgs a;
    a.top = top; a.mid = mid; a.bot = bot; a.dst = dst;
    a.R = R; a.Wd = W / 32; a.pitch = pitch; a.row0 = row0; a.rows = rows;
    a.ngroups = (int)((a.Wd + 61) / 62);
    a.strip = strip > 0 ? std::min(strip, GOL_MAX_STRIP) : golk_auto_strip(rows, a.ngroups, k);
    a.slots = slots;
    a.err = err_or_default(err);
    if (rows <= 0) return hipSuccess;
    if (!a.err) return hipErrorOutOfMemory;
    a.sm = StripMap{};
    if (k == 32) {
        // one workgroup of GOL_BYTES_PIPE_P waves per (column group, strip): rank-weighted strips
        // in one round, else round-tiled strips >= 4k rows
        const bool count = a.slots != nullptr;
        const void *kf = golk_bytes_pipe_fn(count);
        const int cus = device_cus();
        const int64_t slots = resident_workgroups(kf, 64 * BYTES_PIPE_P);
        int64_t nwg = 0;
        uint32_t *claims = GOL_BYTES_PAIRED ? claim_counters(s, cus) : nullptr;
        // the last wave stores a strip through one buffer descriptor: strip rows x pitch < 2^31
        const int64_t max_rows = std::max<int64_t>(1, ((int64_t(1) << 31) - 1) / pitch - 1);
        if (strip <= 0 && cus > 0 &&
            rank_split(rows, a.ngroups, cus, (int)std::min<int64_t>(GOL_BYTES_PER_CU, slots / cus), BYTES_PIPE_RANK_W,
                       2 * k, 1024, a.sm, claims != nullptr, claims, GOL_BYTES_NS) && a.sm.period <= max_rows) {
            nwg = (int64_t)cus * a.sm.per_cu;
        } else {
            a.sm = StripMap{};
            if (strip <= 0) {
                a.strip = (int)std::min<int64_t>(rows, std::max<int64_t>(8 * k, rows * a.ngroups / 1024));
                a.strip = (int)round_tiled_strip(rows, a.ngroups, slots, 4 * k, 1024, a.strip);
            }
            a.strip = (int)std::min<int64_t>(a.strip, max_rows);
            nwg = (int64_t)a.ngroups * ((rows + a.strip - 1) / a.strip);
        }
        return golk_bytes_pipe_launch(count, (unsigned)nwg, a, s);
    }
    const int nstrips = (int)((rows + a.strip - 1) / a.strip);
    dim3 grid((a.ngroups + 3) / 4, nstrips);
    switch (k) {
    case 1: hipLaunchKernelGGL(bytes_blocked_kernel<1>, grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(bytes_blocked_kernel<2>, grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL(bytes_blocked_kernel<4>, grid, dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL(bytes_blocked_kernel<8>, grid, dim3(256), 0, s, a); break;
    case 16: hipLaunchKernelGGL(bytes_blocked_kernel<16>, grid, dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t golk_nonbinary(const uint8_t *bytes, int64_t rows, int64_t W, int64_t stride, uint32_t *flag, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(nonbinary_kernel, dim3(grid_for(rows * W, 256, 256 * 16)), dim3(256), 0, s, bytes, rows, W, stride,
                       flag);
    return hipGetLastError();
}

hipError_t golk_random_fill(uint32_t *dst, int64_t rows, int64_t grow0, int64_t W, int64_t pitch, uint64_t seed,
                            hipStream_t s)
{
    const int64_t Ww = W / 64;
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(random_fill_kernel, dim3(grid_for(rows * Ww, 256, 256 * 64)), dim3(256), 0, s, dst, rows,
                       grow0, Ww, pitch, seed);
    return hipGetLastError();
}

hipError_t golk_popcount(const uint32_t *src, int64_t rows, int64_t Wd, int64_t pitch, uint64_t *slots, hipStream_t s)
{
    hipLaunchKernelGGL(popcount_kernel, dim3(grid_for(rows * Wd, 256, 256 * 16)), dim3(256), 0, s, src, rows, Wd,
                       pitch, slots);
    return hipGetLastError();
}

hipError_t golk_slots_reduce(uint64_t *slots, int64_t n, uint64_t *out, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(slots_reduce_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, slots, n, out);
    return hipGetLastError();
}

hipError_t golk_hash(const uint32_t *src, int64_t rows, int64_t grow0, int64_t Wd, int64_t pitch, uint64_t *slots,
                     hipStream_t s)
{
    hipLaunchKernelGGL(hash_kernel, dim3(grid_for(rows * (Wd / 2), 256, 256 * 16)), dim3(256), 0, s, src, rows,
                       grow0, Wd / 2, pitch, slots);
    return hipGetLastError();
}

hipError_t golk_count_bytes(const uint8_t *src, int64_t rows, int64_t W, int64_t stride, uint64_t *slots,
                            hipStream_t s)
{
    hipLaunchKernelGGL(count_nonzero_bytes_kernel, dim3(grid_for(rows * W, 256, 256 * 16)), dim3(256), 0, s, src,
                       rows, W, stride, slots);
    return hipGetLastError();
}

hipError_t golk_pack(const uint8_t *bytes, int64_t rows, int64_t W, int64_t stride, uint32_t *bits, int64_t pitch,
                     uint32_t *nonbinary, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(pack_kernel, dim3(grid_for(rows * (W / 32), 256, 256 * 64)), dim3(256), 0, s, bytes, rows, W,
                       stride, bits, pitch, nonbinary);
    return hipGetLastError();
}

hipError_t golk_unpack(const uint32_t *bits, int64_t rows, int64_t W, int64_t pitch, uint8_t *bytes, int64_t stride,
                       hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_kernel, dim3(grid_for(rows * (W / 32), 256, 256 * 64)), dim3(256), 0, s, bits, rows, W,
                       pitch, bytes, stride);
    return hipGetLastError();
}

hipError_t golk_row_counts(bool bits_mode, const void *board, const void *prev, int64_t rows, int64_t width_units,
                           int64_t pitch, int64_t *out, hipStream_t s)
{
    const int wpb = 4;
    if (rows <= 0) return hipSuccess;
    dim3 grid((unsigned)((rows + wpb - 1) / wpb));
    if (bits_mode)
        hipLaunchKernelGGL(row_counts_bits_kernel, grid, dim3(64 * wpb), 0, s, (const uint32_t *)board,
                           (const uint32_t *)prev, rows, width_units, pitch, out);
    else
        hipLaunchKernelGGL(row_counts_bytes_kernel, grid, dim3(64 * wpb), 0, s, (const uint8_t *)board,
                           (const uint8_t *)prev, rows, width_units, pitch, out);
    return hipGetLastError();
}

hipError_t golk_alive_list(bool bits_mode, const void *board, const void *prev, int64_t rows, int64_t width_units,
                           int64_t pitch, const int64_t *offs, int32_t *xy, int64_t cap, int64_t y0, hipStream_t s)
{
    const int wpb = 4;
    if (rows <= 0) return hipSuccess;
    dim3 grid((unsigned)((rows + wpb - 1) / wpb));
    if (bits_mode)
        hipLaunchKernelGGL(alive_list_bits_kernel, grid, dim3(64 * wpb), 0, s, (const uint32_t *)board,
                           (const uint32_t *)prev, rows, width_units, pitch, offs, xy, cap, y0);
    else
        hipLaunchKernelGGL(alive_list_bytes_kernel, grid, dim3(64 * wpb), 0, s, (const uint8_t *)board,
                           (const uint8_t *)prev, rows, width_units, pitch, offs, xy, cap, y0);
    return hipGetLastError();
}

hipError_t golk_ipc_signal(uint32_t *flag, uint32_t value, hipStream_t s)
{
    hipLaunchKernelGGL(ipc_signal_kernel, dim3(1), dim3(64), 0, s, flag, value);
    return hipGetLastError();
}

hipError_t golk_ipc_wait(const uint32_t *const *flags, int n, uint32_t want, uint64_t timeout_ticks, uint32_t *err,
                         hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    if (n > GOLK_IPC_MAX_WAIT || !err) return hipErrorInvalidValue;
    IpcWaitArgs a;
    a.f0 = flags[0];
    a.f1 = n > 1 ? flags[1] : flags[0];
    a.f2 = n > 2 ? flags[2] : flags[0];
    a.f3 = n > 3 ? flags[3] : flags[0];
    a.n = n;
    a.want = want;
    a.timeout = timeout_ticks;
    a.err = err;
    hipLaunchKernelGGL(ipc_wait_kernel, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}
#endif  // GOL_TU_BAND_PIPE
#endif  // GOL_TU_BYTES_PIPE
