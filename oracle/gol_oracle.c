/*
 * gol_oracle.c -- CPU restatement of the reference Game-of-Life hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libgolhip.so, the
 * golhip Python package) links, loads or calls this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only
 * as the checker / the timed CPU baseline ("kind": "port").
 *
 * Parity is pinned against the reference's own fixtures (tests/golden/, copied
 * byte-for-byte from /root/reference/check and /root/reference/images):
 *   - check/images/{16,64,512}x{0,1,100}.pgm  (gol_test.go:24-28, pgm_test.go:19-23)
 *   - check/alive/{16,64,512}.csv turns 1..10000 (count_test.go:71-89)
 * The reference itself is Go and there is no Go toolchain in this image, so
 * oracle/_ref (a build of the reference) does not exist; see DESIGN.md.
 *
 * Two independent restatements live here:
 *   (1) oracle_next_state_slab / oracle_count_neighbours: a literal per-cell
 *       port of worker.go:15-70 (byte board, 255 = alive, exact "== 0" birth
 *       and "== 255" survival, every other byte becomes 0).
 *   (2) oracle_bits_*: a word-parallel B3/S23 on a 64-cells-per-uint64 torus,
 *       used for long runs (10,000-turn alive CSVs) and big random boards.
 *       It is cross-checked against (1) in tests/test_oracle.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

/* ------------------------------------------------------------------------ */
/* (1) literal port of worker.go                                             */
/* ------------------------------------------------------------------------ */

/* worker.go:44-70 calculateSurroundings.  The reference wraps BOTH axes with
 * len(world[0]) (the width); on the square boards it is defined for that is
 * the same as wrapping rows with H.  We wrap rows with H and columns with W. */
int oracle_count_neighbours(const uint8_t *world, int64_t H, int64_t W, int64_t stride,
                            int64_t row, int64_t col)
{
    int64_t above = row - 1, below = row + 1;          /* worker.go:46-52 */
    if (row == 0) above = H - 1;
    if (row == H - 1) below = 0;
    int64_t left = col - 1, right = col + 1;           /* worker.go:53-59 */
    if (col == 0) left = W - 1;
    if (col == W - 1) right = 0;
    const uint8_t n[8] = {                             /* worker.go:61-63 */
        world[above * stride + left], world[above * stride + col], world[above * stride + right],
        world[row * stride + left],                              world[row * stride + right],
        world[below * stride + left], world[below * stride + col], world[below * stride + right]};
    int count = 0;
    for (int i = 0; i < 8; i++)                        /* worker.go:64-68 */
        if (n[i] == 255) count++;
    return count;
}

/* worker.go:15-42 calculateNextState for rows [y0, y1) of the full board.
 * out has (y1-y0) rows of W bytes, row pitch out_stride. */
int oracle_next_state_slab(const uint8_t *world, int64_t H, int64_t W, int64_t stride,
                           int64_t y0, int64_t y1, uint8_t *out, int64_t out_stride)
{
    if (H <= 0 || W <= 0 || y0 < 0 || y1 > H || y0 > y1) return -1;
    for (int64_t y = 0; y < y1 - y0; y++) {
        uint8_t *o = out + y * out_stride;
        memset(o, 0, (size_t)W);                        /* worker.go:18-21 (make -> zero) */
        for (int64_t x = 0; x < W; x++) {
            uint8_t c = world[(y + y0) * stride + x];
            if (c == 0) {                               /* worker.go:26-30 */
                if (oracle_count_neighbours(world, H, W, stride, y + y0, x) == 3) o[x] = 255;
            }
            if (c == 255) {                             /* worker.go:31-37 */
                int s = oracle_count_neighbours(world, H, W, stride, y + y0, x);
                if (s < 2 || s > 3) o[x] = 0;
                if (s == 2 || s == 3) o[x] = c;
            }
        }
    }
    return 0;
}

/* broker.go:135-139 (even split) and broker.go:172-206 (uneven split): the
 * first H % T slabs get H/T + 1 rows, the rest H/T, in order. */
int oracle_partition(int64_t H, int64_t T, int64_t i, int64_t *y0, int64_t *y1)
{
    if (T <= 0 || i < 0 || i >= T || H < 0) return -1;
    if (H % T == 0) {
        *y0 = i * H / T;
        *y1 = (i + 1) * H / T;
        return 0;
    }
    int64_t rem = H % T, base = H / T;
    int64_t start = i * base + (i < rem ? i : rem);
    *y0 = start;
    *y1 = start + base + (i < rem ? 1 : 0);
    return 0;
}

/* broker.go:47-58 calculateAliveCells: row-major scan, "!= 0". xy receives
 * (x, y) pairs (util.Cell{X, Y}); returns the number of alive cells (which may
 * exceed cap; only the first cap pairs are written). */
int64_t oracle_alive_cells(const uint8_t *world, int64_t H, int64_t W, int64_t stride,
                           int64_t *xy, int64_t cap)
{
    int64_t n = 0;
    for (int64_t y = 0; y < H; y++)
        for (int64_t x = 0; x < W; x++)
            if (world[y * stride + x] != 0) {
                if (n < cap) { xy[2 * n] = x; xy[2 * n + 1] = y; }
                n++;
            }
    return n;
}

struct slab_job {
    const uint8_t *world; int64_t H, W, y0, y1; uint8_t *out;
};

static void *slab_thread(void *p)
{
    struct slab_job *j = (struct slab_job *)p;
    oracle_next_state_slab(j->world, j->H, j->W, j->W, j->y0, j->y1, j->out + j->y0 * j->W, j->W);
    return NULL;
}

/* broker.go:62-234 Operations.Run turn loop: `threads` slabs per turn, each
 * computed by the literal worker port (one pthread per slab mirrors one
 * worker process), gathered back in slab order.  world is H*W bytes,
 * contiguous; it is updated in place.  turns == 0 returns it unchanged. */
int oracle_run(uint8_t *world, int64_t H, int64_t W, int64_t turns, int64_t threads)
{
    if (threads <= 0 || H <= 0 || W <= 0 || turns < 0) return -1;
    uint8_t *next = (uint8_t *)malloc((size_t)(H * W));
    if (!next) return -2;
    struct slab_job *jobs = (struct slab_job *)calloc((size_t)threads, sizeof *jobs);
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof *tid);
    for (int64_t t = 0; t < turns; t++) {
        for (int64_t i = 0; i < threads; i++) {
            jobs[i].world = world; jobs[i].H = H; jobs[i].W = W; jobs[i].out = next;
            oracle_partition(H, threads, i, &jobs[i].y0, &jobs[i].y1);
            if (threads == 1) slab_thread(&jobs[i]);
            else pthread_create(&tid[i], NULL, slab_thread, &jobs[i]);
        }
        if (threads > 1)
            for (int64_t i = 0; i < threads; i++) pthread_join(tid[i], NULL);
        memcpy(world, next, (size_t)(H * W));
    }
    free(tid); free(jobs); free(next);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* (2) word-parallel restatement on a bit-packed torus                        */
/*     layout: 64 cells per uint64, bit b of word w of row y is cell           */
/*     x = 64*w + b (LSB = lowest x), rows contiguous, W/64 words per row.     */
/* ------------------------------------------------------------------------ */

static inline uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t oracle_splitmix64(uint64_t x) { return splitmix64(x); }

/* Synthetic board: word(y, w) = splitmix64(seed ^ (y*Ww + w)),
 * Bernoulli(1/2) per cell.  Rows [y0, y0+rows) of a board Ww words wide. */
void oracle_random_words(uint64_t seed, int64_t y0, int64_t rows, int64_t Ww, uint64_t *out)
{
    for (int64_t y = 0; y < rows; y++)
        for (int64_t w = 0; w < Ww; w++)
            out[y * Ww + w] = splitmix64(seed ^ (uint64_t)((y0 + y) * Ww + w));
}

/* Order-independent board hash: sum over words of splitmix64(word ^ splitmix64(index)).
 * Row shards can be hashed separately (y0 = the shard's first global row) and summed. */
uint64_t oracle_hash_words(const uint64_t *words, int64_t y0, int64_t rows, int64_t Ww)
{
    uint64_t h = 0;
    for (int64_t y = 0; y < rows; y++)
        for (int64_t w = 0; w < Ww; w++) {
            uint64_t idx = (uint64_t)((y0 + y) * Ww + w);
            h += splitmix64(words[y * Ww + w] ^ splitmix64(idx));
        }
    return h;
}

uint64_t oracle_popcount_words(const uint64_t *words, int64_t n)
{
    uint64_t c = 0;
    for (int64_t i = 0; i < n; i++) c += (uint64_t)__builtin_popcountll(words[i]);
    return c;
}

/* byte board ({0,255}) <-> bit words; pack treats exactly 255 as alive. */
void oracle_pack(const uint8_t *bytes, int64_t H, int64_t W, int64_t stride, uint64_t *words)
{
    int64_t Ww = W / 64;
    for (int64_t y = 0; y < H; y++)
        for (int64_t w = 0; w < Ww; w++) {
            uint64_t v = 0;
            for (int b = 0; b < 64; b++)
                if (bytes[y * stride + 64 * w + b] == 255) v |= 1ULL << b;
            words[y * Ww + w] = v;
        }
}

void oracle_unpack(const uint64_t *words, int64_t H, int64_t W, uint8_t *bytes, int64_t stride)
{
    int64_t Ww = W / 64;
    for (int64_t y = 0; y < H; y++)
        for (int64_t x = 0; x < W; x++)
            bytes[y * stride + x] = ((words[y * Ww + x / 64] >> (x % 64)) & 1) ? 255 : 0;
}

/* One B3/S23 generation on the torus, word-parallel: count the 8 neighbours
 * with bit-sliced adders, alive' = (n == 3) | (alive & n == 2). */
static void bits_generation(const uint64_t *src, uint64_t *dst, int64_t H, int64_t Ww)
{
    for (int64_t y = 0; y < H; y++) {
        const uint64_t *ra = src + ((y + H - 1) % H) * Ww;
        const uint64_t *rc = src + y * Ww;
        const uint64_t *rb = src + ((y + 1) % H) * Ww;
        for (int64_t w = 0; w < Ww; w++) {
            int64_t wl = (w + Ww - 1) % Ww, wr = (w + 1) % Ww;
            uint64_t nb[8];
            const uint64_t *rows[3] = {ra, rc, rb};
            int k = 0;
            for (int r = 0; r < 3; r++) {
                uint64_t c = rows[r][w];
                uint64_t l = (c << 1) | (rows[r][wl] >> 63);   /* neighbour at x-1 */
                uint64_t rr = (c >> 1) | (rows[r][wr] << 63);  /* neighbour at x+1 */
                nb[k++] = l;
                nb[k++] = rr;
                if (r != 1) nb[k++] = c;
            }
            /* bit-sliced sum of 8 one-bit inputs -> s0, s1, s2 (count mod 8) and s3 (count >= 8) */
            uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
            for (int i = 0; i < 8; i++) {
                uint64_t c0 = s0 & nb[i];
                s0 ^= nb[i];
                uint64_t c1 = s1 & c0;
                s1 ^= c0;
                uint64_t c2 = s2 & c1;
                s2 ^= c1;
                s3 |= c2;
            }
            uint64_t alive = rc[w];
            uint64_t is3 = s0 & s1 & ~s2 & ~s3;
            uint64_t is2 = ~s0 & s1 & ~s2 & ~s3;
            dst[y * Ww + w] = is3 | (alive & is2);
        }
    }
}

/* Run `turns` generations in place on an H x (64*Ww) torus.  If counts is
 * non-NULL, counts[t] = alive cells after turn t+1. */
int oracle_bits_run(uint64_t *words, int64_t H, int64_t Ww, int64_t turns, int64_t *counts)
{
    if (H <= 0 || Ww <= 0 || turns < 0) return -1;
    uint64_t *tmp = (uint64_t *)malloc((size_t)(H * Ww) * sizeof(uint64_t));
    if (!tmp) return -2;
    for (int64_t t = 0; t < turns; t++) {
        bits_generation(words, tmp, H, Ww);
        memcpy(words, tmp, (size_t)(H * Ww) * sizeof(uint64_t));
        if (counts) counts[t] = (int64_t)oracle_popcount_words(words, H * Ww);
    }
    free(tmp);
    return 0;
}
