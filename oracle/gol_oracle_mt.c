/*
 * gol_oracle_mt.c -- TEST INFRASTRUCTURE ONLY: the word-parallel restatement of
 * gol_oracle.c (2), multi-threaded and in place, for alive-count series of
 * full-size boards (tools/pin_counts_oracle.py -> tests/golden/oracle_counts.json).
 *
 * Nothing in the product links, loads or calls this file.  It follows the same
 * rule and layout as gol_oracle.c's oracle_bits_run (64 cells per uint64, bit b
 * of word w of row y is cell x = 64*w + b; worker.go:24-40's B3/S23 on the torus
 * of worker.go:44-70, rows wrapped with H and columns with W): the 8 neighbour
 * words of a word are summed by the same sequential bit-sliced adder, and
 * alive' = (n == 3) | (alive & n == 2).  What differs is only the schedule:
 *   - rows are split into T bands, one thread each (a barrier per generation);
 *   - a band is updated in place: each thread keeps the original of the row above
 *     the one it writes (and copies of its two halo rows, taken before anyone
 *     writes), so a 2^37-cell board needs one 16 GiB buffer, not two;
 *   - the inner loop over the interior words has no wraparound arithmetic (the
 *     first and last word of a row take the wrapped neighbours separately), so
 *     the compiler vectorises it;
 *   - the alive count is taken from the words as they are written.
 * tests/test_oracle.py checks it against oracle_bits_run on boards from 1 x 64
 * up, every thread count, every turn.
 */
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* A spinning barrier (yielding after a while): the futex wake-ups of pthread_barrier_wait cost
 * ~1 ms per generation on this container's VM (8 threads no faster than 1 on a 128 MiB board). */
struct spin_bar {
    int n;
    int count;       /* arrivals in this phase */
    unsigned phase;
};
static void bar_wait(struct spin_bar *b)
{
    const unsigned ph = __atomic_load_n(&b->phase, __ATOMIC_ACQUIRE);
    if (__atomic_add_fetch(&b->count, 1, __ATOMIC_ACQ_REL) == b->n) {
        __atomic_store_n(&b->count, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&b->phase, ph + 1, __ATOMIC_RELEASE);
        return;
    }
    for (long i = 0; __atomic_load_n(&b->phase, __ATOMIC_ACQUIRE) == ph; i++) {
        if (i < 4096) __builtin_ia32_pause();
        else sched_yield();  /* a vCPU shared with other work: let it run */
    }
}

/* The sum of the 8 neighbours of the 64 cells of word c (a: the word above, b: below; *l / *r:
 * the words to the left / right, i.e. cells x-64..x-1 / x+64..x+127), then the rule. */
static inline uint64_t gen_word(uint64_t al, uint64_t a, uint64_t ar, uint64_t cl, uint64_t c, uint64_t cr,
                                uint64_t bl, uint64_t b, uint64_t br)
{
    const uint64_t nb[8] = {
        (a << 1) | (al >> 63), a, (a >> 1) | (ar << 63),
        (c << 1) | (cl >> 63),    (c >> 1) | (cr << 63),
        (b << 1) | (bl >> 63), b, (b >> 1) | (br << 63),
    };
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < 8; i++) {
        const uint64_t c0 = s0 & nb[i];
        s0 ^= nb[i];
        const uint64_t c1 = s1 & c0;
        s1 ^= c0;
        const uint64_t c2 = s2 & c1;
        s2 ^= c1;
        s3 |= c2;
    }
    const uint64_t two_or_three = s1 & ~s2 & ~s3;  /* n in {2, 3} */
    return two_or_three & (s0 | c);                 /* n == 3, or n == 2 and alive */
}

/* One row: out = next state of row c given the rows a (above) and b (below); returns its count. */
static uint64_t gen_row(const uint64_t *restrict a, const uint64_t *restrict c, const uint64_t *restrict b,
                        uint64_t *restrict out, int64_t Ww)
{
    if (Ww == 1) {
        out[0] = gen_word(a[0], a[0], a[0], c[0], c[0], c[0], b[0], b[0], b[0]);
        return (uint64_t)__builtin_popcountll(out[0]);
    }
    const int64_t L = Ww - 1;
    const uint64_t first = gen_word(a[L], a[0], a[1], c[L], c[0], c[1], b[L], b[0], b[1]);
    const uint64_t last = gen_word(a[L - 1], a[L], a[0], c[L - 1], c[L], c[0], b[L - 1], b[L], b[0]);
    for (int64_t w = 1; w < L; w++)  /* (out never aliases a, c or b: the caller passes copies) */
        out[w] = gen_word(a[w - 1], a[w], a[w + 1], c[w - 1], c[w], c[w + 1], b[w - 1], b[w], b[w + 1]);
    out[0] = first;
    out[L] = last;
    uint64_t n = 0;
    for (int64_t w = 0; w <= L; w++) n += (uint64_t)__builtin_popcountll(out[w]);
    return n;
}

struct mt_ctx {
    uint64_t *words;
    int64_t H, Ww, turns, every;
    int64_t *counts;
    int T;
    struct spin_bar bar;
    uint64_t *part;  /* per-thread counts of the current generation */
    uint64_t *rows;  /* 4 rows of scratch per thread */
};

struct mt_arg {
    struct mt_ctx *x;
    int t;
};

static void *mt_thread(void *p)
{
    struct mt_arg *g = (struct mt_arg *)p;
    struct mt_ctx *x = g->x;
    const int64_t H = x->H, Ww = x->Ww, T = x->T, t = g->t;
    const int64_t y0 = H * t / T, y1 = H * (t + 1) / T;
    const size_t rb = (size_t)Ww * sizeof(uint64_t);
    uint64_t *buf = x->rows + 4 * Ww * t;
    uint64_t *top = buf, *bot = buf + Ww, *prev = buf + 2 * Ww, *cur = buf + 3 * Ww;
    for (int64_t turn = 0; turn < x->turns; turn++) {
        /* the halo rows as they are before this generation (their owners write them after the barrier) */
        memcpy(top, x->words + ((y0 + H - 1) % H) * Ww, rb);
        memcpy(bot, x->words + (y1 % H) * Ww, rb);
        bar_wait(&x->bar);
        uint64_t n = 0;
        memcpy(prev, top, rb);
        for (int64_t y = y0; y < y1; y++) {
            uint64_t *row = x->words + y * Ww;
            memcpy(cur, row, rb);  /* row y's old cells, the row above of row y + 1 */
            const uint64_t *below = y + 1 < y1 ? row + Ww : bot;
            n += gen_row(prev, cur, below, row, Ww);
            uint64_t *s = prev;
            prev = cur;
            cur = s;
        }
        x->part[t] = n;
        bar_wait(&x->bar);
        if (t == 0 && x->counts && (turn + 1) % x->every == 0) {
            uint64_t c = 0;
            for (int i = 0; i < T; i++) c += x->part[i];
            x->counts[(turn + 1) / x->every - 1] = (int64_t)c;
        }
    }
    return NULL;
}

/* `turns` generations in place on an H x (64*Ww) torus with `threads` threads; counts[i] = the
 * alive cells after turn (i+1)*every (turns / every entries; counts may be NULL). */
int oracle_mt_bits_run(uint64_t *words, int64_t H, int64_t Ww, int64_t turns, int64_t every, int64_t *counts,
                       int threads)
{
    if (H <= 0 || Ww <= 0 || turns < 0 || every <= 0 || threads <= 0) return -1;
    struct mt_ctx x;
    x.words = words; x.H = H; x.Ww = Ww; x.turns = turns; x.every = every; x.counts = counts;
    x.T = threads > H ? (int)H : threads;
    x.part = (uint64_t *)calloc((size_t)x.T, sizeof(uint64_t));
    x.rows = (uint64_t *)malloc((size_t)x.T * 4 * (size_t)Ww * sizeof(uint64_t));
    struct mt_arg *args = (struct mt_arg *)calloc((size_t)x.T, sizeof *args);
    pthread_t *tid = (pthread_t *)calloc((size_t)x.T, sizeof *tid);
    if (!x.part || !x.rows || !args || !tid) {
        free(x.part); free(x.rows); free(args); free(tid);
        return -2;
    }
    x.bar.n = x.T;
    x.bar.count = 0;
    x.bar.phase = 0;
    for (int i = 0; i < x.T; i++) {
        args[i].x = &x;
        args[i].t = i;
        pthread_create(&tid[i], NULL, mt_thread, &args[i]);
    }
    for (int i = 0; i < x.T; i++) pthread_join(tid[i], NULL);
    free(tid); free(args); free(x.part); free(x.rows);
    return 0;
}

/* gol_oracle.c's synthetic board and board hash over `threads` threads (rows split evenly). */
static inline uint64_t splitmix64(uint64_t v)
{
    uint64_t z = v + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct fill_arg {
    uint64_t seed, *words, h;
    int64_t y0, y1, Ww;
    int mode;  /* 0: fill, 1: hash */
};

static void *fill_thread(void *p)
{
    struct fill_arg *f = (struct fill_arg *)p;
    uint64_t h = 0;
    for (int64_t y = f->y0; y < f->y1; y++)
        for (int64_t w = 0; w < f->Ww; w++) {
            const uint64_t idx = (uint64_t)(y * f->Ww + w);
            if (f->mode == 0) f->words[idx] = splitmix64(f->seed ^ idx);
            else h += splitmix64(f->words[idx] ^ splitmix64(idx));
        }
    f->h = h;
    return NULL;
}

static uint64_t fill_or_hash(uint64_t seed, uint64_t *words, int64_t H, int64_t Ww, int threads, int mode)
{
    int T = threads > 64 ? 64 : (threads < 1 ? 1 : threads);
    if (T > H) T = (int)H;
    struct fill_arg a[64];
    pthread_t tid[64];
    for (int i = 0; i < T; i++) {
        a[i].seed = seed; a[i].words = words; a[i].Ww = Ww; a[i].mode = mode;
        a[i].y0 = H * i / T;
        a[i].y1 = H * (i + 1) / T;
        pthread_create(&tid[i], NULL, fill_thread, &a[i]);
    }
    uint64_t h = 0;
    for (int i = 0; i < T; i++) {
        pthread_join(tid[i], NULL);
        h += a[i].h;
    }
    return h;
}

void oracle_mt_random_words(uint64_t seed, int64_t H, int64_t Ww, uint64_t *words, int threads)
{
    fill_or_hash(seed, words, H, Ww, threads, 0);
}

uint64_t oracle_mt_hash_words(const uint64_t *words, int64_t H, int64_t Ww, int threads)
{
    return fill_or_hash(0, (uint64_t *)words, H, Ww, threads, 1);
}
