// Exhaustive search (tools/, not product) behind the pair step of the band pipeline
// (gol_kernels.hip pstage / pair_tail).
//
// Two consecutive output rows n-1 and n share the rows n-1 and n of their 3 x 3 neighbourhoods.
// With a row's horizontal 3-sum as two bits (h0 = xor3, h1 = maj of the cell and its two
// neighbours), the shared part is the pair sum P = b + c (rows n-1, n; 0..6) in binary: p0 = b0^c0,
// k = b0&c0, p1 = xor3(b1,c1,k), p2 = maj(b1,c1,k) -- 4 gates for both rows.  Each row then needs
// a tail over (p0, p1, p2, x0, x1, cell), x = the third row's sum: alive' = [P + x == 3] |
// (cell & [P + x == 4]).  Don't-cares: the cell's row is one of the pair, so a live cell has
// P >= 1 and a dead one P <= 5; P = 7 never occurs.
//
// Result: no 3-gate tail exists (over the binary P; nor over the other 4-gate pair encodings
// (p0, two 2-valued splits of floor/ceil(P/2)); nor with the carry k as a fifth pair signal);
// 152 4-gate tails exist.  The kernel uses g1 = 0x43(p0, x0, cell), g2 = 0x25(p1, p2, x1),
// g3 = 0x8D(p2, cell, g1), out = 0x90(g3, g1, g2): g1 and g2 independent, depth 3.
// Per 32 cells and generation: 2 (row sum) + 4/2 (pair) + 4 (tail) = 8 gates, against 9 for the
// row-by-row circuit (tools/rule_search.c).
//   gcc -O3 -march=native -o /tmp/rsp tools/rule_search_pair.c && /tmp/rsp        (~15 min)
#include <stdint.h>
#include <stdio.h>
#include <string.h>
typedef uint64_t u64;

static u64 lut3(unsigned tt, u64 a, u64 b, u64 c)
{
    u64 r = 0;
    for (int i = 0; i < 8; i++)
        if ((tt >> i) & 1) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
}

int main(void)
{
    // points: P (3 bits, 0..7), x (2 bits), cell; signals 0 p0, 1 p1, 2 p2, 3 x0, 4 x1, 5 cell
    u64 X[6] = {0}, F = 0, care = 0;
    for (int pt = 0; pt < 64; pt++) {
        const int P = pt & 7, A = (pt >> 3) & 3, c = (pt >> 5) & 1;
        const u64 bit = 1ull << pt;
        if (P & 1) X[0] |= bit;
        if (P & 2) X[1] |= bit;
        if (P & 4) X[2] |= bit;
        if (A & 1) X[3] |= bit;
        if (A & 2) X[4] |= bit;
        if (c) X[5] |= bit;
        const int T = P + A;
        if (T == 3 || (T == 4 && c)) F |= bit;
        if (P <= 6 && (c ? P >= 1 : P <= 5)) care |= bit;
    }
    long found = 0;
    // g1 over the inputs, g2 over inputs + g1, g3 over inputs + g1 + g2, out = LUT(g3, y, z):
    // for each (g1, g2, g3's inputs, y, z) the LUTs of g3 and out exist iff, within every class
    // of (y, z), F is a function of g3 -- a 2-colouring of the classes' polarities (16 tries).
    for (int i1 = 0; i1 < 6; i1++)
        for (int j1 = i1 + 1; j1 < 6; j1++)
            for (int k1 = j1 + 1; k1 < 6; k1++)
                for (unsigned t1 = 0; t1 < 256; t1++) {
                    u64 S[9];
                    memcpy(S, X, sizeof X);
                    S[6] = lut3(t1, X[i1], X[j1], X[k1]);
                    for (int i2 = 0; i2 < 7; i2++)
                        for (int j2 = i2 + 1; j2 < 7; j2++)
                            for (int k2 = j2 + 1; k2 < 7; k2++)
                                for (unsigned t2 = 0; t2 < 256; t2++) {
                                    S[7] = lut3(t2, S[i2], S[j2], S[k2]);
                                    for (int a = 0; a < 8; a++)
                                        for (int b = a + 1; b < 8; b++)
                                            for (int c = b + 1; c < 8; c++) {
                                                u64 cm[8];
                                                for (int m = 0; m < 8; m++)
                                                    cm[m] = ((m & 4) ? S[a] : ~S[a]) & ((m & 2) ? S[b] : ~S[b]) &
                                                            ((m & 1) ? S[c] : ~S[c]) & care;
                                                for (int y = 0; y < 8; y++)
                                                    for (int z = y + 1; z < 8; z++) {
                                                        if (!(y == 7 || z == 7 || a == 7 || b == 7 || c == 7)) continue;
                                                        unsigned r1[4], r0[4];
                                                        int ok = 1, cons[4];
                                                        for (int K = 0; K < 4 && ok; K++) {
                                                            const u64 km = ((K & 2) ? S[y] : ~S[y]) & ((K & 1) ? S[z] : ~S[z]);
                                                            r1[K] = r0[K] = 0;
                                                            for (int m = 0; m < 8; m++) {
                                                                const u64 pm = cm[m] & km, f = F & pm;
                                                                if (!pm) continue;
                                                                if (f == pm) r1[K] |= 1u << m;
                                                                else if (f == 0) r0[K] |= 1u << m;
                                                                else { ok = 0; break; }
                                                            }
                                                            cons[K] = r1[K] && r0[K];
                                                        }
                                                        if (!ok) continue;
                                                        for (int pol = 0; pol < 16; pol++) {
                                                            unsigned N1 = 0, N0 = 0;
                                                            for (int K = 0; K < 4; K++) {
                                                                if (!cons[K]) continue;
                                                                N1 |= ((pol >> K) & 1) ? r0[K] : r1[K];
                                                                N0 |= ((pol >> K) & 1) ? r1[K] : r0[K];
                                                            }
                                                            if (N1 & N0) continue;
                                                            const unsigned t3 = N1 & 0xff;
                                                            const u64 g3 = lut3(t3, S[a], S[b], S[c]);
                                                            unsigned to = 0;
                                                            for (int idx = 0; idx < 8; idx++) {
                                                                const u64 pm = ((idx & 4) ? g3 : ~g3) & ((idx & 2) ? S[y] : ~S[y]) &
                                                                               ((idx & 1) ? S[z] : ~S[z]) & care;
                                                                if (pm && (F & pm) == pm) to |= 1u << idx;
                                                            }
                                                            if (((lut3(to, g3, S[y], S[z]) ^ F) & care) == 0) {
                                                                found++;
                                                                printf("g1=%02x(%d,%d,%d) g2=%02x(%d,%d,%d) g3=%02x(%d,%d,%d) out=%02x(g3,%d,%d)\n",
                                                                       t1, i1, j1, k1, t2, i2, j2, k2, t3, a, b, c, to, y, z);
                                                            }
                                                            break;
                                                        }
                                                    }
                                            }
                                }
                }
    printf("%ld circuits\n", found);
    return 0;
}
