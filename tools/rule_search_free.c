// Exhaustive search (tools/, not product): does a 3-gate tail exist for the band pipeline's pair
// step when the pair's shared signals may be ANY functions of the pair sum P = b + c (0..6)?
// (tools/rule_search_pair.c searched fixed encodings of P)  Per value of P
// the shared signals are constants, so a tail gate with s free inputs realises, per P, one of its
// 2^s cofactors, chosen freely per P.  Every structure of three 3-input gates over the wires
// {x0, x1, cell, g1, g2} plus free inputs is searched; a tail must give
// alive' = [P + x == 3] | (cell & [P + x == 4]) on every (P, x, cell) except the two impossible
// ones (cell alive with P = 0, dead with P = 6: the cell's row is one of the pair).
// Result (round 6): total 0 -- no 3-gate tail for any encoding of the pair.
//   gcc -O3 -march=native -fopenmp -o /tmp/rsf tools/rule_search_free.c && /tmp/rsf     (~2 min, 8 cores)
// over wires {x0, x1, cell, g1, g2} + free slots.
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static const uint8_t WM[3] = {0xAA, 0xCC, 0xF0};  // x0, x1, cell over minterms m = x0 | x1<<1 | cell<<2
static uint8_t T[7], C[7];
static uint8_t ev(unsigned tt, int w, const uint8_t *in)
{
    uint8_t r = 0;
    for (int i = 0; i < (1 << w); i++)
        if ((tt >> i) & 1) {
            uint8_t m = 0xFF;
            for (int j = 0; j < w; j++) m &= ((i >> j) & 1) ? in[j] : (uint8_t)~in[j];
            r |= m;
        }
    return r;
}
// option lists for a gate of w wires
static int opts(int w, unsigned L[][4], int *n)
{
    int k = 0;
    if (w == 3) for (unsigned t = 0; t < 256; t++) { L[k][0] = t; n[k++] = 1; }
    else if (w == 2) for (unsigned a = 0; a < 16; a++) for (unsigned b = a; b < 16; b++) { L[k][0] = a; L[k][1] = b; n[k++] = a == b ? 1 : 2; }
    else if (w == 1) { L[0][0] = 0; L[0][1] = 3; L[0][2] = 2; L[0][3] = 1; n[0] = 4; k = 1; }
    return k;
}
int main(void)
{
    for (int P = 0; P < 7; P++) {
        T[P] = 0; C[P] = 0;
        for (int m = 0; m < 8; m++) {
            int x = (m & 1) + 2 * ((m >> 1) & 1), c = (m >> 2) & 1, t = P + x;
            if (t == 3 || (t == 4 && c)) T[P] |= 1 << m;
            if (c ? P >= 1 : P <= 5) C[P] |= 1 << m;
        }
    }
    static unsigned L1[256][4], L2[256][4], L3[256][4];
    static int n1[256], n2[256], n3[256];
    long sols = 0;
    for (int W1 = 1; W1 < 8; W1++)  // subset of {x0,x1,cell}
        for (int W2 = 1; W2 < 16; W2++) {  // subset of {x0,x1,cell,g1}
            if (__builtin_popcount(W2) > 3) continue;
            for (int W3 = 0; W3 < 32; W3++) {  // subset of {x0,x1,cell,g1,g2}, must hold g2
                if (!(W3 & 16) || __builtin_popcount(W3) > 3) continue;
                if (!(W2 & 8) && !(W3 & 8)) continue;  // g1 used
                int w1 = __builtin_popcount(W1), w2 = __builtin_popcount(W2), w3 = __builtin_popcount(W3);
                int k1 = opts(w1, L1, n1), k2 = opts(w2, L2, n2), k3 = opts(w3, L3, n3);
                long found = 0;
                #pragma omp parallel for reduction(+:found) schedule(dynamic)
                for (int a = 0; a < k1; a++) {
                    uint8_t in[3]; int q;
                    uint8_t g1v[4]; int ng1 = 0;
                    q = 0; for (int j = 0; j < 3; j++) if (W1 >> j & 1) in[q++] = WM[j];
                    for (int i = 0; i < n1[a]; i++) g1v[ng1++] = ev(L1[a][i], w1, in);
                    for (int b = 0; b < k2; b++) {
                        uint8_t pr1[16], pr2[16]; int np = 0;
                        for (int i = 0; i < ng1; i++) {
                            q = 0; for (int j = 0; j < 3; j++) if (W2 >> j & 1) in[q++] = WM[j];
                            if (W2 & 8) in[q++] = g1v[i];
                            for (int t = 0; t < n2[b]; t++) { pr1[np] = g1v[i]; pr2[np++] = ev(L2[b][t], w2, in); }
                        }
                        for (int c3 = 0; c3 < k3; c3++) {
                            uint64_t O[4] = {0, 0, 0, 0};
                            for (int p = 0; p < np; p++) {
                                q = 0; for (int j = 0; j < 3; j++) if (W3 >> j & 1) in[q++] = WM[j];
                                if (W3 & 8) in[q++] = pr1[p];
                                in[q++] = pr2[p];
                                for (int t = 0; t < n3[c3]; t++) { uint8_t o = ev(L3[c3][t], w3, in); O[o >> 6] |= 1ull << (o & 63); }
                            }
                            int ok = 1;
                            for (int P = 0; P < 7 && ok; P++) {
                                int hit = 0;
                                for (int o = 0; o < 256 && !hit; o++) if ((O[o >> 6] >> (o & 63) & 1) && !((o ^ T[P]) & C[P])) hit = 1;
                                ok = hit;
                            }
                            if (ok) {
                                found++;
                                if (found <= 3) {
                                    #pragma omp critical
                                    printf("W1=%x W2=%x W3=%x f1={%x,%x,%x,%x}/%d f2={%x,%x}/%d f3={%x,%x}/%d\n", W1, W2, W3, L1[a][0], L1[a][1], L1[a][2], L1[a][3], n1[a],
                                           L2[b][0], L2[b][1], n2[b], L3[c3][0], L3[c3][1], n3[c3]);
                                }
                            }
                        }
                    }
                }
                if (found) printf("structure W1=%x W2=%x W3=%x: %ld\n", W1, W2, W3, found);
                sols += found;
            }
        }
    printf("total %ld\n", sols);
    return 0;
}
