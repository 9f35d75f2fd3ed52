// Exhaustive search (tools/, not product): can the Life rule tail -- given 2-bit encodings of
// A = a0+b0+c0 and B = a1+b1+c1 (the vertical sums of the three rows' horizontal 3-sums) and the
// cell -- be computed with 3 three-input gates (v_bitop3_b32)?  32 points (A, B, cell); the care
// mask drops (A=0,B=0,cell=1) and (A=3,B=3,cell=0), impossible because the centre row's sum
// includes the cell.  Result used in gol_kernels.hip (TT_G1, TT_G2, TT_OUT): encoding A0 B0.
//   gcc -O2 -o /tmp/rule_search tools/rule_search.c && /tmp/rule_search
#include <stdint.h>
#include <stdio.h>

static int alive(int A, int B, int cell) {
    int T = A + 2 * B;
    return T == 3 || (T == 4 && cell);
}

// encodings of a 4-valued variable by two "splits": split 0 = odd {1,3}, 1 = >=2 {2,3}, 2 = mid {1,2}
static int feat(int split, int v) {
    if (split == 0) return v & 1;
    if (split == 1) return v >= 2;
    return v == 1 || v == 2;
}

static uint32_t lut3(uint32_t tt, uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r = 0;
    for (int i = 0; i < 8; i++) {
        if (!((tt >> i) & 1)) continue;
        uint32_t m = ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
        r |= m;
    }
    return r;
}

// does target (on care) depend only on columns p, q, r?
static int fits(uint32_t F, uint32_t care, uint32_t p, uint32_t q, uint32_t r) {
    for (int i = 0; i < 8; i++) {
        uint32_t m = ((i & 4) ? p : ~p) & ((i & 2) ? q : ~q) & ((i & 1) ? r : ~r) & care;
        uint32_t f = F & m;
        if (f != 0 && f != m) return 0;
    }
    return 1;
}

int main(void) {
    const int encs[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    for (int ea = 0; ea < 3; ea++)
        for (int eb = 0; eb < 3; eb++) {
            uint32_t x[8] = {0}, F = 0, care = 0;
            for (int pt = 0; pt < 32; pt++) {
                int A = pt & 3, B = (pt >> 2) & 3, cell = (pt >> 4) & 1;
                int bits[5] = {feat(encs[ea][0], A), feat(encs[ea][1], A), feat(encs[eb][0], B), feat(encs[eb][1], B), cell};
                for (int j = 0; j < 5; j++)
                    if (bits[j]) x[j] |= 1u << pt;
                if (alive(A, B, cell)) F |= 1u << pt;
                if (!((A == 0 && B == 0 && cell == 1) || (A == 3 && B == 3 && cell == 0))) care |= 1u << pt;
            }
            long found = 0;
            // g1 over 3 of the 5 inputs, g2 over 3 of (5 inputs + g1), out over 3 of (5 + g1 + g2)
            for (int i1 = 0; i1 < 5; i1++)
                for (int j1 = i1 + 1; j1 < 5; j1++)
                    for (int k1 = j1 + 1; k1 < 5; k1++)
                        for (uint32_t t1 = 0; t1 < 256; t1++) {
                            x[5] = lut3(t1, x[i1], x[j1], x[k1]);
                            for (int i2 = 0; i2 < 6; i2++)
                                for (int j2 = i2 + 1; j2 < 6; j2++)
                                    for (int k2 = j2 + 1; k2 < 6; k2++) {
                                        if (k2 != 5) continue;  // g2 uses g1 (else the search is symmetric)
                                        for (uint32_t t2 = 0; t2 < 256; t2++) {
                                            x[6] = lut3(t2, x[i2], x[j2], x[k2]);
                                            for (int a = 0; a < 7; a++)
                                                for (int b = a + 1; b < 7; b++)
                                                    for (int c = b + 1; c < 7; c++) {
                                                        if (c != 6) continue;
                                                        if (fits(F, care, x[a], x[b], x[c])) {
                                                            if (found < 5)
                                                                printf("enc A%d B%d: g1=%02x(%d,%d,%d) g2=%02x(%d,%d,%d) out(%d,%d,%d)\n", ea, eb, t1, i1, j1, k1, t2, i2, j2, k2, a, b, c);
                                                            found++;
                                                        }
                                                    }
                                        }
                                    }
                        }
            // also: g1, g2 independent (both on inputs), out uses both
            for (int i1 = 0; i1 < 5; i1++)
                for (int j1 = i1 + 1; j1 < 5; j1++)
                    for (int k1 = j1 + 1; k1 < 5; k1++)
                        for (uint32_t t1 = 0; t1 < 256; t1++) {
                            x[5] = lut3(t1, x[i1], x[j1], x[k1]);
                            for (int i2 = 0; i2 < 5; i2++)
                                for (int j2 = i2 + 1; j2 < 5; j2++)
                                    for (int k2 = j2 + 1; k2 < 5; k2++)
                                        for (uint32_t t2 = 0; t2 < 256; t2++) {
                                            x[6] = lut3(t2, x[i2], x[j2], x[k2]);
                                            for (int a = 0; a < 5; a++)
                                                if (fits(F, care, x[a], x[5], x[6])) {
                                                    if (found < 5) printf("enc A%d B%d: par g1=%02x g2=%02x out(%d,g1,g2)\n", ea, eb, t1, t2, a);
                                                    found++;
                                                }
                                        }
                        }
            printf("encoding A%d B%d: %ld circuits\n", ea, eb, found);
            fflush(stdout);
        }
    return 0;
}
