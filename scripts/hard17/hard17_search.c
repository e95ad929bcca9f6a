/* hard17_search.c -- widen the hard 17-clue corpus by a {-1, +1} clue
 * exchange search (VERDICT r03 "next" item 3).  Workload tooling, not the
 * product and not the oracle: scripts/make_hard17.py builds and runs it,
 * then certifies every board it prints with the oracle's independent counter
 * (oracle_count_solutions_fast == 1) before committing the corpus.
 *
 * From a 17-clue puzzle P with one completion: drop clue a (a 16-clue
 * puzzle Q), enumerate Q's completions (skipped past CAP), and for every
 * empty cell b and digit v count the completions holding v at b.  Where
 * exactly one does, Q + (b, v) is a 17-clue puzzle with exactly one
 * completion.  New boards are deduplicated by isomorphism class: the
 * minimal string (0 < 1 < ... after relabelling digits by first
 * appearance) over transposition, band / stack permutations and row /
 * column permutations inside them -- the group gen.py's _symmetry_images
 * draws from.  Breadth-first from the seeds until TARGET classes.
 *
 *   hard17_search SEEDS_FILE TARGET CAP > classes.txt
 * prints one canonical 81-char class per line (seeds first). */
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int PEER[81][20], UNIT[27][9];

static void init_tables(void)
{
    for (int u = 0; u < 9; u++)
        for (int k = 0; k < 9; k++) {
            UNIT[u][k] = 9 * u + k;                                    /* row u */
            UNIT[9 + u][k] = 9 * k + u;                                /* column u */
            UNIT[18 + u][k] = 27 * (u / 3) + 3 * (u % 3) + 9 * (k / 3) + k % 3;  /* box u */
        }
    for (int i = 0; i < 81; i++) {
        int n = 0, r = i / 9, c = i % 9;
        for (int j = 0; j < 81; j++) {
            if (j == i) continue;
            int rj = j / 9, cj = j % 9;
            if (rj == r || cj == c || (rj / 3 == r / 3 && cj / 3 == c / 3)) PEER[i][n++] = j;
        }
    }
}

/* naked + hidden singles to a fixpoint; 0 on a contradiction */
static int propagate(uint16_t *c)
{
    for (int changed = 1; changed;) {
        changed = 0;
        for (int i = 0; i < 81; i++) {
            if (!c[i]) return 0;
            if (c[i] & (c[i] - 1)) continue;
            for (int k = 0; k < 20; k++) {
                int p = PEER[i][k];
                if (c[p] & c[i]) {
                    c[p] &= (uint16_t)~c[i];
                    if (!c[p]) return 0;
                    changed = 1;
                }
            }
        }
        for (int u = 0; u < 27; u++) {
            uint16_t once = 0, twice = 0;
            for (int k = 0; k < 9; k++) {
                uint16_t x = c[UNIT[u][k]];
                twice |= once & x;
                once |= x;
            }
            if (once != 0x1FF) return 0;
            uint16_t single = once & (uint16_t)~twice;
            if (!single) continue;
            for (int k = 0; k < 9; k++) {
                int cell = UNIT[u][k];
                uint16_t x = c[cell] & single;
                if (x && c[cell] != x) {
                    if (x & (x - 1)) return 0; /* two digits forced into one cell */
                    c[cell] = x;
                    changed = 1;
                }
            }
        }
    }
    return 1;
}

typedef struct {
    long count, cap;
    uint32_t tally[81][9];
    uint8_t *sols; /* the completions themselves when keep (cap x 81 bytes) */
    int keep;
} Enum;

static void enum_rec(uint16_t *c, Enum *e)
{
    if (e->count > e->cap || !propagate(c)) return;
    int best = -1, bn = 10;
    for (int i = 0; i < 81; i++) {
        int n = __builtin_popcount(c[i]);
        if (n > 1 && n < bn) {
            bn = n;
            best = i;
            if (n == 2) break;
        }
    }
    if (best < 0) {
        if (e->keep && e->count < e->cap)
            for (int i = 0; i < 81; i++) e->sols[81 * e->count + i] = (uint8_t)__builtin_ctz(c[i]);
        e->count++;
        for (int i = 0; i < 81; i++) e->tally[i][__builtin_ctz(c[i])]++;
        return;
    }
    for (uint16_t m = c[best]; m; m &= (uint16_t)(m - 1)) {
        uint16_t s[81];
        memcpy(s, c, sizeof s);
        s[best] = m & (uint16_t)(0u - m);
        enum_rec(s, e);
        if (e->count > e->cap) return;
    }
}

static void cand_of(const uint8_t *g, uint16_t *c)
{
    for (int i = 0; i < 81; i++) c[i] = g[i] ? (uint16_t)(1u << (g[i] - 1)) : 0x1FF;
}

/* ---- canonical form (minlex over the symmetry group) */
static int PERM3[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};

static int ROWS[2592][9], COLS[1296][9];

static void init_canon(void)
{
    int nr = 0, nc = 0;
    int(*cols)[9] = COLS, (*rows)[9] = ROWS;
    for (int bp = 0; bp < 6; bp++)
        for (int a = 0; a < 6; a++)
            for (int b = 0; b < 6; b++)
                for (int d = 0; d < 6; d++) {
                    const int in[3] = {a, b, d};
                    for (int k = 0; k < 9; k++) cols[nc][k] = 3 * PERM3[bp][k / 3] + PERM3[in[k / 3]][k % 3];
                    nc++;
                }
    for (int t = 0; t < 2; t++)
        for (int k = 0; k < 1296; k++) {
            memcpy(rows[nr], cols[k], sizeof rows[nr]);
            rows[nr][0] |= t << 8; /* transposition flag in row 0's high bits */
            nr++;
        }
}

static void canon(const uint8_t *g_in, uint8_t *best)
{
    const int nr = 2592, nc = 1296;
    int(*cols)[9] = COLS, (*rows)[9] = ROWS;
    memset(best, 255, 81);
    for (int ri = 0; ri < nr; ri++) {
        const int t = rows[ri][0] >> 8;
        int R[9];
        for (int k = 0; k < 9; k++) R[k] = rows[ri][k] & 0xFF;
        for (int ci = 0; ci < nc; ci++) {
            const int *C = cols[ci];
            uint8_t map[10] = {0}, next = 1;
            int k = 0, less = 0;
            for (; k < 81; k++) {
                int r = R[k / 9], c = C[k % 9];
                uint8_t x = t ? g_in[9 * c + r] : g_in[9 * r + c];
                if (x) {
                    if (!map[x]) map[x] = next++;
                    x = map[x];
                }
                if (!less) {
                    if (x > best[k]) break;
                    if (x < best[k]) less = 1;
                }
                if (less) best[k] = x;
            }
        }
    }
}


/* ---- an isomorphism invariant (cheap): two rounds of colour refinement
 * over the clues' row / column / box / band / stack / digit relations,
 * minimised over transposition.  Isomorphic boards always hash alike, so
 * counting distinct hashes under-counts classes, never over-counts. */
static uint64_t mix(uint64_t h, uint64_t x)
{
    h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    return h * 0xff51afd7ed558ccdull;
}

static int cmp_u64(const void *a, const void *b)
{
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

static uint64_t inv_one(const uint8_t *g)
{
    int cell[81], n = 0;
    for (int i = 0; i < 81; i++)
        if (g[i]) cell[n++] = i;
    uint64_t col[81], nxt[81];
    for (int a = 0; a < n; a++) col[a] = 1;
    for (int round = 0; round < 3; round++) {
        for (int a = 0; a < n; a++) {
            int ra = cell[a] / 9, ca = cell[a] % 9;
            /* relation kinds: same row, col, box, band-only, stack-only, digit */
            uint64_t rel[6][81];
            int rn[6] = {0};
            for (int b = 0; b < n; b++) {
                if (b == a) continue;
                int rb = cell[b] / 9, cb = cell[b] % 9;
                int k = -1;
                if (rb == ra) k = 0;
                else if (cb == ca) k = 1;
                else if (rb / 3 == ra / 3 && cb / 3 == ca / 3) k = 2;
                else if (rb / 3 == ra / 3) k = 3;
                else if (cb / 3 == ca / 3) k = 4;
                if (k >= 0) rel[k][rn[k]++] = mix(col[b], (uint64_t)(g[cell[b]] == g[cell[a]]));
                if (g[cell[b]] == g[cell[a]]) rel[5][rn[5]++] = mix(col[b], (uint64_t)(k + 7));
            }
            uint64_t h = mix(col[a], 12345);
            for (int k = 0; k < 6; k++) {
                qsort(rel[k], rn[k], sizeof(uint64_t), cmp_u64);
                h = mix(h, 1000 + k);
                for (int j = 0; j < rn[k]; j++) h = mix(h, rel[k][j]);
            }
            nxt[a] = h;
        }
        memcpy(col, nxt, sizeof col);
    }
    qsort(col, n, sizeof(uint64_t), cmp_u64);
    uint64_t h = 77;
    for (int a = 0; a < n; a++) h = mix(h, col[a]);
    return h;
}

static uint64_t invariant(const uint8_t *g)
{
    uint8_t t[81];
    for (int r = 0; r < 9; r++)
        for (int c = 0; c < 9; c++) t[9 * c + r] = g[9 * r + c];
    uint64_t a = inv_one(g), b = inv_one(t);
    return a < b ? a : b;
}

/* ---- a set of invariants */
typedef struct {
    uint64_t *keys;
    size_t cap;
    long n;
} Set;

static int set_add(Set *s, uint64_t k)
{
    k |= 1; /* 0 marks a free slot */
    size_t i = (k * 0x9E3779B97F4A7C15ull) >> 40 & (s->cap - 1);
    while (s->keys[i]) {
        if (s->keys[i] == k) return 0;
        i = (i + 1) & (s->cap - 1);
    }
    s->keys[i] = k;
    s->n++;
    return 1;
}

static Set g_set;
static long g_target, g_qn, g_qcap;
static uint8_t *g_queue;

static void emit(const uint8_t *N)
{
    uint64_t k = invariant(N);
#pragma omp critical
    {
        if (g_set.n < g_target && g_qn < g_qcap && set_add(&g_set, k)) {
            memcpy(g_queue + 81 * g_qn++, N, 81);
            for (int i = 0; i < 81; i++) putchar('0' + N[i]);
            putchar('\n');
            fflush(stdout);
        }
    }
}

/* drop one clue, add one */
static void expand1(const uint8_t *P, long cap, Enum *e)
{
    for (int a = 0; a < 81 && g_set.n < g_target; a++) {
        if (!P[a]) continue;
        uint8_t Q[81];
        memcpy(Q, P, 81);
        Q[a] = 0;
        memset(e->tally, 0, sizeof e->tally);
        e->count = 0;
        e->cap = cap;
        e->keep = 0;
        uint16_t c[81];
        cand_of(Q, c);
        enum_rec(c, e);
        if (e->count > cap || e->count < 2) continue;
        for (int b = 0; b < 81; b++) {
            if (Q[b]) continue;
            for (int v = 0; v < 9; v++) {
                if (e->tally[b][v] != 1) continue;
                uint8_t N[81];
                memcpy(N, Q, 81);
                N[b] = (uint8_t)(v + 1);
                emit(N);
            }
        }
    }
}

/* drop two clues, add two: the 16-clue board Q + (b1, v1) is kept when it
 * has 2..M2 completions (enumerated); then every (b2, v2) held by exactly
 * one of them makes a 17-clue board with one completion.  Enumerating the
 * 15-clue board Q itself is out of reach (> 2e5 completions each). */
enum { M2 = 64 };
static void expand2(const uint8_t *P, Enum *e)
{
    for (int a1 = 0; a1 < 81; a1++) {
        if (!P[a1]) continue;
        for (int a2 = a1 + 1; a2 < 81 && g_set.n < g_target; a2++) {
            if (!P[a2]) continue;
            uint8_t Q[81];
            memcpy(Q, P, 81);
            Q[a1] = Q[a2] = 0;
            uint16_t cq[81];
            cand_of(Q, cq);
            if (!propagate(cq)) continue;
            for (int b1 = 0; b1 < 81; b1++) {
                if (Q[b1] || b1 == a1 || b1 == a2) continue;
                for (uint16_t m = cq[b1]; m; m &= (uint16_t)(m - 1)) {
                    const int v1 = __builtin_ctz(m);
                    memset(e->tally, 0, sizeof e->tally);
                    e->count = 0;
                    e->cap = M2;
                    e->keep = 0;
                    uint16_t c[81];
                    memcpy(c, cq, sizeof c);
                    c[b1] = (uint16_t)(1u << v1);
                    enum_rec(c, e);
                    if (e->count > M2 || e->count < 2) continue;
                    for (int b2 = 0; b2 < 81; b2++) {
                        if (Q[b2] || b2 == b1) continue;
                        for (int v2 = 0; v2 < 9; v2++) {
                            if (e->tally[b2][v2] != 1) continue;
                            uint8_t N[81];
                            memcpy(N, Q, 81);
                            N[b1] = (uint8_t)(v1 + 1);
                            N[b2] = (uint8_t)(v2 + 1);
                            emit(N);
                        }
                    }
                }
            }
        }
    }
}

int main(int argc, char **argv)
{
    init_tables();
    init_canon();
    if (argc == 2 && !strcmp(argv[1], "--canon")) {
        /* exact classes: canonical form of every board on stdin, duplicates dropped */
        char line[256];
        long cap = 1 << 16, n = 0;
        uint8_t(*in)[81] = malloc(81 * (size_t)cap), (*out)[81] = malloc(81 * (size_t)cap);
        while (fgets(line, sizeof line, stdin) && n < cap)
            if (strlen(line) >= 81) {
                for (int i = 0; i < 81; i++) in[n][i] = (uint8_t)(line[i] - '0');
                n++;
            }
#pragma omp parallel for schedule(dynamic, 4)
        for (long p = 0; p < n; p++) canon(in[p], out[p]);
        for (long p = 0; p < n; p++) {
            int dup = 0;
            for (long q = 0; q < p && !dup; q++) dup = !memcmp(out[p], out[q], 81);
            if (dup) continue;
            for (int i = 0; i < 81; i++) putchar('0' + out[p][i]);
            putchar('\n');
        }
        return 0;
    }
    if (argc < 5) {
        fprintf(stderr, "usage: %s SEEDS TARGET CAP1 USE2 | --canon < boards\n", argv[0]);
        return 2;
    }
    g_target = atol(argv[2]);
    const long cap1 = atol(argv[3]);
    const int use2 = atoi(argv[4]);
    FILE *f = fopen(argv[1], "r");
    if (!f) return 2;
    g_set.cap = 1 << 22;
    g_set.keys = calloc(g_set.cap, sizeof(uint64_t));
    g_qcap = 1 << 20;
    g_queue = malloc(81 * (size_t)g_qcap);
    char line[256];
    while (fgets(line, sizeof line, f))
        if (strlen(line) >= 81) {
            uint8_t g[81];
            for (int i = 0; i < 81; i++) g[i] = (uint8_t)(line[i] == '.' ? 0 : line[i] - '0');
            emit(g);
        }
    fclose(f);
    /* {-1,+1} closure first (cheap), then one {-2,+2} expansion of the
     * oldest not yet so expanded board, and again */
    long head1 = 0, head2 = 0;
    while (g_set.n < g_target) {
        if (head1 < g_qn) {
            const long lo = head1, hi = g_qn;
            head1 = hi;
#pragma omp parallel
            {
                Enum *e = malloc(sizeof(Enum));
#pragma omp for schedule(dynamic, 1)
                for (long q = lo; q < hi; q++)
                    if (g_set.n < g_target) expand1(g_queue + 81 * q, cap1, e);
                free(e);
            }
            fprintf(stderr, "{-1,+1}: %ld classes\n", g_set.n);
            continue;
        }
        if (head2 >= g_qn || !use2) break;
        /* a block of boards at once, one per thread */
        const long lo = head2, hi = head2 + 8 < g_qn ? head2 + 8 : g_qn;
        head2 = hi;
#pragma omp parallel
        {
            Enum *e = malloc(sizeof(Enum));
#pragma omp for schedule(dynamic, 1)
            for (long q = lo; q < hi; q++)
                if (g_set.n < g_target && use2) expand2(g_queue + 81 * q, e);
            free(e);
        }
        fprintf(stderr, "{-2,+2} on %ld..%ld: %ld classes\n", lo, hi, g_set.n);
    }
    return 0;
}
