/*
 * blokus_oracle.c — TEST INFRASTRUCTURE ONLY. Not part of the product; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it (as the checker /
 * the CPU baseline), never as the thing measured or shipped.
 *
 * A plain-C, cell-by-cell restatement of the Blokus rules engine the reference drives through
 * `colosseumrl.envs.blokus` (imported at blokus_rl/colossumrl/blokus_wrapper.py:8-14, called at
 * :42, :86, :103-105, :122-124, :159-161, :173). That dependency is un-vendored and unpinned
 * (setup.py:11 `colosseumrl@git+...#egg=master`) and absent here, so its published behaviour is
 * restated from what the reference itself pins:
 *   - the 21 standard polyominoes, each used at most once;
 *   - turn order colour 1 -> 2 -> 3 -> 4; start corners (0,0), (0,N-1), (N-1,0), (N-1,N-1)
 *     for 4 players, (0,0), (N-1,N-1) for 2 (docs/images/AlphaZero GIF recordings);
 *   - a colour's first piece covers its corner; later pieces touch an own-colour piece
 *     corner-to-corner and never edge-to-edge;
 *   - a player with no legal move is skipped; the game ends when nobody can move;
 *   - winner(s) = most squares placed (ties -> several), mapped by the wrapper to -1 / 3 / 1
 *     (blokus_wrapper.py:164-186).
 * Pinned against the reference's recorded games (tests/golden/ JSON decoded from docs/ GIFs)
 * and the known answers 30433 / 919 actions (docs/README.md:128, :51) and 58 first moves.
 *
 * It deliberately shares no code with the HIP product: cells are a byte grid, legality is a
 * per-placement cell walk, orientations come from its own transform enumeration. It reads and
 * writes the product's 384-byte packed state (include/blokus_engine.h) so results compare
 * byte for byte.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MAXN 20
#define MAXP 4
#define NPIECE 21
#define STATE_BYTES 384

/* The 21 standard Blokus pieces, cells as (row, col). */
static const int PIECE_CELLS[NPIECE][5][2] = {
    {{0, 0}},                                         /* 1  monomino      */
    {{0, 0}, {0, 1}},                                 /* 2  domino        */
    {{0, 0}, {0, 1}, {0, 2}},                         /* 3  I3            */
    {{0, 0}, {1, 0}, {1, 1}},                         /* 4  V3            */
    {{0, 0}, {0, 1}, {0, 2}, {0, 3}},                 /* 5  I4            */
    {{0, 0}, {1, 0}, {2, 0}, {2, 1}},                 /* 6  L4            */
    {{0, 0}, {0, 1}, {0, 2}, {1, 1}},                 /* 7  T4            */
    {{0, 1}, {0, 2}, {1, 0}, {1, 1}},                 /* 8  S4            */
    {{0, 0}, {0, 1}, {1, 0}, {1, 1}},                 /* 9  O4            */
    {{0, 1}, {0, 2}, {1, 0}, {1, 1}, {2, 1}},         /* 10 F5            */
    {{0, 0}, {0, 1}, {0, 2}, {0, 3}, {0, 4}},         /* 11 I5            */
    {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {3, 1}},         /* 12 L5            */
    {{0, 1}, {1, 1}, {2, 0}, {2, 1}, {3, 0}},         /* 13 N5            */
    {{0, 0}, {0, 1}, {1, 0}, {1, 1}, {2, 0}},         /* 14 P5            */
    {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {2, 1}},         /* 15 T5            */
    {{0, 0}, {0, 2}, {1, 0}, {1, 1}, {1, 2}},         /* 16 U5            */
    {{0, 0}, {1, 0}, {2, 0}, {2, 1}, {2, 2}},         /* 17 V5            */
    {{0, 0}, {1, 0}, {1, 1}, {2, 1}, {2, 2}},         /* 18 W5            */
    {{0, 1}, {1, 0}, {1, 1}, {1, 2}, {2, 1}},         /* 19 X5            */
    {{0, 1}, {1, 0}, {1, 1}, {2, 1}, {3, 1}},         /* 20 Y5            */
    {{0, 0}, {0, 1}, {1, 1}, {2, 1}, {2, 2}},         /* 21 Z5            */
};
static const int PIECE_SIZE[NPIECE] = {1, 2, 3, 3, 4, 4, 4, 4, 4, 5, 5,
                                       5, 5, 5, 5, 5, 5, 5, 5, 5, 5};

typedef struct {
    int piece, orient, row, col;
    int ncell;
    int cell_r[5], cell_c[5];
} action_t;

typedef struct {
    int N, P, maxc;
    int npieces;
    int A;
    action_t* act;
    int corner_r[MAXP], corner_c[MAXP];
} bko_ctx;

/* unpacked state */
typedef struct {
    int8_t cell[MAXN][MAXN]; /* 0 empty, k+1 = colour k */
    uint32_t pieces[MAXP];
    int to_move, ply;
    uint32_t flags;
} ustate;

/* ---------------------------------------------------------------- orientations */
/* The eight symmetries of the square, applied in this fixed order; the first transform that
 * yields a new (normalised, sorted) cell set defines the next orientation index. */
static void transform(int k, int r, int c, int* orr, int* occ) {
    switch (k) {
    case 0: *orr = r;  *occ = c;  break;
    case 1: *orr = c;  *occ = -r; break;
    case 2: *orr = -r; *occ = -c; break;
    case 3: *orr = -c; *occ = r;  break;
    case 4: *orr = r;  *occ = -c; break;
    case 5: *orr = -c; *occ = -r; break;
    case 6: *orr = -r; *occ = c;  break;
    default: *orr = c; *occ = r;  break;
    }
}

static int cell_cmp(const void* a, const void* b) {
    const int* x = (const int*)a;
    const int* y = (const int*)b;
    if (x[0] != y[0]) return x[0] - y[0];
    return x[1] - y[1];
}

/* returns number of distinct orientations; shapes[o][k][2] sorted, normalised */
static int piece_orientations(int p, int shapes[8][5][2], int* h, int* w) {
    int n = PIECE_SIZE[p], count = 0;
    for (int k = 0; k < 8; ++k) {
        int cells[5][2], minr = 99, minc = 99, maxr = -99, maxc = -99;
        for (int i = 0; i < n; ++i) {
            transform(k, PIECE_CELLS[p][i][0], PIECE_CELLS[p][i][1], &cells[i][0], &cells[i][1]);
            if (cells[i][0] < minr) minr = cells[i][0];
            if (cells[i][1] < minc) minc = cells[i][1];
        }
        for (int i = 0; i < n; ++i) {
            cells[i][0] -= minr;
            cells[i][1] -= minc;
            if (cells[i][0] > maxr) maxr = cells[i][0];
            if (cells[i][1] > maxc) maxc = cells[i][1];
        }
        qsort(cells, n, sizeof(cells[0]), cell_cmp);
        int dup = 0;
        for (int o = 0; o < count && !dup; ++o) dup = memcmp(shapes[o], cells, sizeof(int) * 2 * n) == 0;
        if (!dup) {
            memcpy(shapes[count], cells, sizeof(int) * 2 * n);
            h[count] = maxr + 1;
            w[count] = maxc + 1;
            ++count;
        }
    }
    return count;
}

/* ---------------------------------------------------------------- context */
void* bko_create(int N, int P, int maxc) {
    if (N < 5 || N > MAXN || (P != 2 && P != 4) || maxc < 1 || maxc > 5) return NULL;
    bko_ctx* c = (bko_ctx*)calloc(1, sizeof(bko_ctx));
    c->N = N;
    c->P = P;
    c->maxc = maxc;
    c->npieces = 0;
    for (int p = 0; p < NPIECE; ++p)
        if (PIECE_SIZE[p] <= maxc) c->npieces = p + 1;
    /* count, then fill (piece, orientation, row, col) order */
    int cap = 0;
    for (int pass = 0; pass < 2; ++pass) {
        int id = 0;
        for (int p = 0; p < c->npieces; ++p) {
            int shapes[8][5][2], h[8], w[8];
            int no = piece_orientations(p, shapes, h, w);
            for (int o = 0; o < no; ++o)
                for (int r = 0; r + h[o] <= N; ++r)
                    for (int col = 0; col + w[o] <= N; ++col) {
                        if (pass == 1) {
                            action_t* a = &c->act[id];
                            a->piece = p;
                            a->orient = o;
                            a->row = r;
                            a->col = col;
                            a->ncell = PIECE_SIZE[p];
                            for (int k = 0; k < a->ncell; ++k) {
                                a->cell_r[k] = r + shapes[o][k][0];
                                a->cell_c[k] = col + shapes[o][k][1];
                            }
                        }
                        ++id;
                    }
        }
        if (pass == 0) {
            cap = id;
            c->act = (action_t*)calloc((size_t)cap, sizeof(action_t));
        }
        c->A = id;
    }
    if (P == 4) {
        int rr[4] = {0, 0, N - 1, N - 1}, cc[4] = {0, N - 1, 0, N - 1};
        for (int k = 0; k < 4; ++k) { c->corner_r[k] = rr[k]; c->corner_c[k] = cc[k]; }
    } else {
        c->corner_r[0] = 0; c->corner_c[0] = 0;
        c->corner_r[1] = N - 1; c->corner_c[1] = N - 1;
    }
    return c;
}

void bko_destroy(void* h) {
    bko_ctx* c = (bko_ctx*)h;
    if (!c) return;
    free(c->act);
    free(c);
}

int bko_action_size(void* h) { return ((bko_ctx*)h)->A; }
int bko_num_pieces(void* h) { return ((bko_ctx*)h)->npieces; }

void bko_action_table(void* h, int32_t* out) {
    bko_ctx* c = (bko_ctx*)h;
    for (int i = 0; i < c->A; ++i) {
        out[4 * i + 0] = c->act[i].piece;
        out[4 * i + 1] = c->act[i].orient;
        out[4 * i + 2] = c->act[i].row;
        out[4 * i + 3] = c->act[i].col;
    }
}

void bko_action_cells(void* h, int16_t* out) {
    bko_ctx* c = (bko_ctx*)h;
    for (int i = 0; i < c->A; ++i)
        for (int k = 0; k < 5; ++k)
            out[5 * i + k] = k < c->act[i].ncell ? (int16_t)(c->act[i].cell_r[k] * c->N + c->act[i].cell_c[k]) : -1;
}

/* ---------------------------------------------------------------- pack / unpack */
static void unpack(const bko_ctx* c, const uint8_t* st, ustate* u) {
    uint32_t occ[4][20];
    memcpy(occ, st, sizeof(occ));
    memset(u, 0, sizeof(*u));
    for (int k = 0; k < 4; ++k)
        for (int r = 0; r < c->N; ++r)
            for (int col = 0; col < c->N; ++col)
                if ((occ[k][r] >> col) & 1u) u->cell[r][col] = (int8_t)(k + 1);
    memcpy(u->pieces, st + 320, 16);
    memcpy(&u->to_move, st + 344, 4);
    memcpy(&u->ply, st + 348, 4);
    memcpy(&u->flags, st + 352, 4);
}

static uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Board hash: see include/blokus_engine.h — XOR over non-empty colour rows of
 * mix64((colour*32 + row) << 32 | row_bits), seeded. */
static uint64_t board_hash(const uint32_t occ[4][20]) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int k = 0; k < 4; ++k)
        for (int r = 0; r < 20; ++r)
            if (occ[k][r]) h ^= mix64(((uint64_t)(k * 32 + r) << 32) | occ[k][r]);
    return h;
}

static void pack(const bko_ctx* c, const ustate* u, uint8_t* st) {
    uint32_t occ[4][20];
    memset(occ, 0, sizeof(occ));
    for (int r = 0; r < c->N; ++r)
        for (int col = 0; col < c->N; ++col)
            if (u->cell[r][col]) occ[u->cell[r][col] - 1][r] |= 1u << col;
    memset(st, 0, STATE_BYTES);
    memcpy(st, occ, sizeof(occ));
    memcpy(st + 320, u->pieces, 16);
    uint64_t h = board_hash(occ);
    memcpy(st + 336, &h, 8);
    memcpy(st + 344, &u->to_move, 4);
    memcpy(st + 348, &u->ply, 4);
    memcpy(st + 352, &u->flags, 4);
}

/* ---------------------------------------------------------------- rules */
static int has_cells(const bko_ctx* c, const ustate* u, int k) {
    for (int r = 0; r < c->N; ++r)
        for (int col = 0; col < c->N; ++col)
            if (u->cell[r][col] == k + 1) return 1;
    return 0;
}

static int own_at(const bko_ctx* c, const ustate* u, int r, int col, int k) {
    if (r < 0 || col < 0 || r >= c->N || col >= c->N) return 0;
    return u->cell[r][col] == k + 1;
}

static int is_legal(const bko_ctx* c, const ustate* u, int k, int first, const action_t* a) {
    if (!((u->pieces[k] >> a->piece) & 1u)) return 0;
    int anchored = 0;
    for (int i = 0; i < a->ncell; ++i) {
        int r = a->cell_r[i], col = a->cell_c[i];
        if (u->cell[r][col]) return 0;
        if (own_at(c, u, r - 1, col, k) || own_at(c, u, r + 1, col, k) || own_at(c, u, r, col - 1, k) ||
            own_at(c, u, r, col + 1, k))
            return 0;
        if (first) {
            if (r == c->corner_r[k] && col == c->corner_c[k]) anchored = 1;
        } else if (own_at(c, u, r - 1, col - 1, k) || own_at(c, u, r - 1, col + 1, k) ||
                   own_at(c, u, r + 1, col - 1, k) || own_at(c, u, r + 1, col + 1, k)) {
            anchored = 1;
        }
    }
    return anchored;
}

static int count_legal(const bko_ctx* c, const ustate* u, int k, uint64_t* mask, int stop_at_first) {
    int first = !has_cells(c, u, k), n = 0;
    if (mask) memset(mask, 0, sizeof(uint64_t) * (size_t)((c->A + 63) / 64));
    for (int id = 0; id < c->A; ++id)
        if (is_legal(c, u, k, first, &c->act[id])) {
            ++n;
            if (mask) mask[id >> 6] |= 1ull << (id & 63);
            if (stop_at_first) return n;
        }
    return n;
}

void bko_init_state(void* h, uint8_t* st) {
    bko_ctx* c = (bko_ctx*)h;
    ustate u;
    memset(&u, 0, sizeof(u));
    uint32_t full = (c->npieces >= 32) ? 0xFFFFFFFFu : ((1u << c->npieces) - 1u);
    for (int k = 0; k < c->P; ++k) u.pieces[k] = full;
    pack(c, &u, st);
}

/* player < 0 -> to_move. Returns the legal count. mask may be NULL. */
int bko_legal_mask(void* h, const uint8_t* st, int player, uint64_t* mask) {
    bko_ctx* c = (bko_ctx*)h;
    ustate u;
    unpack(c, st, &u);
    int k = player < 0 ? u.to_move : player;
    return count_legal(c, &u, k, mask, 0);
}

void bko_legal_mask_batch(void* h, const uint8_t* states, int B, uint64_t* masks, int32_t* counts) {
    bko_ctx* c = (bko_ctx*)h;
    int W = (c->A + 63) / 64;
    for (int b = 0; b < B; ++b)
        counts[b] = bko_legal_mask(h, states + (size_t)b * STATE_BYTES, -1, masks + (size_t)b * W);
}

/* Apply action id for to_move; returns next player, or -1 if illegal (out untouched). */
int bko_next_state(void* h, const uint8_t* st, int action, uint8_t* out) {
    bko_ctx* c = (bko_ctx*)h;
    ustate u;
    unpack(c, st, &u);
    int k = u.to_move;
    if (action < 0 || action >= c->A) return -1;
    const action_t* a = &c->act[action];
    if (!is_legal(c, &u, k, !has_cells(c, &u, k), a)) return -1;
    for (int i = 0; i < a->ncell; ++i) u.cell[a->cell_r[i]][a->cell_c[i]] = (int8_t)(k + 1);
    u.pieces[k] &= ~(1u << a->piece);
    u.ply += 1;
    /* skip rule: next colour in cyclic order with a legal move (the mover itself last) */
    int next = -1;
    for (int d = 1; d <= c->P; ++d) {
        int q = (k + d) % c->P;
        if ((u.flags >> (4 + q)) & 1u) continue;
        if (count_legal(c, &u, q, NULL, 1) > 0) {
            next = q;
            break;
        }
        u.flags |= 1u << (4 + q);
    }
    if (next < 0) {
        u.flags |= 1u;
        next = (k + 1) % c->P;
    }
    u.to_move = next;
    pack(c, &u, out);
    return next;
}

/* Returns 1 if game over and fills scores[P] (-1 / 3 / 1), else 0 (scores zeroed). */
int bko_game_ended(void* h, const uint8_t* st, double* scores) {
    bko_ctx* c = (bko_ctx*)h;
    ustate u;
    unpack(c, st, &u);
    for (int k = 0; k < c->P; ++k) scores[k] = 0.0;
    if (!(u.flags & 1u)) return 0;
    int sq[MAXP] = {0}, best = -1, nwin = 0;
    for (int r = 0; r < c->N; ++r)
        for (int col = 0; col < c->N; ++col)
            if (u.cell[r][col]) sq[u.cell[r][col] - 1]++;
    for (int k = 0; k < c->P; ++k)
        if (sq[k] > best) best = sq[k];
    for (int k = 0; k < c->P; ++k) nwin += sq[k] == best;
    for (int k = 0; k < c->P; ++k) scores[k] = sq[k] == best ? (nwin == 1 ? 3.0 : 1.0) : -1.0;
    return 1;
}

void bko_square_counts(void* h, const uint8_t* st, int32_t* out) {
    bko_ctx* c = (bko_ctx*)h;
    ustate u;
    unpack(c, st, &u);
    for (int k = 0; k < c->P; ++k) out[k] = 0;
    for (int r = 0; r < c->N; ++r)
        for (int col = 0; col < c->N; ++col)
            if (u.cell[r][col]) out[u.cell[r][col] - 1]++;
}

void bko_observe(void* h, const uint8_t* st, float* obs) {
    bko_ctx* c = (bko_ctx*)h;
    ustate u;
    unpack(c, st, &u);
    int NN = c->N * c->N;
    memset(obs, 0, sizeof(float) * (size_t)(2 * c->P * NN));
    for (int r = 0; r < c->N; ++r)
        for (int col = 0; col < c->N; ++col)
            if (u.cell[r][col]) obs[(u.cell[r][col] - 1) * NN + r * c->N + col] = 1.0f;
    for (int i = 0; i < NN; ++i) obs[(c->P + u.to_move) * NN + i] = 1.0f;
}

uint64_t bko_hash(void* h, const uint8_t* st) {
    (void)h;
    uint32_t occ[4][20];
    memcpy(occ, st, sizeof(occ));
    return board_hash(occ);
}

/* Build a state from a colour grid (cells[N*N], 0 empty, k+1 colour k), pieces and to_move;
 * used to replay the recorded games. */
void bko_make_state(void* h, const int8_t* cells, const uint32_t* pieces, int to_move, int ply,
                    uint32_t flags, uint8_t* st) {
    bko_ctx* c = (bko_ctx*)h;
    ustate u;
    memset(&u, 0, sizeof(u));
    for (int r = 0; r < c->N; ++r)
        for (int col = 0; col < c->N; ++col) u.cell[r][col] = cells[r * c->N + col];
    memcpy(u.pieces, pieces, 16);
    u.to_move = to_move;
    u.ply = ply;
    u.flags = flags;
    pack(c, &u, st);
}
