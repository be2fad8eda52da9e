// legal_rows.h — the batched legal-move bitmask kernel (bk_legal_mask), row-parallel form.
//
// Mapping: one 64-lane wave holds floor(64/N) boards, one lane per board row (N=20 -> 3 boards,
// lanes 0-59; N=7 -> 9 boards). Each lane keeps its row and the next four rows of the mover's
// forbidden / anchor bitboards in registers; in the batched kernel's default (lean) step in board
// order, "cell (dr, dc) of a placement with origin column c" being bit c of row[dr] >> dc, and in
// the search's single-board bitmasks BIT-REVERSED, bit (31-c) of rev_row[dr] << dc (one
// v_lshl_or_b32 per cell and plane).
// The 91 fixed orientations are unrolled at compile time from orient_table.h, so the inner
// loop has no table loads and every cell offset is an immediate. For each orientation the lane
// produces the W legal origin columns of its origin row and ORs that W-bit field into its
// board's LDS bitmask at bit base_o + r*W; the masks then stream out as u64 rows.
#pragma once
#include <utility>

#include "common.h"
#include "orient_table.h"

namespace bk {

__device__ const int kNoPlayer = -1;  // k_legal_mask_rows: the player read when none is given

struct RowCtx {
  uint32_t fr[5];      // bit-reversed forbidden rows r..r+4
  uint32_t ar[5];      // bit-reversed anchor rows r..r+4
  uint32_t rowok[6];   // rowok[h] = ~0 when a placement of height h fits below row r (and the lane is real)
  uint32_t pieces;     // unused pieces of the mover
  uint32_t upieces;    // wave-uniform: the pieces some board of the wave still has (skip the rest)
  int rN1;             // r * (N + 1): bit offset of origin row r is base + r*(N+1) - r*w
  int r;
  int rw[6];           // lean step (SPLIT 3): rw[w] = r*(N+1) - r*w, opaque to the compiler
  uint32_t* mb;        // this lane's board bitmask in LDS
};

// One fixed orientation for one origin row, branch-free: 2 ops per cell (v_lshl_or into the
// forbidden and anchor accumulators), then legal = anchor & ~forbidden, validity masks, and the
// W-bit field ORed into the board's LDS bitmask (two 32-bit ORs; the second is 0 unless the field
// straddles a word).
// SKIP0: a wave holding ONE board (lanes 0..N-1 its rows, the rest idle) ORs only non-zero fields:
// otherwise the idle lanes and the empty rows, which all address the word of row 0, serialise on
// it (the leaf bitmask of the search: 52.7 vs 53.8 us a leaf step). The 3-board legal kernel
// keeps the unconditional form (its branch-free ORs measured 12.1 vs 15.4 us with the skip).
// NT: the board size at compile time (20: the classic board with all 21 pieces), 0 = dp.N at run
// time; with NT the piece test, W, R and the field bases are constants and the 91 steps are one
// basic block (at run time every step is a scalar branch around an out-of-line block)
template <int O, int WPB, int SPLIT, bool SKIP0 = false, int NT = 0>
__device__ __forceinline__ void orient_step(const DevPreset& dp, const RowCtx& c, int wave, int& base) {
  constexpr OrientC oc = kOrient[O];
  if (NT ? oc.piece >= kNumPieces : oc.piece >= dp.num_pieces) return;  // wave-uniform (presets use a prefix of the pieces)
  const int W = (NT ? NT : dp.N) - oc.w + 1;
  const int R = (NT ? NT : dp.N) - oc.h + 1;
  // another wave of the workgroup owns this orientation, or no board of the wave has its piece
  // (scalar test; the bits stay as zeroed)
  if ((WPB > 1 && (O % WPB) != wave) || !((c.upieces >> oc.piece) & 1u)) {
    base += R * W;
    return;
  }
  if constexpr (SPLIT == 3) {
    // the lean step (k_legal_mask_rows' default): rows in board order, so cell (dr, dc) of origin
    // column c is bit c of row[dr] >> dc and the field needs no v_bfrev; the column and row validity live in fr
    // (columns >= N and rows past the board forbidden: a field bit past W or an origin row past
    // N - h then has a forbidden cell, since every orientation has a cell at dc = 0 and one at
    // dr = h - 1); the field's bit offset is one add of the wave-uniform base to a per-lane
    // constant. tests/test_legal_lean_algebra.py restates this arithmetic against the oracle.
    uint32_t bad = c.fr[oc.dr[0]] >> oc.dc[0];
    uint32_t good = c.ar[oc.dr[0]] >> oc.dc[0];
#pragma unroll
    for (int k = 1; k < oc.n; ++k) {
      bad |= c.fr[oc.dr[k]] >> oc.dc[k];
      good |= c.ar[oc.dr[k]] >> oc.dc[k];
    }
    const uint32_t pmask = (uint32_t)__builtin_amdgcn_sbfe((int)c.pieces, oc.piece, 1);
    const uint32_t v = good & ~bad & pmask;
    const int bit = base + c.rw[oc.w];
    const uint64_t x = (uint64_t)v << (bit & 31);
    uint32_t* dst = c.mb + (bit >> 5);
    atomicOr(dst, (uint32_t)x);
    atomicOr(dst + 1, (uint32_t)(x >> 32));
    base += R * W;
    return;
  }
  uint32_t bad = c.fr[oc.dr[0]] << oc.dc[0];
  uint32_t good = c.ar[oc.dr[0]] << oc.dc[0];
#pragma unroll
  for (int k = 1; k < oc.n; ++k) {
    bad |= c.fr[oc.dr[k]] << oc.dc[k];
    good |= c.ar[oc.dr[k]] << oc.dc[k];
  }
  const uint32_t colmask = (1u << W) - 1u;  // wave-uniform
  const uint32_t pmask = (uint32_t)__builtin_amdgcn_sbfe((int)c.pieces, oc.piece, 1);
  // SKIP0 (one board per wave, row_ctx): rows past the board are forbidden in fr, no row mask
  const uint32_t v = __brev(good & ~bad) & colmask & (SKIP0 ? ~0u : c.rowok[oc.h]) & pmask;
  const int bit = base + c.rN1 - c.r * oc.w;
  const uint64_t x = (uint64_t)v << (bit & 31);
  uint32_t* dst = c.mb + (bit >> 5);
  if (SPLIT) {
    // even and odd origin rows in separate LDS instructions: two lanes of one instruction are
    // >= 2W >= 32 bits apart, so they never OR into the same word (no same-address serialisation)
    if ((c.r & 1) == 0) {
      atomicOr(dst, (uint32_t)x);
      atomicOr(dst + 1, (uint32_t)(x >> 32));
    }
    if (c.r & 1) {  // the other word first: otherwise the compiler merges the two branches
      atomicOr(dst + 1, (uint32_t)(x >> 32));
      atomicOr(dst, (uint32_t)x);
    }
  } else if (SKIP0) {
    if (v) {
      atomicOr(dst, (uint32_t)x);
      if ((uint32_t)(x >> 32)) atomicOr(dst + 1, (uint32_t)(x >> 32));
    }
  } else {
    atomicOr(dst, (uint32_t)x);
    atomicOr(dst + 1, (uint32_t)(x >> 32));
  }
  base += R * W;
}

template <int WPB, int SPLIT, bool SKIP0 = false, int NT = 0, size_t... Os>
__device__ __forceinline__ void orient_all(const DevPreset& dp, const RowCtx& c, int wave,
                                           std::index_sequence<Os...>) {
  int base = 0;
  (orient_step<(int)Os, WPB, SPLIT, SKIP0, NT>(dp, c, wave, base), ...);
}

// The bit offset of orientation O's fields in the mask, base(O) = sum over O' < O of
// (N - h' + 1)(N - w' + 1) = cnt N^2 + b N + c with compile-time prefix sums (the orientations
// of the pieces a preset uses are a prefix of the table, sorted by piece).
struct OrientBase {
  int cnt[kNumOrient + 1], b[kNumOrient + 1], c[kNumOrient + 1];
};
constexpr OrientBase make_orient_base() {
  OrientBase t{};
  for (int i = 0; i < kNumOrient; ++i) {
    t.cnt[i + 1] = t.cnt[i] + 1;
    t.b[i + 1] = t.b[i] + (2 - kOrient[i].h - kOrient[i].w);
    t.c[i + 1] = t.c[i] + (1 - kOrient[i].h) * (1 - kOrient[i].w);
  }
  return t;
}
constexpr OrientBase kOrientBase = make_orient_base();

// Wave W of WPB's orientations (O = W, W + WPB, ...) straight: no steps over the other waves'
// orientations (stepping over 85 of 91 unrolled orientations per wave, each a scalar branch and
// the base update, took ~14k cycles per leaf bitmask at 16 waves: the walk, not the work)
template <int O>
__device__ __forceinline__ void orient_step_at(const DevPreset& dp, const RowCtx& c) {
  constexpr OrientC oc = kOrient[O];
  if (oc.piece >= dp.num_pieces) return;  // wave-uniform
  const int N = dp.N;
  int base = kOrientBase.cnt[O] * N * N + kOrientBase.b[O] * N + kOrientBase.c[O];
  orient_step<O, 1, 0, true>(dp, c, 0, base);
}
template <int W, int WPB, size_t... Ks>
__device__ __forceinline__ void orient_part(const DevPreset& dp, const RowCtx& c, std::index_sequence<Ks...>) {
  (orient_step_at<W + (int)Ks * WPB>(dp, c), ...);
}
template <int WPB, size_t... Ws>
__device__ __forceinline__ void orient_dispatch(const DevPreset& dp, const RowCtx& c, int wave,
                                                std::index_sequence<Ws...>) {
  // wave-uniform: each wave runs only its own instance
  ((wave == (int)Ws ? orient_part<(int)Ws, WPB>(dp, c, std::make_index_sequence<(kNumOrient - (int)Ws + WPB - 1) / WPB>{})
                    : void()),
   ...);
}

// The lean step of orientation O at its compile-time base (board size NT): wave W of WPB runs the
// orientations O = W, W + WPB, ... (k_legal_mask_rows' multi-wave lean variants)
template <int O, int NT>
__device__ __forceinline__ void orient_step_nt(const DevPreset& dp, const RowCtx& c) {
  int base = kOrientBase.cnt[O] * NT * NT + kOrientBase.b[O] * NT + kOrientBase.c[O];
  orient_step<O, 1, 3, false, NT>(dp, c, 0, base);
}
template <int W, int WPB, int NT, size_t... Ks>
__device__ __forceinline__ void orient_part_nt(const DevPreset& dp, const RowCtx& c, std::index_sequence<Ks...>) {
  (orient_step_nt<W + (int)Ks * WPB, NT>(dp, c), ...);
}
template <int WPB, int NT, size_t... Ws>
__device__ __forceinline__ void orient_dispatch_nt(const DevPreset& dp, const RowCtx& c, int wave,
                                                   std::index_sequence<Ws...>) {
  ((wave == (int)Ws
        ? orient_part_nt<(int)Ws, WPB, NT>(dp, c, std::make_index_sequence<(kNumOrient - (int)Ws + WPB - 1) / WPB>{})
        : void()),
   ...);
}

// The row context of colour q on the board s (LDS) for lanes 0..N-1 (the board's rows); lanes
// past N (rows past the board) are all forbidden. first: q has no cell yet. (The lean step on
// board-order rows here measured 0.3% slower end to end: the search's bitmasks skip used pieces
// and zero fields, so their VALU is not on the step's critical path.)
__device__ __forceinline__ RowCtx row_ctx(const DevPreset& dp, const uint32_t* s, int q, uint32_t* m32) {
  const int l = lane_id();
  const int N = dp.N;
  const bool ok = l < N;
  const int r = ok ? l : 0;
  const uint32_t own = ok ? s[q * kMaxN + r] : 0u;
  const uint32_t occ = ok ? (s[r] | s[kMaxN + r] | s[2 * kMaxN + r] | s[3 * kMaxN + r]) : 0u;
  const uint32_t up = (ok && r > 0) ? s[q * kMaxN + r - 1] : 0u;
  const uint32_t dn = (ok && r + 1 < N) ? s[q * kMaxN + r + 1] : 0u;
  const bool first = __ballot(own != 0u) == 0ull;
  uint32_t forb = 0u, anch = 0u;
  if (ok) {
    forb = (occ | own << 1 | own >> 1 | up | dn) & dp.full_row;
    if (first)
      anch = (r == dp.corner_r(q)) ? (1u << dp.corner_c(q)) : 0u;
    else
      anch = (up << 1 | up >> 1 | dn << 1 | dn >> 1) & dp.full_row;
  }
  RowCtx c;
  // the lanes past the board (rows >= N) are all forbidden: a placement reaching below the board
  // then has a forbidden cell in every origin column < W (its bottom row's cell), so the single-
  // board steps (SKIP0, orient_any) need no per-height row mask — six fewer live registers in the
  // search's descent, which spilled them to scratch (a vmcnt(0) reload per orientation tested)
  c.fr[0] = ok ? __brev(forb) : ~0u;
  c.ar[0] = __brev(anch);
#pragma unroll
  for (int d = 1; d < 5; ++d) {
    const int src = l + d > kWave - 1 ? kWave - 1 : l + d;
    c.fr[d] = __shfl(c.fr[0], src, kWave);
    c.ar[d] = __shfl(c.ar[0], src, kWave);
  }
  c.r = r;
  c.rN1 = r * (N + 1);
  c.pieces = s[kWPieces + q];
  c.upieces = __builtin_amdgcn_readfirstlane(c.pieces);
#pragma unroll
  for (int h = 0; h < 6; ++h) c.rowok[h] = ~0u;  // unused by the single-board steps (above)
  c.mb = m32;
  return c;
}

// Does the context's colour have a legal placement? The orientations of its unused pieces in
// table order, each the same per-row test as orient_step, until the first one with a legal origin
// (registers only: no table loads, no LDS).
template <size_t... Os>
__device__ __forceinline__ bool orient_any(const DevPreset& dp, const RowCtx& c, std::index_sequence<Os...>) {
  bool found = false;
  auto step = [&](auto oi) {
    constexpr int O = decltype(oi)::value;
    constexpr OrientC oc = kOrient[O];
    if (found || oc.piece >= dp.num_pieces || !((c.upieces >> oc.piece) & 1u)) return;  // wave-uniform
    uint32_t bad = c.fr[oc.dr[0]] << oc.dc[0];
    uint32_t good = c.ar[oc.dr[0]] << oc.dc[0];
#pragma unroll
    for (int k = 1; k < oc.n; ++k) {
      bad |= c.fr[oc.dr[k]] << oc.dc[k];
      good |= c.ar[oc.dr[k]] << oc.dc[k];
    }
    const uint32_t colmask = (1u << (dp.N - oc.w + 1)) - 1u;
    const uint32_t v = __brev(good & ~bad) & colmask;  // rows past the board: forbidden in fr (row_ctx)
    found = __ballot(v != 0u) != 0ull;
  };
  (step(std::integral_constant<int, (int)Os>{}), ...);
  return found;
}
__device__ __forceinline__ bool rows_any_legal(const DevPreset& dp, const uint32_t* s, int q) {
  if (!s[kWPieces + q]) return false;
  const RowCtx c = row_ctx(dp, s, q, nullptr);
  if (__ballot((c.ar[0] & ~c.fr[0]) != 0u) == 0ull) return false;  // no free anchor cell
  return orient_any(dp, c, std::make_index_sequence<kNumOrient>{});
}

// The legal-move bitmask of colour q built by all WPB waves of the workgroup (the state in LDS,
// m32 zeroed here): wave w evaluates the orientations O with O % WPB == w, all OR into m32.
template <int WPB>
__device__ __forceinline__ void build_mask_rows_wg(const DevPreset& dp, const uint32_t* s, int q, uint32_t* m32,
                                                   int wave) {
#ifndef BK_MASK_STAMP
#define BK_MASK_STAMP(i) do { } while (0)
#endif
  for (int i = threadIdx.x; i < dp.W32pad / 4; i += kWave * WPB)
    reinterpret_cast<uint4*>(m32)[i] = make_uint4(0u, 0u, 0u, 0u);
  const RowCtx c = row_ctx(dp, s, q, m32);
  BK_MASK_STAMP(5);
  __syncthreads();
  BK_MASK_STAMP(6);
  orient_dispatch<WPB>(dp, c, wave, std::make_index_sequence<WPB>{});
  BK_MASK_STAMP(7);
  __syncthreads();
}

// One board per wave (the state already in LDS): lanes 0..N-1 are the board's rows, the same
// unrolled orientation steps as below, the bitmask ORed into m32 (zeroed here). Replaces the
// item loop wherever a single wave owns a single board (k_select's leaf, k_legal_ids, ...).
__device__ __forceinline__ void build_mask_rows(const DevPreset& dp, const uint32_t* s, int q, uint32_t* m32) {
  const int l = lane_id();
  for (int i = l; i < dp.W32pad / 4; i += kWave) reinterpret_cast<uint4*>(m32)[i] = make_uint4(0u, 0u, 0u, 0u);
  const RowCtx c = row_ctx(dp, s, q, m32);
  BK_BOARD_SYNC();
  orient_all<1, 0, true>(dp, c, 0, std::make_index_sequence<kNumOrient>{});
  BK_BOARD_SYNC();
}

// Workgroup = WPB waves sharing one group of boards_per_wave boards: wave w evaluates the
// orientations O with O % WPB == w (round robin keeps the cell work balanced), all OR into the
// same LDS masks, then the WPB waves stream the masks out together.
// LDS: boards_per_wave * W32pad words. Grid: ceil(B / boards_per_wave) blocks of 64*WPB.
constexpr int kLegalStoreIt = 4;  // uint4 rows per thread of the store phase: W64 / 2 <= 4 x 64 (N <= 20)
constexpr int kClassicW64 = 476, kClassicW32pad = 952;  // the classic board's mask rows (30433 ids)
template <int WPB, int SPLIT, int BPW = 0, int NT = 0>
__global__ __launch_bounds__(64 * WPB) void k_legal_mask_rows(DevPreset dp, const uint32_t* __restrict__ states,
                                                              const int32_t* __restrict__ players, int B,
                                                              uint64_t* __restrict__ masks,
                                                              int32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t m32[];
  __shared__ int cnt_sh[kWave];
#ifndef BK_LEGAL_ABL
#define BK_LEGAL_ABL 0  // diagnostic timing builds only: 1 no orientation work, 2 no mask stores, 8 empty
#endif
  if constexpr ((BK_LEGAL_ABL & 8) != 0) return;
  const int l = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int N = NT ? NT : dp.N;
  const int bpw = BPW ? BPW : kWave / N;
  const int j = l / N;
  const int r = l - j * N;
  const int b0 = blockIdx.x * bpw;
  const int b = b0 + j;
  const bool ok = j < bpw && b < B;
  if constexpr (NT > 0 && WPB == 1) {
    // the classic board: 3 boards x 238 uint4 (W32pad = 952), a compile-time trip count
    constexpr int kZ = (3 * kClassicW32pad / 4 + kWave - 1) / kWave;
#pragma unroll
    for (int k = 0; k < kZ; ++k) {
      const int i = l + k * kWave;
      if (k < kZ - 1 || i < 3 * kClassicW32pad / 4) reinterpret_cast<uint4*>(m32)[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  } else {
    for (int i = threadIdx.x; i < bpw * dp.W32pad / 4; i += kWave * WPB)
      reinterpret_cast<uint4*>(m32)[i] = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x < kWave) cnt_sh[threadIdx.x] = 0;
  }

  uint32_t o0 = 0u, o1 = 0u, o2 = 0u, o3 = 0u, pieces4[kMaxP] = {0u, 0u, 0u, 0u};
  int q = 0;
  if (ok) {  // independent loads: the four colour rows, the four piece sets, the mover
    const uint32_t* s = states + (size_t)b * kStateWords;
    o0 = s[r];
    o1 = s[kMaxN + r];
    o2 = s[2 * kMaxN + r];
    o3 = s[3 * kMaxN + r];
#pragma unroll
    for (int k = 0; k < kMaxP; ++k) pieces4[k] = s[kWPieces + k];
    // the state's mover and the given player both read unconditionally with the rest (a null
    // `players` reads a -1 constant): read only when players[b] < 0, the mover was a second round
    // trip after the rows, and one wave's latency is the launch at the config's batch
    const int* pp = players ? players + b : &kNoPlayer;
    const int pq = *pp;
    const uint32_t tm = s[kWToMove];
    q = pq < 0 ? (int)tm : pq;
  }
  const uint32_t own = q == 0 ? o0 : q == 1 ? o1 : q == 2 ? o2 : o3;
  const uint32_t pieces = q == 0 ? pieces4[0] : q == 1 ? pieces4[1] : q == 2 ? pieces4[2] : pieces4[3];
  const uint32_t occ = o0 | o1 | o2 | o3;
  const uint32_t up_raw = __shfl(own, l - 1 < 0 ? 0 : l - 1, kWave);
  const uint32_t dn_raw = __shfl(own, l + 1 > kWave - 1 ? kWave - 1 : l + 1, kWave);
  const uint32_t up = r > 0 ? up_raw : 0u;
  const uint32_t dn = r + 1 < N ? dn_raw : 0u;
  const uint64_t owners = __ballot(ok && own != 0u);
  const uint64_t rows_of_board = (N >= 64 ? ~0ull : ((1ull << N) - 1ull)) << (j * N);
  const bool first = (owners & rows_of_board) == 0ull;
  uint32_t forb = 0u, anch = 0u;
  if (ok) {
    forb = (occ | own << 1 | own >> 1 | up | dn) & dp.full_row;
    if (first)
      anch = (r == dp.corner_r(q)) ? (1u << dp.corner_c(q)) : 0u;
    else
      anch = (up << 1 | up >> 1 | dn << 1 | dn >> 1) & dp.full_row;
  }
  RowCtx c;
  // rows past the board (and idle lanes) forbidden, as row_ctx: the single-board step form
  // (SKIP0, the WPB > 1 variants' orient_step_at) relies on it instead of rowok
  c.fr[0] = ok ? __brev(forb) : ~0u;
  c.ar[0] = __brev(anch);
  if constexpr (SPLIT == 3) {
    c.fr[0] = ok ? (forb | ~dp.full_row) : ~0u;
    c.ar[0] = anch;
  }
#pragma unroll
  for (int d = 1; d < 5; ++d) {
    const int src = l + d > kWave - 1 ? kWave - 1 : l + d;
    c.fr[d] = __shfl(c.fr[0], src, kWave);
    c.ar[d] = __shfl(c.ar[0], src, kWave);
    c.fr[d] = (ok && r + d < N) ? c.fr[d] : ~0u;  // the next board's rows are past this board
  }
  c.r = r;
  c.rN1 = r * (N + 1);
  if constexpr (SPLIT == 3) {
#pragma unroll
    for (int w = 1; w < 6; ++w) {
      c.rw[w] = c.rN1 - r * w;
      asm volatile("" : "+v"(c.rw[w]));  // keep base + rw[w] one add (no re-association)
    }
  }
  c.pieces = pieces;
  // no piece skip here: with 3 boards per wave a piece absent from all three is rare, and the
  // branches cost the compiler its sharing of the shifted rows across orientations (+50% VALU)
  c.upieces = ~0u;
#pragma unroll
  for (int h = 0; h < 6; ++h) c.rowok[h] = (ok && r + h <= N) ? ~0u : 0u;
  c.mb = m32 + (j < bpw ? j : 0) * dp.W32pad;
  __syncthreads();  // mask zeroing complete
  if constexpr ((BK_LEGAL_ABL & 1) != 0) {
  } else if constexpr (WPB > 1 && SPLIT == 3 && NT > 0) {
    orient_dispatch_nt<WPB, NT>(dp, c, wave, std::make_index_sequence<WPB>{});
  } else if constexpr (WPB > 1) {
    // each wave only its own orientations at compile-time bases: orient_all's walk over the
    // other waves' orientations (a scalar branch + base update each) doubled the instruction count
    orient_dispatch<WPB>(dp, c, wave, std::make_index_sequence<WPB>{});
  } else {
    orient_all<WPB, SPLIT, false, NT>(dp, c, wave, std::make_index_sequence<kNumOrient>{});
  }
  __syncthreads();
  if constexpr (NT > 0 && WPB == 1) {
    // the classic board, one wave: all 3 x 4 LDS reads, then the 16-B stores; the counts of
    // boards 0 and 1 share one wave reduction (16-bit halves: a count is < 2^15), stored by lane 0
    constexpr int kRow4 = kClassicW64 / 2;  // uint4 per board mask
    uint4 v[3][kLegalStoreIt];
#pragma unroll
    for (int jj = 0; jj < 3; ++jj)
#pragma unroll
      for (int k = 0; k < kLegalStoreIt; ++k) {
        const int p = l + k * kWave;
        v[jj][k] = (k < kLegalStoreIt - 1 || p < kRow4)
                       ? reinterpret_cast<const uint4*>(m32 + jj * kClassicW32pad)[p]
                       : make_uint4(0u, 0u, 0u, 0u);
      }
    int cnt[3] = {0, 0, 0};
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      const bool live = b0 + jj < B;
      uint4* dst = reinterpret_cast<uint4*>(masks + (size_t)(b0 + jj) * kClassicW64);
#pragma unroll
      for (int k = 0; k < kLegalStoreIt; ++k) {
        const int p = l + k * kWave;
        if (live && (k < kLegalStoreIt - 1 || p < kRow4)) {
          if constexpr ((BK_LEGAL_ABL & 2) == 0) dst[p] = v[jj][k];
        }
        cnt[jj] += __popc(v[jj][k].x) + __popc(v[jj][k].y) + __popc(v[jj][k].z) + __popc(v[jj][k].w);
      }
    }
    const int c01 = wave_total(cnt[0] | (cnt[1] << 16));
    const int c2 = wave_total(cnt[2]);
    if (counts && l == 0) {
      counts[b0] = c01 & 0xFFFF;
      if (b0 + 1 < B) counts[b0 + 1] = (int)((unsigned)c01 >> 16);
      if (b0 + 2 < B) counts[b0 + 2] = c2;
    }
    return;
  }
  // stream out every board of the group: 16-B stores when rows are 16-B aligned (W64 even);
  // popcounts accumulate per lane, one wave reduction and one LDS add per board
  const int nb = B - b0 < bpw ? B - b0 : bpw;
  for (int jj = 0; jj < nb; ++jj) {
    int cnt = 0;
    if ((dp.W64 & 1) == 0) {
      const uint4* src = reinterpret_cast<const uint4*>(m32 + jj * dp.W32pad);
      uint4* dst = reinterpret_cast<uint4*>(masks + (size_t)(b0 + jj) * dp.W64);
      // all of the board's LDS reads before its stores (4 x 64 uint4 cover W64 <= 512 at N <= 20:
      // the read-store round trip per 16 B cost ~0.5 us a launch at 4096 boards)
      uint4 v[kLegalStoreIt];
#pragma unroll
      for (int k = 0; k < kLegalStoreIt; ++k) {
        const int p = threadIdx.x + k * kWave * WPB;
        v[k] = p < dp.W64 / 2 ? src[p] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int k = 0; k < kLegalStoreIt; ++k) {
        const int p = threadIdx.x + k * kWave * WPB;
        if constexpr ((BK_LEGAL_ABL & 2) != 0) {
          if (p < dp.W64 / 2 && v[k].x == 0x9e3779b9u) dst[p] = v[k];  // (almost) never: loads stay live
        } else {
          if (p < dp.W64 / 2) dst[p] = v[k];
        }
        cnt += __popc(v[k].x) + __popc(v[k].y) + __popc(v[k].z) + __popc(v[k].w);
      }
    } else {
      for (int p = threadIdx.x; p < dp.W64; p += kWave * WPB) {
        const uint32_t* src = m32 + jj * dp.W32pad + 2 * p;
        const uint64_t v = (uint64_t)src[0] | ((uint64_t)src[1] << 32);
        masks[(size_t)(b0 + jj) * dp.W64 + p] = v;
        cnt += __popcll(v);
      }
    }
    cnt = wave_sum(cnt);
    if (l == 0) atomicAdd(&cnt_sh[jj], cnt);
  }
  __syncthreads();
  if (counts && threadIdx.x < nb) counts[b0 + threadIdx.x] = cnt_sh[threadIdx.x];
}

// ---- staged form (BK_LEGAL_WPB=31): no LDS atomics ----
// The mask is the concatenation, in (orientation, origin row) order, of every row's W-bit field
// of legal origin columns. The atomic form ORs each field into its (one or two) words: 182 LDS
// atomics per wave, same-word lanes serialised (PMC: 72% of the LDS cycles were conflicts). Here
// each lane stores its field whole, one conflict-free ds_write_b32 per orientation at a slot
// (orientation, row) of its board's stage, and the words are then assembled from a host-built
// pack table: output u32 word k is the OR of at most three fields, entry = (slot, sh) with
// contribution hi32(field << sh) (sh = start bit - 32k + 32; an empty entry has sh = 0 -> 0).
constexpr int kStageRows = kMaxN + 4;  // rows kMaxN.. are spare slots for the lanes past the boards
constexpr int kStageWords = kNumOrient * kStageRows;
constexpr int kStageMaxBoards = 9;     // floor(64 / 7)
constexpr int kPackPrefetch = 8;       // table entries per lane held in registers (W64 <= 512 at N=20)
__host__ __device__ constexpr int legal_stage_lds_bytes(int N) {
  return 4 * ((kWave / N + (kWave - (kWave / N) * N > kStageRows - kMaxN ? 1 : 0)) * kStageWords + kWave);
}

template <int O>
__device__ __forceinline__ void orient_stage(const DevPreset& dp, const RowCtx& c) {
  constexpr OrientC oc = kOrient[O];
  if (oc.piece >= dp.num_pieces) return;  // wave-uniform (not in the mask)
  const int W = dp.N - oc.w + 1;
  uint32_t bad = c.fr[oc.dr[0]] << oc.dc[0];
  uint32_t good = c.ar[oc.dr[0]] << oc.dc[0];
#pragma unroll
  for (int k = 1; k < oc.n; ++k) {
    bad |= c.fr[oc.dr[k]] << oc.dc[k];
    good |= c.ar[oc.dr[k]] << oc.dc[k];
  }
  const uint32_t colmask = (1u << W) - 1u;
  const uint32_t pmask = (uint32_t)__builtin_amdgcn_sbfe((int)c.pieces, oc.piece, 1);
  c.mb[O * kStageRows] = __brev(good & ~bad) & colmask & c.rowok[oc.h] & pmask;  // immediate offset
}
template <size_t... Os>
__device__ __forceinline__ void orient_stage_all(const DevPreset& dp, const RowCtx& c, std::index_sequence<Os...>) {
  (orient_stage<(int)Os>(dp, c), ...);
}
__device__ __forceinline__ uint32_t pack_word(uint64_t e, const uint32_t* st) {
  uint32_t w = 0u;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint32_t ent = (uint32_t)(e >> (18 * i)) & 0x3FFFFu;
    const uint64_t f = (uint64_t)st[ent & 0xFFFu] << (ent >> 12);
    w |= (uint32_t)(f >> 32);
  }
  return w;
}

// One wave per group of floor(64/N) boards (lanes = board rows, as k_legal_mask_rows).
// LDS: legal_stage_lds_bytes(). pack: [W64] x uint4 (the entries of words 2p, 2p+1).
template <int MaxBoards>  // kStageMaxBoards (a template so the header's kernel links once)
__global__ __launch_bounds__(64) void k_legal_mask_staged(DevPreset dp, const uint32_t* __restrict__ states,
                                                          const int32_t* __restrict__ players, int B,
                                                          const uint4* __restrict__ pack,
                                                          uint64_t* __restrict__ masks,
                                                          int32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t st32[];
  const int l = lane_id();
  const int N = dp.N;
  const int bpw = kWave / N;
  const int j = l / N;
  const int r = l - j * N;
  const int b0 = blockIdx.x * bpw;
  const int b = b0 + j;
  const bool ok = j < bpw && b < B;
  uint32_t o0 = 0u, o1 = 0u, o2 = 0u, o3 = 0u, pieces4[kMaxP] = {0u, 0u, 0u, 0u};
  int q = 0;
  if (ok) {
    const uint32_t* s = states + (size_t)b * kStateWords;
    o0 = s[r];
    o1 = s[kMaxN + r];
    o2 = s[2 * kMaxN + r];
    o3 = s[3 * kMaxN + r];
#pragma unroll
    for (int k = 0; k < kMaxP; ++k) pieces4[k] = s[kWPieces + k];
    q = players ? players[b] : -1;
    if (q < 0) q = (int)s[kWToMove];
  }
  // the pack table's entries of this lane's words, loaded now: they arrive under the
  // orientation work (a dependent table load per word in the pack loop cost ~3 us per launch)
  uint4 pe[kPackPrefetch];
#pragma unroll
  for (int i = 0; i < kPackPrefetch; ++i)
    pe[i] = l + i * kWave < dp.W64 ? pack[l + i * kWave] : make_uint4(0u, 0u, 0u, 0u);
  const uint32_t own = q == 0 ? o0 : q == 1 ? o1 : q == 2 ? o2 : o3;
  const uint32_t pieces = q == 0 ? pieces4[0] : q == 1 ? pieces4[1] : q == 2 ? pieces4[2] : pieces4[3];
  const uint32_t occ = o0 | o1 | o2 | o3;
  const uint32_t up_raw = __shfl(own, l - 1 < 0 ? 0 : l - 1, kWave);
  const uint32_t dn_raw = __shfl(own, l + 1 > kWave - 1 ? kWave - 1 : l + 1, kWave);
  const uint32_t up = r > 0 ? up_raw : 0u;
  const uint32_t dn = r + 1 < N ? dn_raw : 0u;
  const uint64_t owners = __ballot(ok && own != 0u);
  const uint64_t rows_of_board = (N >= 64 ? ~0ull : ((1ull << N) - 1ull)) << (j * N);
  const bool first = (owners & rows_of_board) == 0ull;
  uint32_t forb = 0u, anch = 0u;
  if (ok) {
    forb = (occ | own << 1 | own >> 1 | up | dn) & dp.full_row;
    if (first)
      anch = (r == dp.corner_r(q)) ? (1u << dp.corner_c(q)) : 0u;
    else
      anch = (up << 1 | up >> 1 | dn << 1 | dn >> 1) & dp.full_row;
  }
  RowCtx c;
  c.fr[0] = __brev(forb);
  c.ar[0] = __brev(anch);
#pragma unroll
  for (int d = 1; d < 5; ++d) {
    const int src = l + d > kWave - 1 ? kWave - 1 : l + d;
    c.fr[d] = __shfl(c.fr[0], src, kWave);
    c.ar[d] = __shfl(c.ar[0], src, kWave);
  }
  c.r = r;
  c.rN1 = r * (N + 1);
  c.pieces = pieces;
  c.upieces = ~0u;
#pragma unroll
  for (int h = 0; h < 6; ++h) c.rowok[h] = (ok && r + h <= N) ? ~0u : 0u;
  // the lanes past the last board (their fields are 0) store into board 0's spare rows, or into
  // a scratch stage after the boards when there are more of them than spare rows (never packed)
  const int idle = l - bpw * N;
  c.mb = j < bpw ? st32 + j * kStageWords + r
                 : (kWave - bpw * N <= kStageRows - kMaxN ? st32 + kMaxN + idle : st32 + bpw * kStageWords + idle);
  orient_stage_all(dp, c, std::make_index_sequence<kNumOrient>{});
  __syncthreads();
  const int nb = B - b0 < bpw ? B - b0 : bpw;
  int cnt[MaxBoards];
#pragma unroll
  for (int jj = 0; jj < MaxBoards; ++jj) cnt[jj] = 0;
  auto pack_one = [&](int p, const uint4 e) {
    const uint64_t e0 = (uint64_t)e.x | ((uint64_t)e.y << 32);
    const uint64_t e1 = (uint64_t)e.z | ((uint64_t)e.w << 32);
#pragma unroll
    for (int jj = 0; jj < MaxBoards; ++jj) {
      if (jj < nb) {
        const uint32_t* sb = st32 + jj * kStageWords;
        const uint32_t lo = pack_word(e0, sb);
        const uint32_t hi = pack_word(e1, sb);
        masks[(size_t)(b0 + jj) * dp.W64 + p] = (uint64_t)lo | ((uint64_t)hi << 32);
        cnt[jj] += __popc(lo) + __popc(hi);
      }
    }
  };
#pragma unroll
  for (int i = 0; i < kPackPrefetch; ++i)
    if (l + i * kWave < dp.W64) pack_one(l + i * kWave, pe[i]);
  for (int p = l + kPackPrefetch * kWave; p < dp.W64; p += kWave) pack_one(p, pack[p]);
#pragma unroll
  for (int jj = 0; jj < MaxBoards; ++jj) {
    if (jj < nb) {
      const int s = wave_sum(cnt[jj]);
      if (counts && l == 0) counts[b0 + jj] = s;
    }
  }
}

}  // namespace bk
