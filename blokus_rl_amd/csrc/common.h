// common.h — device-side building blocks shared by the env and MCTS kernels (gfx950).
//
// Execution model: every board-level kernel runs ONE 64-lane wave per board (blockDim = 64),
// so a board's state, its forbidden/anchor rows and its legal-move bitmask live in that wave's
// LDS slice and every cross-lane step is a ballot / shuffle / LDS exchange inside one wave.
// Bitboards: one u32 per board row (bit c = column c), N <= 20.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tables.h"

namespace bk {

constexpr int kWave = 64;

// Kernel-argument view of a preset (passed by value).
struct DevPreset {
  int N, P, A, W64, W32, W32pad, num_items, num_pieces;
  uint32_t full_pieces;
  uint32_t full_row;  // (1 << N) - 1
  // the start corners, one byte per colour: an index by the (runtime) colour is a shift of a kernel
  // argument held in SGPRs, not a byte load from the kernarg segment (a memory round trip per use)
  uint32_t corner_r4, corner_c4;
  __device__ __forceinline__ int corner_r(int q) const { return (int)((corner_r4 >> (8 * q)) & 0xFFu); }
  __device__ __forceinline__ int corner_c(int q) const { return (int)((corner_c4 >> (8 * q)) & 0xFFu); }
  int16_t piece_item_off[kNumPieces + 1];
  const uint64_t* items;  // [num_items]
  const uint4* act_it;    // [A]: the action's item (lo, hi words) and its act word (item | col << 16 | piece << 24)
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Hash term of one non-empty colour row (matches include/blokus_engine.h).
__device__ __forceinline__ uint64_t row_key(int colour, int row, uint32_t bits) {
  return mix64(((uint64_t)(colour * 32 + row) << 32) | bits);
}

__device__ __forceinline__ uint64_t state_hash(const uint32_t* s) {
  return (uint64_t)s[kWHash] | ((uint64_t)s[kWHash + 1] << 32);
}

// ---- wave primitives on DPP (row_shr 1/2/4/8, row_bcast 15/31) + readlane: VALU-latency
// chains instead of ds_bpermute round trips through the LDS crossbar.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

// Generic inclusive wave scan: OP(acc_from_lower, mine) applied in Kogge-Stone order.
#define BK_WAVE_SCAN(x, DPP, OP)                                 \
  do {                                                           \
    const int l_ = lane_id(), rl_ = l_ & 15;                      \
    auto t_ = DPP<0x111>(x); if (rl_ >= 1) x = OP(t_, x);         \
    t_ = DPP<0x112>(x); if (rl_ >= 2) x = OP(t_, x);              \
    t_ = DPP<0x114>(x); if (rl_ >= 4) x = OP(t_, x);              \
    t_ = DPP<0x118>(x); if (rl_ >= 8) x = OP(t_, x);              \
    t_ = DPP<0x142>(x); if ((l_ & 31) >= 16) x = OP(t_, x);       \
    t_ = DPP<0x143>(x); if (l_ >= 32) x = OP(t_, x);              \
  } while (0)

__device__ __forceinline__ int op_add_i(int a, int b) { return a + b; }
__device__ __forceinline__ float op_add_f(float a, float b) { return a + b; }
__device__ __forceinline__ float op_max_f(float a, float b) { return fmaxf(a, b); }

__device__ __forceinline__ int wave_incl_scan(int x) {
  BK_WAVE_SCAN(x, dpp_i, op_add_i);
  return x;
}

__device__ __forceinline__ int readlane_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// Wave-wide results, returned uniform (in every lane).
__device__ __forceinline__ int wave_sum(int x) {
  BK_WAVE_SCAN(x, dpp_i, op_add_i);
  return readlane_i(x, kWave - 1);
}
// The wave total of x (integer add), uniform: a reduction into lane 63, not a scan — each DPP step
// reads 0 where the scan masks a lane (bound_ctrl, and the rows a broadcast does not write keep the
// `old` 0), so the adds need no lane selects (~12 VALU instead of the scan's ~24).
__device__ __forceinline__ int wave_total(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);  // row_shr:8: lane 15 of a row = its sum
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1 and 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2 and 3
  return readlane_i(x, kWave - 1);
}
__device__ __forceinline__ float wave_sum_f(float x) {
  BK_WAVE_SCAN(x, dpp_f, op_add_f);
  return readlane_f(x, kWave - 1);
}
__device__ __forceinline__ float wave_max_f(float x) {
  BK_WAVE_SCAN(x, dpp_f, op_max_f);
  return readlane_f(x, kWave - 1);
}

// LDS handoff between the lanes of the one wave that owns a board, in the board-level helpers
// below and the search's per-tree stages (mcts_dev.h). Their kernels are 64-thread workgroups
// and keep the barrier; a kernel that runs those stages on one wave of a larger workgroup can
// define BK_BOARD_SYNC() as wave_lds_sync() instead: a wave's LDS operations complete in issue
// order, so only the compiler must be kept from moving LDS accesses across the handoff.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
#ifndef BK_BOARD_SYNC
#define BK_BOARD_SYNC() __syncthreads()
#endif

// Copy a 384-byte state global -> LDS (96 words; lanes 0..63 + 0..31).
__device__ __forceinline__ void load_state(uint32_t* s, const uint32_t* g) {
  const int l = lane_id();
  s[l] = g[l];
  if (l < kStateWords - kWave) s[kWave + l] = g[kWave + l];
}
__device__ __forceinline__ void store_state(uint32_t* g, const uint32_t* s) {
  const int l = lane_id();
  g[l] = s[l];
  if (l < kStateWords - kWave) g[kWave + l] = s[kWave + l];
}

// Forbidden / anchor rows of colour q, packed per row as forb | (anch << 32), into fa[0..N).
//   forb = occupied by anyone, or edge-adjacent to colour q;
//   anch = diagonal-adjacent to colour q, or q's start corner while q has no cell yet.
// Returns true when some anchor cell is free (no free anchor -> no legal placement).
__device__ __forceinline__ bool compute_fa(const DevPreset& dp, const uint32_t* s, int q, uint64_t* fa) {
  const int l = lane_id();
  const int N = dp.N;
  uint32_t own = 0, up = 0, dn = 0, occ = 0;
  if (l < N) {
    own = s[q * kMaxN + l];
    up = l > 0 ? s[q * kMaxN + l - 1] : 0u;
    dn = l + 1 < N ? s[q * kMaxN + l + 1] : 0u;
    occ = s[l] | s[kMaxN + l] | s[2 * kMaxN + l] | s[3 * kMaxN + l];
  }
  const bool first = __ballot(own != 0) == 0ull;
  uint32_t forb = 0, anch = 0;
  if (l < N) {
    forb = (occ | own << 1 | own >> 1 | up | dn) & dp.full_row;
    if (first)
      anch = (l == dp.corner_r(q)) ? (1u << dp.corner_c(q)) : 0u;
    else
      anch = (up << 1 | up >> 1 | dn << 1 | dn >> 1) & dp.full_row;
    fa[l] = (uint64_t)forb | ((uint64_t)anch << 32);
  }
  const bool any = __ballot((anch & ~forb) != 0u) != 0ull;
  BK_BOARD_SYNC();
  return any;
}

// Legal origin columns of one item (orientation x origin row): bit c set <=> the placement
// with origin (r, c) covers no forbidden cell and at least one anchor cell.
__device__ __forceinline__ uint32_t eval_item(uint64_t it, const uint64_t* fa) {
  const int r = (int)((it >> 16) & 31u);
  const int W = (int)((it >> 21) & 31u);
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t cell = (uint32_t)(it >> (34 + 6 * k)) & 63u;
    acc |= fa[r + (int)(cell & 7u)] >> (cell >> 3);
  }
  // The 64-bit shift drags at most 4 anchor bits into bits >= 28 of the forbidden half;
  // W <= 20 keeps them outside the column mask.
  return (uint32_t)(acc >> 32) & ~(uint32_t)acc & ((1u << W) - 1u);
}

__device__ __forceinline__ int item_piece(uint64_t it) { return (int)((it >> 26) & 31u); }
__device__ __forceinline__ int item_base(uint64_t it) { return (int)(it & 0xFFFFu); }
__device__ __forceinline__ int item_W(uint64_t it) { return (int)((it >> 21) & 31u); }

// Full legal-move bitmask of colour q into LDS m32[0..W32pad) (zeroed here).
__device__ __forceinline__ void build_mask(const DevPreset& dp, const uint32_t* s, int q, uint64_t* fa,
                                           uint32_t* m32) {
  const int l = lane_id();
  for (int i = l; i < dp.W32pad; i += kWave) m32[i] = 0u;
  const bool any = compute_fa(dp, s, q, fa);  // contains the barrier ordering the zeroing
  const uint32_t pieces = s[kWPieces + q];
  if (any && pieces) {
    for (int pc = 0; pc < dp.num_pieces; ++pc) {
      if (!((pieces >> pc) & 1u)) continue;  // wave-uniform
      const int end = dp.piece_item_off[pc + 1];
      // four items per lane per trip: their LDS row reads and shifts are independent chains
      for (int i0 = dp.piece_item_off[pc] + l; i0 < end; i0 += 4 * kWave) {
        uint64_t it[4];
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) it[u] = i0 + u * kWave < end ? dp.items[i0 + u * kWave] : 0ull;
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i0 + u * kWave < end ? eval_item(it[u], fa) : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (v[u]) {
            const int base = item_base(it[u]);
            const int w = base >> 5, sh = base & 31;
            atomicOr(&m32[w], v[u] << sh);
            if (sh + item_W(it[u]) > 32) atomicOr(&m32[w + 1], v[u] >> (32 - sh));
          }
        }
      }
    }
  }
  BK_BOARD_SYNC();
}

// Does colour q have at least one legal placement? (early exit on the first hit)
__device__ __forceinline__ bool has_any_legal(const DevPreset& dp, const uint32_t* s, int q, uint64_t* fa) {
  const uint32_t pieces = s[kWPieces + q];
  if (!pieces) return false;
  if (!compute_fa(dp, s, q, fa)) return false;
  const int l = lane_id();
  for (int pc = 0; pc < dp.num_pieces; ++pc) {
    if (!((pieces >> pc) & 1u)) continue;
    const int beg = dp.piece_item_off[pc], end = dp.piece_item_off[pc + 1];
    for (int i0 = beg + l; i0 - l < end; i0 += 2 * kWave) {  // two items per lane per trip
      const int i1 = i0 + kWave;
      const uint64_t a0 = i0 < end ? dp.items[i0] : 0ull;
      const uint64_t a1 = i1 < end ? dp.items[i1] : 0ull;
      const uint32_t v = (i0 < end ? eval_item(a0, fa) : 0u) | (i1 < end ? eval_item(a1, fa) : 0u);
      if (__ballot(v != 0u)) return true;
    }
  }
  return false;
}

// Placement of action a by the player to move, in place on the LDS copy s: the cells, the
// incremental board hash, the piece retired, the ply count. VALIDATE: check legality first
// (returns 1, s untouched, if a is not legal); without it the caller vouches for a (the search's
// stored children are legal by construction). Returns 0 on success.
template <bool VALIDATE = true>
__device__ __forceinline__ int place_action(const DevPreset& dp, uint32_t* s, int a, uint64_t* fa) {
  const int l = lane_id();
  const int p = (int)s[kWToMove];
  if (a < 0 || a >= dp.A) return 1;
  // one 16-B load (the act word and its item together: the descent's placement was two dependent
  // round trips per level, queued behind the policy-row gather of the fused step)
  uint4 e = dp.act_it[a];
  asm volatile("" : "+v"(e.x), "+v"(e.y), "+v"(e.z), "+v"(e.w));  // one load (not the word, then the item)
  const uint32_t ad = e.z;
  const uint64_t it = (uint64_t)e.x | ((uint64_t)e.y << 32);
  const int c = (int)((ad >> 16) & 0xFFu);
  const int pc = (int)(ad >> 24);
  if (VALIDATE) {
    const bool piece_ok = (s[kWPieces + p] >> pc) & 1u;
    compute_fa(dp, s, p, fa);
    const uint32_t v = eval_item(it, fa);
    if (!piece_ok || !((v >> c) & 1u)) return 1;  // wave-uniform
  }
  const int r = (int)((it >> 16) & 31u);
  uint64_t hx = 0;
  if (l < 5) {
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const uint32_t cell = (uint32_t)(it >> (34 + 6 * k)) & 63u;
      if ((int)(cell & 7u) == l) bits |= 1u << (c + (int)(cell >> 3));
    }
    if (bits) {
      const int row = r + l;
      const uint32_t old = s[p * kMaxN + row];
      const uint32_t nw = old | bits;
      hx = (old ? row_key(p, row, old) : 0ull) ^ row_key(p, row, nw);
      s[p * kMaxN + row] = nw;
    }
  }
  // xor-reduce lanes 0..4 (scalar reads)
  const uint64_t hsum = readlane_u64(hx, 0) ^ readlane_u64(hx, 1) ^ readlane_u64(hx, 2) ^ readlane_u64(hx, 3) ^
                        readlane_u64(hx, 4);
  if (l == 0) {
    const uint64_t h = state_hash(s) ^ hsum;
    s[kWHash] = (uint32_t)h;
    s[kWHash + 1] = (uint32_t)(h >> 32);
    s[kWPieces + p] &= ~(1u << pc);
    s[kWPly] += 1u;
  }
  BK_BOARD_SYNC();
  return 0;
}

// The turn after colour p's placement: the next colour in cyclic order that has a legal move (a
// colour found without one is cached as dead); nobody -> game over. ANY(q): does colour q have a
// legal placement on s.
template <typename AnyLegal>
__device__ __forceinline__ void advance_turn(const DevPreset& dp, uint32_t* s, int p, AnyLegal any) {
  const int l = lane_id();
  uint32_t flags = s[kWFlags];
  int next = -1;
  for (int d = 1; d <= dp.P; ++d) {
    const int q = (p + d) % dp.P;
    if ((flags >> (kFlagDeadShift + q)) & 1u) continue;
    if (any(q)) { next = q; break; }
    flags |= 1u << (kFlagDeadShift + q);
  }
  if (next < 0) { flags |= kFlagOver; next = (p + 1) % dp.P; }
  BK_BOARD_SYNC();
  if (l == 0) { s[kWFlags] = flags; s[kWToMove] = (uint32_t)next; }
  BK_BOARD_SYNC();
}

// Functional next state, in place on the LDS copy s (mirrors colosseumrl next_state as called
// at blokus_wrapper.py:103-105): place action a for the player to move, retire the piece,
// update the board hash, then hand the turn to the next colour in cyclic order that has a
// legal move (a colour found without one is cached as dead); nobody -> game over.
// Returns 0 on success, 1 if a is not legal (s untouched).
__device__ __forceinline__ int apply_action(const DevPreset& dp, uint32_t* s, int a, uint64_t* fa) {
  const int p = (int)s[kWToMove];
  if (place_action<true>(dp, s, a, fa)) return 1;
  advance_turn(dp, s, p, [&](int q) { return has_any_legal(dp, s, q, fa); });
  return 0;
}

// Squares placed by colour k.
__device__ __forceinline__ int squares_of(const DevPreset& dp, const uint32_t* s, int k) {
  int n = 0;
  for (int r = 0; r < dp.N; ++r) n += __popc(s[k * kMaxN + r]);
  return n;
}

// Terminal scores (blokus_wrapper.py:164-186): -1 losers, 3 sole winner, 1 each tied winner.
__device__ __forceinline__ void terminal_scores(const DevPreset& dp, const uint32_t* s, double* out) {
  int sq[kMaxP] = {0, 0, 0, 0}, best = -1, nwin = 0;
  for (int k = 0; k < dp.P; ++k) { sq[k] = squares_of(dp, s, k); best = sq[k] > best ? sq[k] : best; }
  for (int k = 0; k < dp.P; ++k) nwin += sq[k] == best;
  for (int k = 0; k < dp.P; ++k) out[k] = sq[k] == best ? (nwin == 1 ? 3.0 : 1.0) : -1.0;
}

// Write the legal ids of LDS mask m32 in ascending order to ids[0..cap); returns K.
__device__ __forceinline__ int compact_ids(const DevPreset& dp, const uint32_t* m32, int32_t* ids, int cap) {
  const int l = lane_id();
  int total = 0;
  for (int w0 = 0; w0 < dp.W32; w0 += kWave) {
    const int w = w0 + l;
    uint32_t bits = w < dp.W32 ? m32[w] : 0u;
    const int cnt = __popc(bits);
    const int incl = wave_incl_scan(cnt);
    int pos = total + incl - cnt;
    while (bits) {
      const int b = __ffs(bits) - 1;
      bits &= bits - 1u;
      if (pos < cap) ids[pos] = w * 32 + b;
      ++pos;
    }
    total += readlane_i(incl, kWave - 1);
  }
  return total;
}

}  // namespace bk
