// mcts_dev.h — device state of the batched search and its per-tree stages (select_tree,
// leaf_logits_tree, expand_tree), shared by the per-stage kernels (mcts.hip: one launch per stage
// over all trees) and the fused leaf step (k_leaf_step / k_leaf_step_ov, mcts.hip). Design notes
// and the reference mapping: mcts.hip.
#pragma once
#include <cmath>
#include <vector>

#include "../../include/blokus_engine.h"
#include "ctx.h"
#include "legal_rows.h"

namespace bk {

constexpr int kMaxDepth = 96;
constexpr int kExpandLdsIds = 2048;  // leaf ids staged in LDS up to this K
constexpr int kGatherRegs = 16;      // logits gathered into registers: K <= 1024 in one round
constexpr int kLeafCap = 2048;       // sparse leaf policy: legal ids per leaf (bk_mcts_leaf_logits)
constexpr int kLeafBlocks = 4;  // workgroups per tree in k_leaf_logits
constexpr int kMaxFeat = 2048;       // policy-feature length staged in LDS
constexpr int kLeafQ = 16;           // leaf logits: float4s of a W row a lane holds (F <= 1024)

// Diagnostic build only (-DBK_STAMPS, `make diag`): per-tree s_memtime stamps at phase
// boundaries of k_select / k_expand_backup; never compiled into the shipped library.
#ifdef BK_STAMPS
static __device__ unsigned long long g_stamps[2][4096][8];
#define BK_STAMP(k, i) \
  do { if (lane_id() == 0 && blockIdx.x < 4096) g_stamps[k][blockIdx.x][i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define BK_STAMP(k, i) do { } while (0)
#endif  // > 84 = most placements a 4-player game can still make

// One node of a tree's hash table, 16 B (one dwordx4 per lane per probe): the board key (0 =
// empty slot), the node's first child in the tree's child region and its child count. A probe
// thus yields the node's children directly; the visit sum the PUCT score needs (mcts.py:41-46
// sums N over the children) comes from the children's N, loaded with the rest of their stats.
struct __attribute__((aligned(16))) TabEntry {
  unsigned long long key;
  uint32_t off;  // first child, relative to the tree's child region
  int32_t K;     // number of children
};

struct DevMcts {
  int T, node_cap, TS;  // TS = table slots per tree (power of two)
  int64_t child_cap_per_tree;
  TabEntry* tab;        // [T*TS]
  int32_t* tree_nodes;  // [T] nodes in the tree (capacity check against node_cap)
  int64_t* tree_children;  // [T] children used in the tree's region
  int32_t* ch_id;       // [T*cpt]
  uint32_t* ch_N;
  double* ch_Q;
  float* ch_P;
  int64_t* path_child;  // [T*kMaxDepth] global child index
  int32_t* path_pl;     // [T*kMaxDepth] player to move at the child (scores index)
  int32_t* depth;       // [T]
  uint32_t* leaf_state; // [T*kStateWords]
  int32_t* leaf_status; // [T]
  double* leaf_scores;  // [T*kMaxP]
  uint64_t* leaf_mask;  // [T*W64] internal copy of the leaf bitmask
  int32_t* leaf_ids;    // [T*kLeafCap] sparse leaf policy: legal ids (ascending)
  float* leaf_logit;    // [T*kLeafCap] their logits
  int32_t* leaf_K;      // [T]
  unsigned long long* counters;  // [8] (errors)
  unsigned long long* tree_ctr;  // [T*8] per-tree counters: uncontended atomics, summed on read
};

// add v to counter k of tree t: fire-and-forget, on an address no other tree touches (every
// tree on one shared counter serialised 256 atomics per stage in L2, which the workgroup's next
// barrier then waited for)
__device__ __forceinline__ void ctr_add(const struct DevMcts& m, int t, int k, unsigned long long v) {
  atomicAdd(&m.tree_ctr[(size_t)t * 8 + k], v);
}

enum { kCtrLevels = 2, kCtrExpanded = 3, kCtrTerminal = 4, kCtrErr = 5, kCtrScanned = 6, kCtrLeafK = 7 };
enum { kErrChildPool = 1, kErrTable = 2, kErrDepth = 4, kErrIllegal = 8, kErrMissingRoot = 16, kErrLeafCap = 32 };

__device__ __forceinline__ uint64_t table_key(const uint32_t* s) {
  const uint64_t h = state_hash(s);
  return h ? h : 1ull;
}

// Wave-parallel linear probe, 64 whole entries per round trip. Found: true, the node's child
// offset (global) and count. Absent: false and *free_slot = the first empty slot of the probe
// sequence (-1 if the table is full).
__device__ __forceinline__ bool table_find(const DevMcts& m, int t, uint64_t key, int64_t& off, int& K,
                                           int* free_slot) {
  const int l = lane_id();
  const uint32_t mask = (uint32_t)m.TS - 1u;
  const uint32_t start = (uint32_t)(key ^ (key >> 29)) & mask;
  const TabEntry* tab = m.tab + (size_t)t * m.TS;
  for (int p0 = 0; p0 < m.TS; p0 += kWave) {
    const uint32_t slot = (start + (uint32_t)(p0 + l)) & mask;
    // the whole 16-B entry in one load: left alone the compiler loads the key, compares, and only
    // then loads (off, K) in the hit branch — a second dependent round trip per probe
    uint4 ev = *reinterpret_cast<const uint4*>(tab + slot);
    asm volatile("" : "+v"(ev.x), "+v"(ev.y), "+v"(ev.z), "+v"(ev.w));
    TabEntry e;
    e.key = (unsigned long long)ev.x | ((unsigned long long)ev.y << 32);
    e.off = ev.z;
    e.K = (int32_t)ev.w;
    const uint64_t hit = __ballot(e.key == key);
    const uint64_t emp = __ballot(e.key == 0ull);
    if (hit) {
      const int src = __ffsll((unsigned long long)hit) - 1;
      off = (int64_t)t * m.child_cap_per_tree + (uint32_t)readlane_i((int)e.off, src);
      K = readlane_i(e.K, src);
      return true;
    }
    if (emp) {
      const int src = __ffsll((unsigned long long)emp) - 1;
      if (free_slot) *free_slot = readlane_i((int)slot, src);
      return false;
    }
  }
  if (free_slot) *free_slot = -1;
  return false;
}

// argmax over (value, index): larger value wins, ties -> smaller index (np.argmax's first max).
// DPP prefix-argmax; lane 63 ends with the wave's argmax, returned uniform.
__device__ __forceinline__ void wave_argmax(double& best, int& bi) {
  const int l = lane_id(), rl = l & 15;
#define BK_ARGMAX_STEP(CTRL, COND)                                 \
  {                                                               \
    const double tb = dpp_d<CTRL>(best);                          \
    const int ti = dpp_i<CTRL>(bi);                               \
    if ((COND) && (tb > best || (tb == best && ti < bi))) {        \
      best = tb;                                                  \
      bi = ti;                                                    \
    }                                                             \
  }
  BK_ARGMAX_STEP(0x111, rl >= 1)
  BK_ARGMAX_STEP(0x112, rl >= 2)
  BK_ARGMAX_STEP(0x114, rl >= 4)
  BK_ARGMAX_STEP(0x118, rl >= 8)
  BK_ARGMAX_STEP(0x142, (l & 31) >= 16)
  BK_ARGMAX_STEP(0x143, l >= 32)
#undef BK_ARGMAX_STEP
  bi = readlane_i(bi, kWave - 1);
  const uint64_t u = readlane_u64((uint64_t)__double_as_longlong(best), kWave - 1);
  best = __longlong_as_double((long long)u);
}

// PUCT choice at a node (mcts.py:41-46): argmax_i Q_i + cpuct*P_i*sqrt(sum N + 1e-6)/(1+N_i);
// also returns the chosen child's action id. Up to kSelB * 64 children (every 20x20 node) in one
// memory round trip: each lane loads all its children's (P, N, Q, id) first, the visit sum is
// the wave's integer sum of N, then the lane scans its children in index order.
constexpr int kSelB = 12;
// waves that take orientations in a leaf bitmask (the rest idle): 8 slices (every 8th
// orientation) — each claiming wave pays its own row context, so 16 slices cost more setup than
// they save (self-play +0.3% at plies 2-8 and 8-18 vs 16; 4: in between; round 6, lib_ab.sh)
constexpr int kMaskWpb = 8;
// eps: the term under the square root (mcts.py:43: 1e-6 with epsilon_fix, the default, else 0)
__device__ __forceinline__ int select_child(const DevMcts& m, int64_t off, int K, double cp, int& id_out,
                                            double eps = 1e-6) {
  const int l = lane_id();
  double best = -INFINITY;
  int bi = 0x7fffffff, bid = 0;
  const float* P = m.ch_P + off;
  const uint32_t* Nn = m.ch_N + off;
  const double* Q = m.ch_Q + off;
  const int32_t* ID = m.ch_id + off;
  if (K <= kSelB * kWave) {
    float p[kSelB];
    uint32_t nn[kSelB];
    double q[kSelB];
    int32_t id[kSelB];
    // unconditional loads at a clamped index (K >= 1), so the compiler issues all of them before
    // the first wait; lanes past K are masked out of the sum and the scan
#pragma unroll
    for (int u = 0; u < kSelB; ++u) {
      const int i = min(l + u * kWave, K - 1);
      p[u] = P[i];
      nn[u] = Nn[i];
      q[u] = Q[i];
      id[u] = ID[i];
    }
    // every load issued before the first wait (one round trip): the compiler would otherwise
    // wait for N's loads (the visit sum) before issuing the others
#pragma unroll
    for (int u = 0; u < kSelB; ++u) asm volatile("" : "+v"(p[u]), "+v"(nn[u]), "+v"(q[u]), "+v"(id[u]));
    uint32_t vs = 0u;
#pragma unroll
    for (int u = 0; u < kSelB; ++u) vs += l + u * kWave < K ? nn[u] : 0u;
    const double sq = sqrt((double)(uint32_t)wave_sum((int)vs) + eps);
#pragma unroll
    for (int u = 0; u < kSelB; ++u) {
      const int i = l + u * kWave;
      if (i < K) {
        const double h = q[u] + ((cp * (double)p[u]) * sq) / (1.0 + (double)nn[u]);
        if (h > best) { best = h; bi = i; bid = id[u]; }
      }
    }
  } else {  // two passes: the visit sum, then the scan
    uint32_t vs = 0u;
    for (int i = l; i < K; i += kWave) vs += Nn[i];
    const double sq = sqrt((double)(uint32_t)wave_sum((int)vs) + eps);
    for (int i = l; i < K; i += kWave) {
      const double h = Q[i] + ((cp * (double)P[i]) * sq) / (1.0 + (double)Nn[i]);
      if (h > best) { best = h; bi = i; bid = ID[i]; }
    }
  }
  wave_argmax(best, bi);
  id_out = readlane_i(bid, bi & (kWave - 1));  // the owning lane's best is the wave's best
  return bi;
}

// k_select's descent on tree t, by one wave: from the root to a board not in the tree or a
// terminal board, the path recorded (mcts.py:37-50); the leaf state stays in LDS for select_leaf.
// lds = kStateWords + 2 kMaxN + W32pad words. Returns the leaf status (wave-uniform): 0 inactive
// tree or error, 1 a leaf for the net, 2 a terminal board.
// pend_key / pend (k_leaf_step_ov): the node of board key pend_key is being added by other waves
// of the workgroup (its table entry: flag pend[0]; then its children: pend[1]; pend[2] != 0 when
// the entry was not made). Before the descent probes that key it waits for the entry, and before
// it reads that node's children for them (flags set with release semantics).
__device__ __forceinline__ void wait_flag_acquire(int* flag) {
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
  asm volatile("buffer_inv sc0" ::: "memory");
}
__device__ __forceinline__ int select_descend(const DevPreset& dp, const DevMcts& m, int t,
                                              const uint32_t* __restrict__ roots, const int32_t* __restrict__ active,
                                              double cpuct, int32_t* __restrict__ status_out, uint32_t* lds,
                                              uint64_t pend_key = 0, int* const* pend = nullptr,
                                              double root_eps = 1e-6) {
  uint32_t* s = lds;
  uint64_t* fa = reinterpret_cast<uint64_t*>(lds + kStateWords);
  const int l = lane_id();
  if (active && !active[t]) {
    if (l == 0) {
      m.leaf_status[t] = 0;
      if (status_out) status_out[t] = 0;
      m.depth[t] = 0;
    }
    return 0;
  }
  BK_STAMP(0, 0);
  load_state(s, roots + (size_t)t * kStateWords);
  BK_BOARD_SYNC();
  BK_STAMP(0, 1);
  double cp = cpuct, eps = root_eps;
  int depth = 0, err = 0;
  long long scanned = 0;
  // the path records of levels 0..63 stay in lane `level`'s registers until the descent ends: a
  // store per level would make every next level's first load wait for it (vmcnt counts stores too),
  // and under the fused step's gather a store takes as long as a round trip to be acknowledged
  int64_t rec_child = 0;
  int rec_pl = 0;
#ifdef BK_STAMPS
  unsigned long long t_probe = 0, t_child = 0, t_apply = 0, t_adv = 0;
#define BK_TACC(v, stmt)                                         \
  do {                                                           \
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime(); \
    stmt;                                                        \
    v += __builtin_amdgcn_s_memtime() - t0_;                     \
  } while (0)
#else
#define BK_TACC(v, stmt) \
  do {                   \
    stmt;                \
  } while (0)
#endif
  for (;;) {
    int64_t off;
    int Kn;
    bool found;
    const uint64_t key = table_key(s);
    int* pend_children = nullptr;
    if (pend && key == pend_key) {
      wait_flag_acquire(pend[0]);  // the new node's table entry (or its failure) is published
      if (readlane_i(*pend[2], 0) == 0) pend_children = pend[1];
      pend = nullptr;
    }
    BK_TACC(t_probe, found = table_find(m, t, key, off, Kn, nullptr));
    if (!found) break;
    if (Kn <= 0) { err |= kErrIllegal; break; }  // a stored node always has a legal move
    if (pend_children) wait_flag_acquire(pend_children);  // and its children are stored
    scanned += Kn;
    int a, ci;
    BK_TACC(t_child, ci = select_child(m, off, Kn, cp, a, eps));
    // no child won the argmax: every PUCT score was NaN (a NaN prior or value from a diverged
    // net); flag it and stop before the unchecked placement and the path record
    if (ci < 0 || ci >= Kn) { err |= kErrIllegal; break; }
    if (depth >= kMaxDepth) { err |= kErrDepth; break; }
    // the child's action is legal by construction (its id came from the node's legal mask)
    const int p = (int)s[kWToMove];
    int bad;
    BK_TACC(t_apply, bad = place_action<false>(dp, s, a, fa));
    BK_TACC(t_adv, if (!bad) advance_turn(dp, s, p, [&](int q) { return rows_any_legal(dp, s, q); }));
    if (bad) { err |= kErrIllegal; break; }
    if (depth < kWave) {
      if (l == depth) {
        rec_child = off + ci;
        rec_pl = (int)s[kWToMove];
      }
    } else if (l == 0) {  // levels 64..kMaxDepth-1 (never at 20x20)
      const size_t pi = (size_t)t * kMaxDepth + depth;
      m.path_child[pi] = off + ci;
      m.path_pl[pi] = (int)s[kWToMove];
    }
    ++depth;
    cp = 1.0;    // the recursive call of mcts.py:50 passes no cpuct
    eps = 1e-6;  // nor epsilon_fix (its default True)
  }
  if (l < depth && l < kWave) {
    const size_t pi = (size_t)t * kMaxDepth + l;
    m.path_child[pi] = rec_child;
    m.path_pl[pi] = rec_pl;
  }
  BK_STAMP(0, 2);
#ifdef BK_STAMPS
  if (lane_id() == 0 && blockIdx.x < 4096) {
    g_stamps[0][blockIdx.x][6] = t_probe;
    g_stamps[0][blockIdx.x][7] = t_child;
    g_stamps[1][blockIdx.x][7] = t_apply;  // (slots 6, 7 of the expand record are free)
    g_stamps[1][blockIdx.x][6] = t_adv;
  }
#endif
#undef BK_TACC
  int status;
  if (err) {
    status = 0;
  } else if (s[kWFlags] & kFlagOver) {
    status = 2;
    if (l == 0) terminal_scores(dp, s, m.leaf_scores + (size_t)t * kMaxP);
  } else {
    status = 1;
  }
  if (l == 0) {
    m.leaf_status[t] = status;
    if (status_out) status_out[t] = status;
    m.depth[t] = depth;
    ctr_add(m, t, kCtrLevels, (unsigned long long)depth);
    ctr_add(m, t, kCtrScanned, (unsigned long long)scanned);
    if (status == 2) ctr_add(m, t, kCtrTerminal, 1ull);
    if (err) atomicOr(&m.counters[kCtrErr], (unsigned long long)err);
  }
  return status;
}

// The observation rows of tree t's leaf (state s in LDS) and its state, by NW waves (thread tid of
// NW * 64): zeros unless status 1. select_leaf's rows, callable on their own.
template <int NW>
__device__ __forceinline__ void leaf_obs_rows(const DevPreset& dp, const DevMcts& m, int t, int status,
                                              float* __restrict__ obs, const uint32_t* s, int tid) {
  if (status == 1 && tid < kWave) store_state(m.leaf_state + (size_t)t * kStateWords, s);
  const int obs_len = 2 * dp.P * dp.N * dp.N;
  float* o = obs ? obs + (size_t)t * obs_len : nullptr;
  const int tm = (int)s[kWToMove];
  const int rows = 2 * dp.P * dp.N;
  for (int pr = tid; o && pr < rows; pr += NW * kWave) {
    const int plane = pr / dp.N, r = pr - plane * dp.N;
    uint32_t bits = 0u;
    if (status == 1) bits = plane < dp.P ? s[plane * kMaxN + r] : ((plane - dp.P) == tm ? dp.full_row : 0u);
    float* dst = o + pr * dp.N;
    if ((dp.N & 3) == 0) {
      for (int c = 0; c < dp.N; c += 4)
        *reinterpret_cast<float4*>(dst + c) = make_float4((float)((bits >> c) & 1u), (float)((bits >> (c + 1)) & 1u),
                                                          (float)((bits >> (c + 2)) & 1u), (float)((bits >> (c + 3)) & 1u));
    } else {
      for (int c = 0; c < dp.N; ++c) dst[c] = (float)((bits >> c) & 1u);
    }
  }
}

// The leaf of a descent (state in LDS), by the NW waves of the workgroup (wave = this one's
// index; 1 = the descending wave alone): for a leaf (status 1) the mover's legal bitmask (the
// orientations split over the waves) and the leaf state to global memory, and for every tree
// the observation rows the net reads (zeros unless status 1). obs and mask_out may be null.
// BUILT: the bitmask is already in LDS (k_leaf_step_ov builds it with mask_slices_claim).
// OBS: write the observation rows here (k_leaf_step_ov's descending wave writes them itself, with
// leaf_obs_rows, while the other waves still compute logits).
template <int NW, bool BUILT = false, bool OBS = true>
__device__ __forceinline__ void select_leaf(const DevPreset& dp, const DevMcts& m, int t, int status,
                                            float* __restrict__ obs, uint64_t* __restrict__ mask_out, uint32_t* lds,
                                            int wave) {
  const uint32_t* s = lds;
  uint32_t* m32 = lds + kStateWords + 2 * kMaxN;
  const int l = lane_id(), tid = wave * kWave + l;
  const int obs_len = 2 * dp.P * dp.N * dp.N;
  if (status == 1) {
    if (BUILT)
      ;
    else if (NW == 1)
      build_mask_rows(dp, s, (int)s[kWToMove], m32);
    else
      build_mask_rows_wg<(NW > kMaskWpb ? kMaskWpb : NW)>(dp, s, (int)s[kWToMove], m32, wave);
    BK_STAMP(0, 3);
    uint64_t* mo = m.leaf_mask + (size_t)t * dp.W64;
    uint64_t* mo2 = mask_out ? mask_out + (size_t)t * dp.W64 : nullptr;
    for (int j = tid; j < dp.W64; j += NW * kWave) {
      const uint64_t w = (uint64_t)m32[2 * j] | ((uint64_t)m32[2 * j + 1] << 32);
      mo[j] = w;
      if (mo2) mo2[j] = w;
    }
    if (wave == 0 && OBS) store_state(m.leaf_state + (size_t)t * kStateWords, s);
  }
  BK_STAMP(0, 4);
  if (!OBS) return;
  // observation row (zeros unless the leaf needs the net): thread = (plane, board row), the row's
  // N floats as float4 stores when N is a multiple of 4 (no per-cell index arithmetic)
  float* o = obs ? obs + (size_t)t * obs_len : nullptr;
  const int tm = (int)s[kWToMove];
  const int rows = 2 * dp.P * dp.N;
  for (int pr = tid; o && pr < rows; pr += NW * kWave) {
    const int plane = pr / dp.N, r = pr - plane * dp.N;
    uint32_t bits = 0u;
    if (status == 1) bits = plane < dp.P ? s[plane * kMaxN + r] : ((plane - dp.P) == tm ? dp.full_row : 0u);
    float* dst = o + pr * dp.N;
    if ((dp.N & 3) == 0) {
      for (int c = 0; c < dp.N; c += 4)
        *reinterpret_cast<float4*>(dst + c) = make_float4((float)((bits >> c) & 1u), (float)((bits >> (c + 1)) & 1u),
                                                          (float)((bits >> (c + 2)) & 1u), (float)((bits >> (c + 3)) & 1u));
    } else {
      for (int c = 0; c < dp.N; ++c) dst[c] = (float)((bits >> c) & 1u);
    }
  }
  BK_STAMP(0, 5);
}

// k_select's work on tree t by one wave: descent + leaf.
__device__ __forceinline__ int select_tree(const DevPreset& dp, const DevMcts& m, int t,
                                           const uint32_t* __restrict__ roots, const int32_t* __restrict__ active,
                                           double cpuct, int32_t* __restrict__ status_out, float* __restrict__ obs,
                                           uint64_t* __restrict__ mask_out, uint32_t* lds) {
  const int status = select_descend(dp, m, t, roots, active, cpuct, status_out, lds);
  select_leaf<1>(dp, m, t, status, obs, mask_out, lds, 0);
  return status;
}

// The policy head's last layer restricted to the leaf's legal ids (the only logits the
// expansion reads): logit[j] = W[id_j] . feat[t] + bias[id_j] for the K legal ids of tree t's
// leaf, instead of the dense [T, A] Linear (blokus_nnet.py:147-148) — K ~ 200 of A = 30433.
// kLeafBlocks workgroups per tree each compact the leaf bitmask (ascending ids) and take a
// contiguous share of the ids; a wave computes four dot products at a time (16 lanes each) over
// the feature row staged in LDS, W rows read as coalesced float4s, several loads in flight.
//
// The leaf's legal ids and feature row into LDS (all threads of the workgroup; two barriers):
// lds = W32pad mask words | kLeafCap ids | F features. Returns K (also stored to leaf_K when c is
// 0), or -1 when tree t has no leaf for the net (block-uniform; no barrier taken then).
__device__ __forceinline__ int leaf_logits_prologue(const DevPreset& dp, const DevMcts& m, int t, int c,
                                                    const float* __restrict__ feat, int64_t ldf, int F,
                                                    uint32_t* lds) {
  uint32_t* m32 = lds;                                                   // W32pad words
  int32_t* ids = reinterpret_cast<int32_t*>(lds + dp.W32pad);            // kLeafCap
  float* f = reinterpret_cast<float*>(lds + dp.W32pad + kLeafCap);       // F (16-B aligned: W32pad % 4 == 0)
  __shared__ int Ksh;
  if (m.leaf_status[t] != 1) return -1;  // block-uniform: no leaf to evaluate
  const uint64_t* lm = m.leaf_mask + (size_t)t * dp.W64;
  for (int j = threadIdx.x; j < dp.W64; j += blockDim.x) {
    const uint64_t w = lm[j];
    m32[2 * j] = (uint32_t)w;
    m32[2 * j + 1] = (uint32_t)(w >> 32);
  }
  const float* ft = feat + (size_t)t * ldf;
  for (int i = threadIdx.x; i < F; i += blockDim.x) f[i] = ft[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (wave == 0) {
    const int K = compact_ids(dp, m32, ids, kLeafCap);
    if (l == 0) Ksh = K;
  }
  __syncthreads();
  const int K = Ksh;
  if (c == 0 && threadIdx.x == 0) {
    m.leaf_K[t] = K;
    if (K > kLeafCap) atomicOr(&m.counters[kCtrErr], (unsigned long long)kErrLeafCap);
  }
  return K;
}

// The logits of ids [lo, hi) of the prologue's LDS id list by wave `wave` of nw: logit j to
// out_lg[j] (global or LDS), its id to out_ids[j] when out_ids is given. Every logit is summed in
// the same order whichever wave takes it, so any wave split gives the same values, bitwise.

// One logit's dot product W[id] . f by the 16 lanes of a quarter wave (sub = lane & 15): a lane
// sums every 16th float4 — whole trips of four alternate two partial sums, the rest go to the
// first — and the 16 partial sums meet in 4 xor-shuffles. The single definition of the leaf
// logits' arithmetic: k_leaf_logits and the fused leaf steps all sum through it, so their logits
// agree bitwise.
// SKIP: a W float4 is loaded only where the lane's four features are not all zero (the policy
// features are a ReLU's output: ~half of them, a third of whole 128-B lines, are zero); a skipped
// float4 enters the sum as 0 . 0 = +0, exactly what 0 . w would add (a sum that starts at +0 never
// becomes -0, and +-0 leaves a non-zero sum unchanged), so the logits are bitwise those without the
// skip for finite weights — and the skipped lines never leave the Infinity Cache.
// The skipped loads are raw buffer loads at an out-of-range offset (the hardware's range check
// returns zeros without a memory access), so the four loads of a trip stay branch-free and in
// flight together (exec-masked branches made the compiler wait for each).
__device__ __forceinline__ bool nz4(const float4& x) { return x.x != 0.f || x.y != 0.f || x.z != 0.f || x.w != 0.f; }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t w_rsrc(const float* W, unsigned bytes) {
  const uintptr_t a = (uintptr_t)W;
  const uintptr_t u = ((uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                      (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 w_load(__amdgpu_buffer_rsrc_t rs, unsigned off, bool use) {
  using u32x4 = unsigned __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, use ? off : 0xFFFFFFF0u, 0, 0));
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
template <bool SKIP = false>
__device__ __forceinline__ float row_dot16(const float4* __restrict__ r, const float4* f4, int F4, int sub,
                                           __amdgpu_buffer_rsrc_t rs, unsigned roff) {
  float a0 = 0.f, a1 = 0.f;
  int q = sub;
  for (; q + 48 < F4; q += 64) {
    const float4 x0 = f4[q], x1 = f4[q + 16], x2 = f4[q + 32], x3 = f4[q + 48];
    float4 w0, w1, w2, w3;
    if (SKIP) {
      w0 = w_load(rs, roff + 16u * q, nz4(x0));
      w1 = w_load(rs, roff + 16u * (q + 16), nz4(x1));
      w2 = w_load(rs, roff + 16u * (q + 32), nz4(x2));
      w3 = w_load(rs, roff + 16u * (q + 48), nz4(x3));
    } else {
      w0 = r[q];
      w1 = r[q + 16];
      w2 = r[q + 32];
      w3 = r[q + 48];
    }
    a0 += w0.x * x0.x + w0.y * x0.y + w0.z * x0.z + w0.w * x0.w;
    a1 += w1.x * x1.x + w1.y * x1.y + w1.z * x1.z + w1.w * x1.w;
    a0 += w2.x * x2.x + w2.y * x2.y + w2.z * x2.z + w2.w * x2.w;
    a1 += w3.x * x3.x + w3.y * x3.y + w3.z * x3.z + w3.w * x3.w;
  }
  for (; q < F4; q += 16) {
    const float4 x0 = f4[q];
    const float4 w0 = SKIP ? w_load(rs, roff + 16u * q, nz4(x0)) : r[q];
    a0 += w0.x * x0.x + w0.y * x0.y + w0.z * x0.z + w0.w * x0.w;
  }
  float a = a0 + a1;
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) a += __shfl_xor(a, o, 16);
  return a;
}

template <int R = 1>
__device__ __forceinline__ void leaf_logits_dots(const DevPreset& dp, int lo, int hi, int wave, int nw,
                                                 const float* __restrict__ W, const float* __restrict__ bias, int F,
                                                 const uint32_t* lds, int32_t* out_ids, float* out_lg,
                                                 int skipz = 0) {
  const int32_t* ids = reinterpret_cast<const int32_t*>(lds + dp.W32pad);
  const float* f = reinterpret_cast<const float*>(lds + dp.W32pad + kLeafCap);
  const int l = threadIdx.x & 63;
  if (R > 1 && (F & 3) == 0 && F <= 64 * kLeafQ) {
    // R x four ids per wave at a time, 16 lanes each: a lane holds every 16th float4 of each of its
    // R rows (<= kLeafQ a row), all loads issued before the first is used — one memory round trip
    // per R x 4 ids — then sums them in the order of the streaming loop below (the same logits,
    // bitwise); the 16-lane partial sums meet in 4 xor-shuffles
    const int F4 = F >> 2;
    const float4* f4 = reinterpret_cast<const float4*>(f);
    const int sub = l & 15, quad = l >> 4;
    for (int j0 = lo + 4 * R * wave; j0 < hi; j0 += 4 * R * nw) {
      int jr[R], idr[R];
      float4 w[R][kLeafQ];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        jr[u] = j0 + 4 * u + quad;
        idr[u] = ids[jr[u] < hi ? jr[u] : lo];
        const float4* r = reinterpret_cast<const float4*>(W + (size_t)idr[u] * F);
#pragma unroll
        for (int k = 0; k < kLeafQ; ++k) w[u][k] = r[sub + 16 * k < F4 ? sub + 16 * k : F4 - 1];
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int k = 0; k < kLeafQ; ++k) {
          const int q = sub + 16 * k;
          if (q < F4) {
            const float4 x = f4[q];
            const float d = w[u][k].x * x.x + w[u][k].y * x.y + w[u][k].z * x.z + w[u][k].w * x.w;
            // streaming order: whole trips of four (first q + 48 < F4) alternate a0, a1; the rest a0
            if ((k & 1) && sub + 16 * (k | 3) < F4)
              a1 += d;
            else
              a0 += d;
          }
        }
        float a = a0 + a1;
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) a += __shfl_xor(a, o, 16);
        if (sub == 0 && jr[u] < hi) {
          if (out_ids) out_ids[jr[u]] = idr[u];
          out_lg[jr[u]] = a + bias[idr[u]];
        }
      }
    }
  } else if ((F & 3) == 0) {
    // the streaming path (the default, R = 1): every 16th float4 of the row with up to 4 loads in
    // flight; the 16-lane partial sums meet in 4 xor-shuffles
    const int F4 = F >> 2;
    const float4* f4 = reinterpret_cast<const float4*>(f);
    const int sub = l & 15, quad = l >> 4;
    // skipz: the W table as a buffer resource (its byte size must fit the 31-bit range)
    const uint64_t wbytes = (uint64_t)dp.A * (uint64_t)F * 4u;
    const bool sk = skipz && wbytes < 0x7FFFFFF0ull;
    const __amdgpu_buffer_rsrc_t wrs = w_rsrc(W, sk ? (unsigned)wbytes : 0u);
    for (int j0 = lo + 4 * wave; j0 < hi; j0 += 4 * nw) {
      const int j = j0 + quad;
      const bool ok = j < hi;
      const int id = ids[ok ? j : lo];
      const float4* wr = reinterpret_cast<const float4*>(W + (size_t)id * F);
      const float a = sk ? row_dot16<true>(wr, f4, F4, sub, wrs, (unsigned)id * (unsigned)F * 4u)
                            : row_dot16<false>(wr, f4, F4, sub, wrs, 0u);
      if (sub == 0 && ok) {
        if (out_ids) out_ids[j] = id;
        out_lg[j] = a + bias[id];
      }
    }
  } else {
    for (int j = lo + wave; j < hi; j += nw) {
      const int id = ids[j];
      const float* r = W + (size_t)id * F;
      float a = 0.f;
      for (int q = l; q < F; q += kWave) a += r[q] * f[q];
      a = wave_sum_f(a);
      if (l == 0) {
        if (out_ids) out_ids[j] = id;
        out_lg[j] = a + bias[id];
      }
    }
  }
}


// k_leaf_logits' work on tree t by a workgroup of any multiple of 64 threads, share c of nc, R x 4
// ids per wave at a time: lds = W32pad + kLeafCap + F words.
template <int R = 1>
__device__ __forceinline__ void leaf_logits_tree(const DevPreset& dp, const DevMcts& m, int t, int c, int nc,
                                                 const float* __restrict__ feat, int64_t ldf, int F,
                                                 const float* __restrict__ W, const float* __restrict__ bias,
                                                 uint32_t* lds) {
  const int K = leaf_logits_prologue(dp, m, t, c, feat, ldf, F, lds);
  if (K < 0 || K > kLeafCap) return;
  const int lo = (int)((int64_t)K * c / nc), hi = (int)((int64_t)K * (c + 1) / nc);
  leaf_logits_dots<R>(dp, lo, hi, (int)(threadIdx.x >> 6), (int)(blockDim.x >> 6), W, bias, F, lds,
                      m.leaf_ids + (size_t)t * kLeafCap, m.leaf_logit + (size_t)t * kLeafCap);
}

// prior_mode 0: logp = the net's log-probabilities over all A ids -> masked log-softmax + exp
//               (get_valid_dist, neural_network.py:159-173);
// prior_mode 2: the sparse leaf logits of k_leaf_logits (ids + logits of the legal ids) ->
//               the same softmax, no compaction or gather here;
// prior_mode 1: logp holds the prior itself at the legal ids (test hook: identical P fed to the
//               reference and to this engine).
// k_expand_backup's work on tree t, by one wave: lds = W32pad + kExpandLdsIds words
// The tree's scalars, the table probe, the logits and the path records are loaded in as few
// dependent round trips as the data allows: (1) status, depth, node/child counters, leaf key and
// K together; (2) the probe, the logit gather and the path records together; (3) the path
// children's N and Q; then the stores.
__device__ __forceinline__ void expand_tree(const DevPreset& dp, const DevMcts& m, int t, const float* __restrict__ logp,
                                            const float* __restrict__ values, int prior_mode, uint32_t* lds) {
  uint32_t* m32 = lds;  // W32pad words
  __shared__ double vsh[kMaxP];
  const int l = lane_id();
  const bool sparse = prior_mode == 2;
  // (1) independent per-tree loads
  const int status = m.leaf_status[t];
  const int depth = m.depth[t];
  const int node = m.tree_nodes[t];
  const int64_t used = m.tree_children[t];
  const int leafK = sparse ? m.leaf_K[t] : 0;
  const uint64_t key = table_key(m.leaf_state + (size_t)t * kStateWords);
  if (status == 0) return;
  BK_STAMP(1, 0);
  // (2a) the path records (lane d < depth: level d), issued before the expansion's loads
  const size_t pi = (size_t)t * kMaxDepth + l;
  const bool on_path = l < depth;  // depth <= kMaxDepth = 96: levels 64.. are handled below
  const int64_t pchild = on_path ? m.path_child[pi] : 0;
  const int ppl = on_path ? m.path_pl[pi] : 0;
  if (status == 1) {
    int err = 0;
    const int64_t room = m.child_cap_per_tree - used;
    const int64_t off = (int64_t)t * m.child_cap_per_tree + used;
    int32_t* ids_lds = reinterpret_cast<int32_t*>(m32 + dp.W32pad);
    const int cap_lds = kExpandLdsIds;
    int K;
    bool in_lds;
    BK_STAMP(1, 1);
    if (sparse) {
      K = leafK;
      in_lds = true;  // the ids are in leaf_ids: write them into the child region below
      if (K > kLeafCap) err |= kErrLeafCap;
    } else {
      const uint64_t* lm = m.leaf_mask + (size_t)t * dp.W64;
      for (int j = l; j < dp.W64; j += kWave) {
        const uint64_t w = lm[j];
        m32[2 * j] = (uint32_t)w;
        m32[2 * j + 1] = (uint32_t)(w >> 32);
      }
      BK_BOARD_SYNC();
      // legal ids, ascending (np.where order, mcts.py:64): into LDS when K fits, else straight
      // into the tree's child region
      K = compact_ids(dp, m32, ids_lds, cap_lds);
      in_lds = K <= cap_lds;
      if (!in_lds)
        K = compact_ids(dp, m32, m.ch_id + off, room > 0 ? (int)(room < 0x7fffffff ? room : 0x7fffffff) : 0);
      BK_BOARD_SYNC();
    }
    BK_STAMP(1, 2);
    if (node >= m.node_cap) err |= kErrTable;
    if (K > room) err |= kErrChildPool;
    // (2b) the logit gather (all of a lane's loads issued before any is used, K <= 64 *
    // kGatherRegs), beside the table probe below; dense modes gather logp[cid[i]], the sparse
    // mode reads its logits in id order
    const float* lp = sparse ? m.leaf_logit + (size_t)t * kLeafCap : logp + (size_t)t * dp.A;
    const int32_t* cid = sparse ? m.leaf_ids + (size_t)t * kLeafCap : (in_lds ? ids_lds : m.ch_id + off);
    auto logit = [&](int i) { return sparse ? lp[i] : lp[cid[i]]; };
    float x[kGatherRegs];
    int32_t xid[kGatherRegs];
#pragma unroll
    for (int j = 0; j < kGatherRegs; ++j) {
      const int i = l + j * kWave;
      const bool ok = !err && i < K;
      x[j] = ok ? logit(i) : -INFINITY;
      xid[j] = ok && in_lds ? cid[i] : 0;
    }
    int free_slot = -1;
    if (!err) {
      int64_t foff;
      int fK;
      if (table_find(m, t, key, foff, fK, &free_slot) || free_slot < 0) err |= kErrTable;
    }
    BK_STAMP(1, 3);
    if (!err) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < kGatherRegs; ++j) mx = fmaxf(mx, x[j]);
      for (int i = l + kGatherRegs * kWave; i < K; i += kWave) mx = fmaxf(mx, logit(i));
      float lse = 0.0f;
      if (prior_mode != 1) {
        mx = wave_max_f(mx);
        float sum = 0.0f;
#pragma unroll
        for (int j = 0; j < kGatherRegs; ++j) sum += l + j * kWave < K ? expf(x[j] - mx) : 0.0f;
        for (int i = l + kGatherRegs * kWave; i < K; i += kWave) sum += expf(logit(i) - mx);
        sum = wave_sum_f(sum);
        lse = logf(sum);
#pragma unroll
        for (int j = 0; j < kGatherRegs; ++j) x[j] = expf((x[j] - mx) - lse);
      }
      // coalesced child initialisation: child i = (id, N 0, Q 0, P)
#pragma unroll
      for (int j = 0; j < kGatherRegs; ++j) {
        const int i = l + j * kWave;
        if (i < K) {
          if (in_lds) m.ch_id[off + i] = xid[j];
          m.ch_N[off + i] = 0u;
          m.ch_Q[off + i] = 0.0;
          m.ch_P[off + i] = x[j];
        }
      }
      for (int i = l + kGatherRegs * kWave; i < K; i += kWave) {
        const float xi = logit(i);
        if (in_lds) m.ch_id[off + i] = cid[i];
        m.ch_N[off + i] = 0u;
        m.ch_Q[off + i] = 0.0;
        m.ch_P[off + i] = prior_mode != 1 ? expf((xi - mx) - lse) : xi;
      }
      if (l == 0) {
        TabEntry e;
        e.key = key;
        e.off = (uint32_t)used;
        e.K = K;
        m.tab[(size_t)t * m.TS + free_slot] = e;
        m.tree_nodes[t] = node + 1;
        m.tree_children[t] = used + K;
        ctr_add(m, t, kCtrExpanded, 1ull);
        ctr_add(m, t, kCtrLeafK, (unsigned long long)K);
      }
    } else if (l == 0) {
      atomicOr(&m.counters[kCtrErr], (unsigned long long)err);
    }
    if (l < dp.P) vsh[l] = (double)values[(size_t)t * dp.P + l];
  } else {
    if (l < dp.P) vsh[l] = m.leaf_scores[(size_t)t * kMaxP + l];
  }
  BK_STAMP(1, 4);
  BK_BOARD_SYNC();
  // (3) the backup (mcts.py:53-56): each path child of the descent, one lane per level
  if (on_path) {
    const double v = vsh[ppl];
    const uint32_t n = m.ch_N[pchild];
    const double q = m.ch_Q[pchild];
    m.ch_Q[pchild] = ((double)n * q + v) / (double)(n + 1u);
    m.ch_N[pchild] = n + 1u;
  }
  for (int d = l + kWave; d < depth; d += kWave) {  // levels 64..kMaxDepth-1 (never at 20x20)
    const size_t pd = (size_t)t * kMaxDepth + d;
    const int64_t ci = m.path_child[pd];
    const double v = vsh[m.path_pl[pd]];
    const uint32_t n = m.ch_N[ci];
    const double q = m.ch_Q[ci];
    m.ch_Q[ci] = ((double)n * q + v) / (double)(n + 1u);
    m.ch_N[ci] = n + 1u;
  }
  BK_STAMP(1, 5);
}

// ---- k_leaf_step_ov: the expansion split between wave 0 (bookkeeping + backup, then the next
// descent) and the last wave to finish the leaf logits (the new node's children). Together they do
// expand_tree's work in prior mode 2 with the same arithmetic in the same order, so the trees are
// bitwise those of the per-stage launches.
struct StepExpand {
  long long off;  // the new node's first child (global child index)
  int K, err;     // its child count; error flags (nonzero: no children are written)
  int ready;      // wave 0 published off / K / err
  int pready;     // the children (id, N, Q, P) are stored
  int done;       // logit waves finished
  int leaf_ready; // wave 0's descent is done (status_sh, the leaf state and its zeroed mask in LDS)
  int slice;      // next leaf-bitmask slice to claim
  int loaded;     // logit waves whose prologue loads are in LDS
  int counted;    // logit waves whose word counts are in wcnt
  int written;    // logit waves whose legal ids are in LDS
  int kready;     // the leaf's legal ids are compacted: K + 1 (1 + -1 = 0 is never published)
  int hready;     // wave 0 published hd (its backup is done)
  int wcnt[16];   // legal ids per logit wave's 64-word segment of the leaf bitmask
  int hd_status, hd_node;
  long long hd_used;
  unsigned long long hd_key;
};

// wave 0, first: expand_tree's backup (3) with the loads it needs, plus the expansion's own loads
// (node / child counters, leaf key) issued alongside — no dependence on the leaf's logits or K, so
// it runs while the other waves stage and compact the leaf's legal ids. Returns the leaf status.
struct StepHead {
  int status, node;
  int64_t used;
  uint64_t key;
};
// status: the tree's leaf status as the step found it (read once, before any wave of the step can
// run the next descent, which rewrites leaf_status)
__device__ __forceinline__ StepHead backup_first(const DevMcts& m, int t, int P, const float* __restrict__ values,
                                                 int status) {
  __shared__ double vsh[kMaxP];
  const int l = lane_id();
  StepHead h;
  h.status = status;
  const int depth = m.depth[t];
  h.node = m.tree_nodes[t];
  h.used = m.tree_children[t];
  h.key = table_key(m.leaf_state + (size_t)t * kStateWords);
  if (h.status == 0) return h;
  const size_t pi = (size_t)t * kMaxDepth + l;
  const bool on_path = l < depth;  // depth <= kMaxDepth = 96: levels 64.. are handled below
  const int64_t pchild = on_path ? m.path_child[pi] : 0;
  const int ppl = on_path ? m.path_pl[pi] : 0;
  if (h.status == 1) {
    if (l < P) vsh[l] = (double)values[(size_t)t * P + l];
  } else {
    if (l < P) vsh[l] = m.leaf_scores[(size_t)t * kMaxP + l];
  }
  wave_lds_sync();
  if (on_path) {
    const double v = vsh[ppl];
    const uint32_t n = m.ch_N[pchild];
    const double q = m.ch_Q[pchild];
    m.ch_Q[pchild] = ((double)n * q + v) / (double)(n + 1u);
    m.ch_N[pchild] = n + 1u;
  }
  for (int d = l + kWave; d < depth; d += kWave) {  // levels 64..kMaxDepth-1 (never at 20x20)
    const size_t pd = (size_t)t * kMaxDepth + d;
    const int64_t ci = m.path_child[pd];
    const double v = vsh[m.path_pl[pd]];
    const uint32_t n = m.ch_N[ci];
    const double q = m.ch_Q[ci];
    m.ch_Q[ci] = ((double)n * q + v) / (double)(n + 1u);
    m.ch_N[ci] = n + 1u;
  }
  return h;
}

// wave 0, then: the new node (expand_tree's checks, table slot and entry, counters) once K is
// known; publishes off / K / err (release) for the wave that writes the children
__device__ __forceinline__ void expand_head(const DevMcts& m, int t, const StepHead& h, int K, StepExpand* sx) {
  const int l = lane_id();
  int err = 0;
  if (h.status == 1) {
    const int64_t room = m.child_cap_per_tree - h.used;
    if (K > kLeafCap) err |= kErrLeafCap;
    if (h.node >= m.node_cap) err |= kErrTable;
    if (K > room) err |= kErrChildPool;
    int free_slot = -1;
    if (!err) {
      int64_t foff;
      int fK;
      if (table_find(m, t, h.key, foff, fK, &free_slot) || free_slot < 0) err |= kErrTable;
    }
    if (!err) {
      if (l == 0) {
        TabEntry e;
        e.key = h.key;
        e.off = (uint32_t)h.used;
        e.K = K;
        m.tab[(size_t)t * m.TS + free_slot] = e;
        m.tree_nodes[t] = h.node + 1;
        m.tree_children[t] = h.used + K;
        ctr_add(m, t, kCtrExpanded, 1ull);
        ctr_add(m, t, kCtrLeafK, (unsigned long long)K);
      }
    } else if (l == 0) {
      atomicOr(&m.counters[kCtrErr], (unsigned long long)err);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the table entry stored before the flag
  if (l == 0) {
    sx->off = (long long)((int64_t)t * m.child_cap_per_tree + h.used);
    sx->K = K;
    sx->err = h.status == 1 ? err : -1;
    __hip_atomic_store(&sx->ready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// leaf_logits_prologue by the waves 1..NW of the workgroup only (wave 0 is backing up meanwhile):
// their barriers are LDS counters; the compaction is parallel (each wave a 64-word segment of the
// bitmask, offsets from the segment counts: the ids in ascending order, as compact_ids writes
// them). Wave 1 publishes K (sx->kready) and leaf_K. Needs NW * 64 >= W32. status: the leaf status
// the step started from (not m.leaf_status, which wave 0's next descent rewrites meanwhile).
// pre (optional): this thread's word of the leaf bitmask and its feature, loaded before the
// step's first barrier (ok when one of each per thread covers them), so the prologue does not start
// with a round trip of its own after the status is known.
struct LeafPre {
  uint64_t w;
  float f;
  bool ok;
};
template <int NW>
__device__ __forceinline__ LeafPre leaf_pre_load(const DevPreset& dp, const DevMcts& m, int t,
                                                 const float* __restrict__ feat, int64_t ldf, int F) {
  const int tid = threadIdx.x - kWave, nth = NW * kWave;
  LeafPre p;
  p.ok = dp.W64 <= nth && F <= nth;
  p.w = p.ok && tid < dp.W64 ? m.leaf_mask[(size_t)t * dp.W64 + tid] : 0ull;
  p.f = p.ok && tid < F ? feat[(size_t)t * ldf + tid] : 0.0f;
  return p;
}
template <int NW>
__device__ __forceinline__ int leaf_logits_prologue_w(const DevPreset& dp, const DevMcts& m, int t,
                                                      const float* __restrict__ feat, int64_t ldf, int F,
                                                      uint32_t* lds, int wave, StepExpand* sx, int status,
                                                      const LeafPre* pre = nullptr) {
  uint32_t* m32 = lds;
  int32_t* ids = reinterpret_cast<int32_t*>(lds + dp.W32pad);
  float* f = reinterpret_cast<float*>(lds + dp.W32pad + kLeafCap);
  if (status != 1) return -1;  // uniform over these waves: no leaf to evaluate
  const int tid = threadIdx.x - kWave, nth = NW * kWave, l = lane_id();
  if (pre && pre->ok) {
    if (tid < dp.W64) {
      m32[2 * tid] = (uint32_t)pre->w;
      m32[2 * tid + 1] = (uint32_t)(pre->w >> 32);
    }
    if (tid < F) f[tid] = pre->f;
  } else {
    const uint64_t* lm = m.leaf_mask + (size_t)t * dp.W64;
    for (int j = tid; j < dp.W64; j += nth) {
      const uint64_t w = lm[j];
      m32[2 * j] = (uint32_t)w;
      m32[2 * j + 1] = (uint32_t)(w >> 32);
    }
    const float* ft = feat + (size_t)t * ldf;
    for (int i = tid; i < F; i += nth) f[i] = ft[i];
  }
  auto arrive_wait = [&](int* ctr) {  // a barrier of the NW logit waves (LDS counter)
    if (l == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < NW) __builtin_amdgcn_s_sleep(1);
  };
  arrive_wait(&sx->loaded);
  // this wave's segment: words 64 (wave - 1) .. + 63
  const int w = 64 * (wave - 1) + l;
  uint32_t bits = w < dp.W32 ? m32[w] : 0u;
  const int cnt = __popc(bits);
  const int incl = wave_incl_scan(cnt);
  if (l == kWave - 1) sx->wcnt[wave] = incl;
  arrive_wait(&sx->counted);
  int before = 0, K = 0;
  for (int v = 1; v <= NW; ++v) {
    const int c = sx->wcnt[v];
    before += v < wave ? c : 0;
    K += c;
  }
  int pos = before + incl - cnt;
  while (bits) {
    const int b = __ffs(bits) - 1;
    bits &= bits - 1u;
    if (pos < kLeafCap) ids[pos] = w * 32 + b;
    ++pos;
  }
  arrive_wait(&sx->written);
  if (wave == 1 && l == 0) {
    m.leaf_K[t] = K;
    if (K > kLeafCap) atomicOr(&m.counters[kCtrErr], (unsigned long long)kErrLeafCap);
    __hip_atomic_store(&sx->kready, K + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  return K;
}

// The leaf bitmask of the state in LDS (s; m32 zeroed by the caller) built by whichever waves
// call this: each claims slices k = 0..kMaskWpb-1 (the orientations O % kMaskWpb == k, the
// slices of build_mask_rows_wg) from an LDS counter until none is left, ORing into m32. The
// caller's barrier ends the build.
#ifdef BK_STAMPS
// diag: per (tree, wave) of the leaf bitmask claims: entry, slices claimed, exit, longest slice, the
// last slice run again with its code just executed (ORs the same bits), the first claim
static __device__ unsigned long long g_mask_stamps[256][16][6];
#endif
__device__ __forceinline__ void mask_slices_claim(const DevPreset& dp, const uint32_t* s, uint32_t* m32, int* counter) {
#ifdef BK_STAMPS
  const unsigned long long t_in = __builtin_amdgcn_s_memtime();
  unsigned long long n_cl = 0, t_max = 0, t_first_claim = 0;
  int last_k = -1;
#endif
  RowCtx c = row_ctx(dp, s, (int)s[kWToMove], m32);
  for (;;) {
#ifdef BK_STAMPS
    const unsigned long long t_s = __builtin_amdgcn_s_memtime();
    if (t_first_claim == 0) t_first_claim = t_s;
#endif
    // the context opaque per claim: nothing derived from it is hoisted out of the loop (the
    // compiler would otherwise keep every slice's shifted rows live at once)
#pragma unroll
    for (int d = 0; d < 5; ++d) asm volatile("" : "+v"(c.fr[d]), "+v"(c.ar[d]));
    asm volatile("" : "+v"(c.r), "+v"(c.rN1), "+v"(c.pieces));
    int k = 0;
    if (lane_id() == 0) k = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    k = readlane_i(k, 0);
    if (k >= kMaskWpb) break;
    DevPreset dq = dp;  // the scalar sizes opaque per claim as well
    asm volatile("" : "+s"(dq.N), "+s"(dq.num_pieces));
    orient_dispatch<kMaskWpb>(dq, c, k, std::make_index_sequence<kMaskWpb>{});
#ifdef BK_STAMPS
    ++n_cl;
    last_k = k;
    const unsigned long long d = __builtin_amdgcn_s_memtime() - t_s;
    t_max = d > t_max ? d : t_max;
#endif
  }
#ifdef BK_STAMPS
  const unsigned long long t_out = __builtin_amdgcn_s_memtime();
  unsigned long long t_warm = 0;
  if (last_k >= 0) {
    DevPreset dq = dp;
    asm volatile("" : "+s"(dq.N), "+s"(dq.num_pieces));
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    orient_dispatch<kMaskWpb>(dq, c, last_k, std::make_index_sequence<kMaskWpb>{});
    t_warm = __builtin_amdgcn_s_memtime() - t0;
  }
  const int w = (int)(threadIdx.x >> 6);
  if (lane_id() == 0 && blockIdx.x < 256 && w < 16) {
    g_mask_stamps[blockIdx.x][w][0] = t_in;
    g_mask_stamps[blockIdx.x][w][1] = n_cl;
    g_mask_stamps[blockIdx.x][w][2] = t_out;
    g_mask_stamps[blockIdx.x][w][3] = t_max;
    g_mask_stamps[blockIdx.x][w][4] = t_warm;
    g_mask_stamps[blockIdx.x][w][5] = t_first_claim;
  }
#endif
}

// The new node's children from the logits in LDS (ids[i], lg[i], i < K), by one wave:
// expand_tree's softmax (prior mode 2) and child initialisation, term for term.
__device__ __forceinline__ void expand_children_lds(const DevMcts& m, int64_t off, int K, const int32_t* ids,
                                                    const float* lg) {
  const int l = lane_id();
  float x[kGatherRegs];
  int32_t xid[kGatherRegs];
#pragma unroll
  for (int j = 0; j < kGatherRegs; ++j) {
    const int i = l + j * kWave;
    const bool ok = i < K;
    x[j] = ok ? lg[i] : -INFINITY;
    xid[j] = ok ? ids[i] : 0;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < kGatherRegs; ++j) mx = fmaxf(mx, x[j]);
  for (int i = l + kGatherRegs * kWave; i < K; i += kWave) mx = fmaxf(mx, lg[i]);
  mx = wave_max_f(mx);
  float sum = 0.0f;
#pragma unroll
  for (int j = 0; j < kGatherRegs; ++j) sum += l + j * kWave < K ? expf(x[j] - mx) : 0.0f;
  for (int i = l + kGatherRegs * kWave; i < K; i += kWave) sum += expf(lg[i] - mx);
  sum = wave_sum_f(sum);
  const float lse = logf(sum);
#pragma unroll
  for (int j = 0; j < kGatherRegs; ++j) x[j] = expf((x[j] - mx) - lse);
#pragma unroll
  for (int j = 0; j < kGatherRegs; ++j) {
    const int i = l + j * kWave;
    if (i < K) {
      m.ch_id[off + i] = xid[j];
      m.ch_N[off + i] = 0u;
      m.ch_Q[off + i] = 0.0;
      m.ch_P[off + i] = x[j];
    }
  }
  for (int i = l + kGatherRegs * kWave; i < K; i += kWave) {
    m.ch_id[off + i] = ids[i];
    m.ch_N[off + i] = 0u;
    m.ch_Q[off + i] = 0.0;
    m.ch_P[off + i] = expf((lg[i] - mx) - lse);
  }
}

}  // namespace bk

// the search handle behind the C-ABI's bk_mcts*
struct bk_mcts {
  bk_ctx* ctx = nullptr;
  bk::DevMcts d{};
  std::vector<void*> allocs;
};
