// mcts.hip — batched AlphaZero MCTS on gfx950 (the search half of the C-ABI).
//
// T independent trees, one per game, one simulation in flight per tree. A simulation of the
// reference (`MCTS.simulate`, blokus_rl/alphazero/mcts.py:13-71) is split into
//   k_select        descent from the root (mcts.py:37-50) to a board not yet in the tree or a
//                   terminal board, recording the path; writes the leaf's observation row and
//                   legal bitmask (mcts.py:60-66) so the caller can batch every tree's leaf into
//                   one policy/value forward pass;
//   (the net)       PyTorch-ROCm forward on the [T, 2P, N, N] leaf batch;
//   k_expand_backup expansion with P = exp(log_softmax(logp[legal ids]))
//                   (neural_network.py:159-173, mcts.py:67-70) and the backup
//                   Q <- (N*Q + v)/(N+1), N += 1 with v = scores[player to move at the child]
//                   (mcts.py:53-56).
// Each tree is touched by exactly one wave per kernel, so its table, node and child regions
// need no atomics. All search arithmetic is float64 (the reference's pinned numpy 1.25 promotes
// every float32 meeting a Python number to float64), compiled with -ffp-contract=off.
// The per-tree stages run on one wave (the descent, the expansion) while the other waves of a
// k_select workgroup wait at a workgroup barrier, so board-level handoffs are wave-scope.
#define BK_BOARD_SYNC() ::bk::wave_lds_sync()
#ifdef BK_STAMPS
#include <hip/hip_runtime.h>
static __device__ unsigned long long g_step_stamps[4096][16];  // diag: k_leaf_step phase stamps
// diag: phases inside the leaf bitmask build of k_leaf_step (slots 5..7), thread 0 of the group
#define BK_MASK_STAMP(i) \
  do { if (threadIdx.x == 0 && blockIdx.x < 4096 && blockDim.x > 256) g_step_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime(); } while (0)
#endif
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/blokus_engine.h"
#include "ctx.h"
#include "legal_rows.h"
#include "mcts_dev.h"

namespace bk {

// grid (kResetBlocks, T) x 256: a flagged tree's table cleared by kResetBlocks workgroups (an
// unflagged tree costs kResetBlocks empty workgroups, not TS / 64: 28 -> ~3 us per ply)
constexpr int kResetBlocks = 8;
__global__ __launch_bounds__(256) void k_reset(DevMcts m, const int32_t* flags) {
  const int t = blockIdx.y;
  if (flags && !flags[t]) return;
  TabEntry* tab = m.tab + (size_t)t * m.TS;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < m.TS; i += kResetBlocks * 256) tab[i] = TabEntry{0ull, 0u, 0};
  if (blockIdx.x == 0 && threadIdx.x == 0) { m.tree_nodes[t] = 0; m.tree_children[t] = 0; }
}

// grid T x 256 threads: wave 0 descends, then the 4 waves build the leaf's legal bitmask (the
// orientations split over the waves) and write its observation rows
constexpr int kSelectWaves = 4;
__global__ __launch_bounds__(64 * kSelectWaves) void k_select(DevPreset dp, DevMcts m, const uint32_t* __restrict__ roots,
                                                              const int32_t* __restrict__ active, double cpuct,
                                                              int32_t* __restrict__ status_out, float* __restrict__ obs,
                                                              uint64_t* __restrict__ mask_out, double root_eps) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ int status_sh;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave == 0) {
    const int st = select_descend(dp, m, blockIdx.x, roots, active, cpuct, status_out, lds, 0, nullptr, root_eps);
    if (lane_id() == 0) status_sh = st;
  }
  __syncthreads();
  select_leaf<kSelectWaves>(dp, m, blockIdx.x, status_sh, obs, mask_out, lds, wave);
}

// grid (T, kLeafBlocks) x 256 threads: workgroup c takes share c of the tree's legal ids
constexpr int kLeafR = 1;  // R x 4 ids per wave at a time (R = 2: 0.93M vs 1.13M sims/s)
__global__ __launch_bounds__(256) void k_leaf_logits(DevPreset dp, DevMcts m, const float* __restrict__ feat,
                                                     int64_t ldf, int F, const float* __restrict__ W,
                                                     const float* __restrict__ bias) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  leaf_logits_tree<kLeafR>(dp, m, blockIdx.x, blockIdx.y, kLeafBlocks, feat, ldf, F, W, bias, lds);
}

// grid T x 64 threads
__global__ __launch_bounds__(64) void k_expand_backup(DevPreset dp, DevMcts m, const float* __restrict__ logp,
                                                      const float* __restrict__ values, int prior_mode) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  expand_tree(dp, m, blockIdx.x, logp, values, prior_mode, lds);
}

// The search half of a simulation plus the next one's descent, per tree, one workgroup of
// kStepWaves waves: the policy Linear over the leaf's legal ids (all waves: the gather's memory
// parallelism of k_leaf_logits' 4 x 4 waves), expand/backup (wave 0, prior mode 2), then — when
// do_select — the next simulation's descent (wave 0) and leaf bitmask / observation (all waves). The same device functions as
// k_leaf_logits -> k_expand_backup -> k_select, so the trees are bitwise those of the three
// launches; what goes is two kernel boundaries per simulation and the grid-wide wait for the
// slowest tree of each stage. Handoffs: this workgroup's global stores visible to its later loads
// (vmcnt(0), barrier, L1 invalidate).
__device__ __forceinline__ void wg_store_handoff() {
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  asm volatile("buffer_inv sc0" ::: "memory");
}
constexpr int kStepWaves = 16;  // waves per tree in k_leaf_step: the logit gather's memory parallelism
__global__ __launch_bounds__(64 * kStepWaves) void k_leaf_step(DevPreset dp, DevMcts m, const float* __restrict__ feat,
                                                                 int64_t ldf, int F, const float* __restrict__ W,
                                                                 const float* __restrict__ bias,
                                                                 const float* __restrict__ values, int do_select,
                                                                 const uint32_t* __restrict__ roots,
                                                                 const int32_t* __restrict__ active, double cpuct,
                                                                 int32_t* __restrict__ status_out,
                                                                 float* __restrict__ obs,
                                                                 uint64_t* __restrict__ mask_out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ int status_sh;
  const int t = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef BK_STAMPS
#define BK_STEP_STAMP(i) \
  do { if (do_select && threadIdx.x == 0 && t < 4096) g_step_stamps[t][i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define BK_STEP_STAMP(i) do { } while (0)
#endif
  BK_STEP_STAMP(0);
  leaf_logits_tree<kLeafR>(dp, m, t, 0, 1, feat, ldf, F, W, bias, lds);
  wg_store_handoff();
  BK_STEP_STAMP(1);
  if (wave == 0) expand_tree(dp, m, t, nullptr, values, 2, lds);
  wg_store_handoff();
  BK_STEP_STAMP(2);
  if (!do_select) return;
  if (wave == 0) {
    const int st = select_descend(dp, m, t, roots, active, cpuct, status_out, lds);
    if (lane_id() == 0) status_sh = st;
  }
  __syncthreads();
  BK_STEP_STAMP(3);
  select_leaf<kStepWaves>(dp, m, t, status_sh, obs, mask_out, lds, wave);
  BK_STEP_STAMP(4);
#undef BK_STEP_STAMP
}

// k_leaf_step with the expansion overlapped (the default; BK_STEP_OVERLAP=0 keeps k_leaf_step).
// After the logit prologue (all waves: the leaf bitmask compacted, the features in LDS), wave 0
// publishes the new node (table entry, child range), backs the value up and — when do_select —
// descends for the next simulation at once, while waves 1.. compute the logits into LDS; the last
// of them to finish writes the new node's children (softmax + init) and releases a flag. The
// descent waits on that flag only if it reaches the new node before its children are stored
// (its children's P are the only data it can need from the other waves). Then all waves build the
// next leaf's bitmask and observation. The logits, priors, backup and descent are expand_tree's
// and select_descend's in the same order, so the trees are bitwise those of the per-stage
// launches; what goes is the wait of the expansion and descent for the slowest logit wave.
// lds = [W32pad mask | kLeafCap ids | F features | kLeafCap logits] then, at sel_off, the
// descent's [state | 2 kMaxN | W32pad].
__global__ __launch_bounds__(64 * kStepWaves) void k_leaf_step_ov(DevPreset dp, DevMcts m, const float* __restrict__ feat,
                                                                    int64_t ldf, int F, const float* __restrict__ W,
                                                                    const float* __restrict__ bias,
                                                                    const float* __restrict__ values, int do_select,
                                                                    const uint32_t* __restrict__ roots,
                                                                    const int32_t* __restrict__ active, double cpuct,
                                                                    int32_t* __restrict__ status_out,
                                                                    float* __restrict__ obs,
                                                                    uint64_t* __restrict__ mask_out, int sel_off,
                                                                    int skipz) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ int status_sh, status0_sh;
  __shared__ StepExpand sx;
  const int t = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef BK_STAMPS
  // diag: 0 start, 1 the new node's entry published (wave 1), 2 wave 0 backup done, 3 wave 0 descent done, 4 the last logit
  // wave done, 9 its children's stores issued, 5 its children stored, 6 the next leaf's bitmask done (all waves), 7 end, 8 wave 0 out of the
  // bitmask claims (select_leaf's own stamps: g_stamps[0][t][4] stores issued, [5] observation issued)
#define BK_OV_STAMP(i) \
  do { if (lane_id() == 0 && do_select && t < 4096) g_step_stamps[t][i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define BK_OV_STAMP(i) do { } while (0)
#endif
  if (threadIdx.x == 0) {
    sx.ready = 0;
    sx.pready = 0;
    sx.done = 0;
    sx.leaf_ready = 0;
    sx.slice = 0;
    sx.loaded = 0;
    sx.counted = 0;
    sx.written = 0;
    sx.kready = 0;
    sx.hready = 0;
    status_sh = 0;
    // the leaf status this step expands, read once before the barrier: wave 0's next descent
    // rewrites m.leaf_status[t] while the logit waves may still be deciding whether to run
    status0_sh = m.leaf_status[t];
  }
  if (wave == 0) BK_OV_STAMP(0);
  // the logit waves' bitmask words and features in flight across the barrier (read whatever the
  // status; used only when it is 1)
  LeafPre pre{0ull, 0.0f, false};
  if (wave > 0) pre = leaf_pre_load<kStepWaves - 1>(dp, m, t, feat, ldf, F);
  __syncthreads();
  const int status0 = status0_sh;
  // waves 1..: the logit prologue (legal ids compacted, features in LDS); wave 0 meanwhile backs
  // the value up (independent of the logits) and then waits for K to publish the new node
  int K = -1;
  if (wave > 0) {
    K = leaf_logits_prologue_w<kStepWaves - 1>(dp, m, t, feat, ldf, F, lds, wave, &sx, status0, &pre);
    if (wave == 1 && K >= 0) {
      // the new node (table entry, child range) from wave 0's loads, as soon as K is known
      wait_flag_acquire(&sx.hready);
      StepHead h;
      h.status = sx.hd_status;
      h.node = sx.hd_node;
      h.used = sx.hd_used;
      h.key = sx.hd_key;
      expand_head(m, t, h, K, &sx);
      BK_OV_STAMP(1);
    }
  }
  const int32_t* ids = reinterpret_cast<const int32_t*>(lds + dp.W32pad);
  float* lg = reinterpret_cast<float*>(lds + dp.W32pad + kLeafCap + F);
  uint32_t* lsel = lds + sel_off;
  uint32_t* m32 = lsel + kStateWords + 2 * kMaxN;
  if (wave == 0) {
    const StepHead h = backup_first(m, t, dp.P, values, status0);
    if (h.status == 1) {
      // wave 1 adds the new node once the leaf's ids are compacted
      if (lane_id() == 0) {
        sx.hd_status = h.status;
        sx.hd_node = h.node;
        sx.hd_used = h.used;
        sx.hd_key = h.key;
        __hip_atomic_store(&sx.hready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else if (lane_id() == 0) {
      sx.err = -1;  // no new node: the children writer and the descent need not wait
      __hip_atomic_store(&sx.ready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    BK_OV_STAMP(2);
    if (do_select) {
      // this wave's backup stores, visible to its own descent loads; the descent starts now and
      // waits for the new node only if it reaches that board (pend: entry, children, failure)
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      asm volatile("buffer_inv sc0" ::: "memory");
      int* pend[3];
      pend[0] = &sx.ready;
      pend[1] = &sx.pready;
      pend[2] = &sx.err;
      const int st = select_descend(dp, m, t, roots, active, cpuct, status_out, lsel, h.key,
                                    h.status == 1 ? pend : nullptr);
      if (st == 1)
        for (int i = lane_id(); i < dp.W32pad / 4; i += kWave) reinterpret_cast<uint4*>(m32)[i] = make_uint4(0u, 0u, 0u, 0u);
      if (lane_id() == 0) {
        status_sh = st;
        __hip_atomic_store(&sx.leaf_ready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      BK_OV_STAMP(3);
      // the next leaf's observation rows and state now, while the logit waves are busy (they were
      // the step's tail, after the bitmask)
      leaf_obs_rows<1>(dp, m, t, st, obs, lsel, lane_id());
    }
  }
  if (wave > 0 && K >= 0 && K <= kLeafCap) {
    leaf_logits_dots<kLeafR>(dp, 0, K, wave - 1, kStepWaves - 1, W, bias, F, lds, nullptr, lg, skipz);
    int done = 0;
    if (lane_id() == 0) done = __hip_atomic_fetch_add(&sx.done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    done = readlane_i(done, 0);
    if (done == kStepWaves - 2) {  // the last logit wave: every logit is in LDS
      BK_OV_STAMP(4);
      while (__hip_atomic_load(&sx.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
        __builtin_amdgcn_s_sleep(1);
      const int err = readlane_i(sx.err, 0);
      if (err == 0) expand_children_lds(m, (int64_t)sx.off, K, ids, lg);
      BK_OV_STAMP(9);  // the children's stores issued
      // the flag orders the children before the descent's reads of them; once the descent is over
      // nobody reads them in this launch, so the stores drain under the bitmask instead of being
      // waited for here (the kernel's end orders them for the next launch)
      const bool descended = readlane_i(__hip_atomic_load(&sx.leaf_ready, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP), 0) != 0;
      if (!descended) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the children stored before the flag
        if (lane_id() == 0) __hip_atomic_store(&sx.pready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (lane_id() == 0) {
        __hip_atomic_store(&sx.pready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      BK_OV_STAMP(5);
    }
  }
  if (do_select) {
    // every wave joins the next leaf's bitmask once it is free and the descent is done: wave 0
    // usually starts it alone while the logit waves finish
    while (__hip_atomic_load(&sx.leaf_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
      __builtin_amdgcn_s_sleep(1);
    if (readlane_i(status_sh, 0) == 1) mask_slices_claim(dp, lsel, m32, &sx.slice);
    if (wave == 0) BK_OV_STAMP(8);  // wave 0 has no slice left to claim
  }
  __syncthreads();
  if (wave == 0) BK_OV_STAMP(6);
  if (!do_select) return;
  select_leaf<kStepWaves, true, false>(dp, m, t, status_sh, obs, mask_out, lsel, wave);
  if (wave == 0) BK_OV_STAMP(7);
#undef BK_OV_STAMP
}

__device__ __forceinline__ double raise_visits(uint32_t n, double e) {
  if (e == 1.0 || n <= 1u) return (double)n;
  return pow((double)n, e);
}

// get_distribution (mcts.py:73-99) / root statistics. mode 0 -> pi, mode 1 -> raw stats.
__global__ __launch_bounds__(64) void k_root(DevMcts m, const uint32_t* __restrict__ roots,
                                             const int32_t* __restrict__ active, double temperature, int mode,
                                             int32_t* ids, double* pi, uint32_t* n_out, double* q_out, float* p_out,
                                             int cap, int32_t* counts) {
  const int t = blockIdx.x;
  const int l = lane_id();
  if (active && !active[t]) {
    if (l == 0) counts[t] = 0;
    return;
  }
  const uint32_t* s = roots + (size_t)t * kStateWords;
  const uint64_t key = table_key(s);
  int64_t off;
  int K;
  if (!table_find(m, t, key, off, K, nullptr)) {
    if (l == 0) { counts[t] = -1; atomicOr(&m.counters[kCtrErr], (unsigned long long)kErrMissingRoot); }
    return;
  }
  if (l == 0) counts[t] = K <= cap ? K : -K;
  const int Kc = K <= cap ? K : cap;
  if (mode == 1) {
    for (int i = l; i < Kc; i += kWave) {
      ids[(size_t)t * cap + i] = m.ch_id[off + i];
      n_out[(size_t)t * cap + i] = m.ch_N[off + i];
      q_out[(size_t)t * cap + i] = m.ch_Q[off + i];
      p_out[(size_t)t * cap + i] = m.ch_P[off + i];
    }
    return;
  }
  for (int i = l; i < Kc; i += kWave) ids[(size_t)t * cap + i] = m.ch_id[off + i];
  double* o = pi + (size_t)t * cap;
  if (temperature == 0.0) {
    // 1/0 raises ZeroDivisionError in the reference -> one-hot at the first max of N
    double best = -1.0;
    int bi = 0x7fffffff;
    for (int i = l; i < K; i += kWave) {
      const double v = (double)m.ch_N[off + i];
      if (v > best) { best = v; bi = i; }
    }
    wave_argmax(best, bi);
    for (int i = l; i < Kc; i += kWave) o[i] = i == bi ? 1.0 : 0.0;
    return;
  }
  // N^(1/T), summed left to right like Python's object-array sum, then normalised.
  // N^1 is exact in the reference (int ** 1.0); device pow() is not correctly rounded, so the
  // default temperature 1 bypasses it. Other temperatures agree to ~1 ulp with host libm.
  // The terms are computed by all lanes into LDS, lane 0 adds them in index order from there (a
  // chain of adds fed by pipelined LDS reads, not a global-memory round trip per term: the
  // sequential loop over the output row took 65-155 us per launch mid-game at K ~ 300-700), and
  // the divisions run on all lanes again: the same terms, order and quotients.
  constexpr int kRootLds = 2048;
  __shared__ double vals[kRootLds];
  __shared__ double total_sh;
  const double e = 1.0 / temperature;
  for (int i = l; i < K && i < kRootLds; i += kWave) vals[i] = raise_visits(m.ch_N[off + i], e);
  __syncthreads();
  if (l == 0) {
    double total = 0.0;
#pragma unroll 8
    for (int i = 0; i < K; ++i) total += i < kRootLds ? vals[i] : raise_visits(m.ch_N[off + i], e);
    total_sh = total;
  }
  __syncthreads();
  const double total = total_sh;
  for (int i = l; i < Kc; i += kWave) {
    const double v = i < kRootLds ? vals[i] : raise_visits(m.ch_N[off + i], e);
    o[i] = total == 0.0 ? 1.0 / (double)K : v / total;
  }
}

}  // namespace bk

using namespace bk;

template <typename T>
static int mcts_alloc(bk_mcts* m, T** p, size_t count) {
  void* q = nullptr;
  int rc = hip_check(hipMalloc(&q, sizeof(T) * (count ? count : 1)), "hipMalloc mcts");
  if (rc) return rc;
  m->allocs.push_back(q);
  *p = (T*)q;
  return BK_OK;
}

extern "C" {

#ifdef BK_STAMPS
int bk_debug_stamps(unsigned long long* out) {  // [2][4096][8] host copy
  return hip_check(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)), "stamps");
}
int bk_debug_mask_stamps(unsigned long long* out) {  // [256][16][6] host copy: leaf bitmask claims
  return hip_check(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mask_stamps), sizeof(g_mask_stamps)), "mask stamps");
}
int bk_debug_step_stamps(unsigned long long* out) {  // [4096][16] host copy: k_leaf_step phases
  return hip_check(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_step_stamps), sizeof(g_step_stamps)), "step stamps");
}
#endif

int bk_mcts_create(bk_ctx* ctx, int trees, int node_cap, int64_t child_cap, bk_mcts** out) {
  BK_REQUIRE(ctx && out && trees > 0 && node_cap > 0 && child_cap >= trees, "bad argument");
  BK_REQUIRE(child_cap / trees <= (int64_t)0xffffffff, "bk_mcts_create: child_cap / trees must fit 32 bits");
  BK_REQUIRE(ctx->d_items, "host-only context (created with device < 0)");
  *out = nullptr;
  bk_mcts* m = new bk_mcts();
  m->ctx = ctx;
  DevMcts& d = m->d;
  d.T = trees;
  d.node_cap = node_cap;
  int TS = 64;
  while (TS < 2 * node_cap) TS <<= 1;
  d.TS = TS;
  d.child_cap_per_tree = child_cap / trees;
  const size_t T = (size_t)trees;
  const int W64 = ctx->dp.W64;
  int rc = hip_check(hipSetDevice(ctx->device), "hipSetDevice");
  if (!rc) {
    // the whole allocation checked against the device's free memory first: an oversized tree set
    // (node_cap grows with the simulations per move) fails here with its size, not inside hipMalloc
    const size_t C0 = (size_t)d.child_cap_per_tree * T;
    const size_t need = T * TS * sizeof(TabEntry) + C0 * (4 + 4 + 8 + 4) +
                        T * (kMaxDepth * 12 + kStateWords * 4 + kMaxP * 8 + W64 * 8 + kLeafCap * 8 + 64 + 64);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && need > free_b) {
      delete m;
      char msg[256];
      snprintf(msg, sizeof msg,
               "bk_mcts_create: %d trees x node_cap %d (child_cap %lld) need %.2f GB of device memory, %.2f GB free",
               trees, node_cap, (long long)child_cap, need / 1e9, free_b / 1e9);
      bk::set_error(msg);
      return BK_ENOMEM;
    }
  }
  if (!rc) rc = mcts_alloc(m, &d.tab, T * TS);
  if (!rc) rc = mcts_alloc(m, &d.tree_nodes, T);
  if (!rc) rc = mcts_alloc(m, &d.tree_children, T);
  const size_t C = (size_t)d.child_cap_per_tree * T;
  if (!rc) rc = mcts_alloc(m, &d.ch_id, C);
  if (!rc) rc = mcts_alloc(m, &d.ch_N, C);
  if (!rc) rc = mcts_alloc(m, &d.ch_Q, C);
  if (!rc) rc = mcts_alloc(m, &d.ch_P, C);
  if (!rc) rc = mcts_alloc(m, &d.path_child, T * kMaxDepth);
  if (!rc) rc = mcts_alloc(m, &d.path_pl, T * kMaxDepth);
  if (!rc) rc = mcts_alloc(m, &d.depth, T);
  if (!rc) rc = mcts_alloc(m, &d.leaf_state, T * kStateWords);
  if (!rc) rc = mcts_alloc(m, &d.leaf_status, T);
  if (!rc) rc = mcts_alloc(m, &d.leaf_scores, T * kMaxP);
  if (!rc) rc = mcts_alloc(m, &d.leaf_mask, T * W64);
  if (!rc) rc = mcts_alloc(m, &d.leaf_ids, T * kLeafCap);
  if (!rc) rc = mcts_alloc(m, &d.leaf_logit, T * kLeafCap);
  if (!rc) rc = mcts_alloc(m, &d.leaf_K, T);
  if (!rc) rc = mcts_alloc(m, &d.counters, 8);
  if (!rc) rc = hip_check(hipMemset(d.counters, 0, 8 * sizeof(unsigned long long)), "memset counters");
  if (!rc) rc = mcts_alloc(m, &d.tree_ctr, T * 8);
  if (!rc) rc = hip_check(hipMemset(d.tree_ctr, 0, T * 8 * sizeof(unsigned long long)), "memset tree counters");
  if (!rc) rc = hip_check(hipMemset(d.leaf_status, 0, T * sizeof(int32_t)), "memset status");
  if (!rc) rc = hip_check(hipMemset(d.depth, 0, T * sizeof(int32_t)), "memset depth");
  if (rc) { bk_mcts_destroy(m); return rc; }
  rc = bk_mcts_reset(m, nullptr, nullptr);
  if (!rc) rc = hip_check(hipDeviceSynchronize(), "sync");
  if (rc) { bk_mcts_destroy(m); return rc; }
  *out = m;
  return BK_OK;
}

int bk_mcts_destroy(bk_mcts* m) {
  if (!m) return BK_OK;
  for (void* p : m->allocs) (void)hipFree(p);
  delete m;
  return BK_OK;
}

int bk_mcts_reset(bk_mcts* m, const int32_t* reset_flags, void* stream) {
  BK_REQUIRE(m, "null mcts");
  hipLaunchKernelGGL(k_reset, dim3(kResetBlocks, m->d.T), dim3(256), 0, (hipStream_t)stream, m->d,
                     reset_flags);
  return launch_check("k_reset");
}

int bk_mcts_select_eps(bk_mcts* m, const void* roots, const int32_t* active, double cpuct, double root_eps,
                       int32_t* leaf_status, float* obs, uint64_t* leaf_mask, void* stream) {
  BK_REQUIRE(m && roots && leaf_status && obs, "bad argument");
  BK_REQUIRE(root_eps >= 0.0, "bk_mcts_select_eps: root_eps >= 0");
  const DevPreset& dp = m->ctx->dp;
  const size_t lds = sizeof(uint32_t) * (size_t)(kStateWords + 2 * kMaxN + dp.W32pad);
  hipLaunchKernelGGL(k_select, dim3(m->d.T), dim3(kWave * kSelectWaves), lds, (hipStream_t)stream, dp, m->d,
                     (const uint32_t*)roots, active, cpuct, leaf_status, obs, leaf_mask, root_eps);
  return launch_check("k_select");
}

int bk_mcts_select(bk_mcts* m, const void* roots, const int32_t* active, double cpuct, int32_t* leaf_status,
                   float* obs, uint64_t* leaf_mask, void* stream) {
  return bk_mcts_select_eps(m, roots, active, cpuct, 1e-6, leaf_status, obs, leaf_mask, stream);
}

int bk_mcts_leaf_logits(bk_mcts* m, const float* feat, int64_t ldf, int F, const float* W, const float* bias,
                        void* stream) {
  BK_REQUIRE(m && feat && W && bias && F > 0 && F <= kMaxFeat && ldf >= F, "bad argument");
  BK_REQUIRE(((uintptr_t)W & 15u) == 0 || (F & 3) != 0, "bk_mcts_leaf_logits: W must be 16-byte aligned");
  const DevPreset& dp = m->ctx->dp;
  const size_t lds = sizeof(uint32_t) * ((size_t)dp.W32pad + kLeafCap + F);
  hipLaunchKernelGGL(k_leaf_logits, dim3(m->d.T, kLeafBlocks), dim3(256), lds, (hipStream_t)stream, dp, m->d, feat,
                     ldf, F, W, bias);
  return launch_check("k_leaf_logits");
}

int bk_mcts_leaf_step(bk_mcts* m, const float* feat, int64_t ldf, int F, const float* W, const float* bias,
                      const float* values, int do_select, const void* roots, const int32_t* active, double cpuct,
                      int32_t* leaf_status, float* obs, uint64_t* leaf_mask, void* stream) {
  BK_REQUIRE(m && feat && W && bias && values && F > 0 && F <= kMaxFeat && ldf >= F, "bad argument");
  BK_REQUIRE(((uintptr_t)W & 15u) == 0 || (F & 3) != 0, "bk_mcts_leaf_step: W must be 16-byte aligned");
  BK_REQUIRE(!do_select || (roots && leaf_status && obs), "bad argument: select outputs");
  const DevPreset& dp = m->ctx->dp;
  const char* ov = getenv("BK_STEP_OVERLAP");  // read per call (graph capture reads it once)
  const int overlap = ov ? atoi(ov) : 1;
  if (overlap) {
    const int sel_off = (int)(((size_t)dp.W32pad + 2 * kLeafCap + F + 3) & ~(size_t)3);
    const size_t words = (size_t)sel_off + kStateWords + 2 * kMaxN + dp.W32pad;
    const char* sz = getenv("BK_LEAF_SKIP0");  // W float4s of all-zero features not loaded (0: load all)
    const int skipz = sz ? atoi(sz) : 1;
    hipLaunchKernelGGL(k_leaf_step_ov, dim3(m->d.T), dim3(kWave * kStepWaves), sizeof(uint32_t) * words,
                       (hipStream_t)stream, dp, m->d, feat, ldf, F, W, bias, values, do_select,
                       (const uint32_t*)roots, active, cpuct, leaf_status, obs, leaf_mask, sel_off, skipz);
    return launch_check("k_leaf_step_ov");
  }
  size_t words = (size_t)dp.W32pad + kLeafCap + F;                               // leaf logits
  words = std::max(words, (size_t)dp.W32pad + kExpandLdsIds);                    // expand
  words = std::max(words, (size_t)(kStateWords + 2 * kMaxN + dp.W32pad));       // select
  hipLaunchKernelGGL(k_leaf_step, dim3(m->d.T), dim3(kWave * kStepWaves), sizeof(uint32_t) * words,
                     (hipStream_t)stream, dp, m->d, feat, ldf, F, W, bias, values, do_select,
                     (const uint32_t*)roots, active, cpuct, leaf_status, obs, leaf_mask);
  return launch_check("k_leaf_step");
}

int bk_mcts_expand_backup(bk_mcts* m, const float* logp, const float* values, int prior_mode, void* stream) {
  BK_REQUIRE(m && values && (prior_mode == 0 || prior_mode == 1 || prior_mode == 2), "bad argument");
  BK_REQUIRE(logp || prior_mode == 2, "bad argument: logp");
  const DevPreset& dp = m->ctx->dp;
  const size_t lds = sizeof(uint32_t) * ((size_t)dp.W32pad + kExpandLdsIds);
  hipLaunchKernelGGL(k_expand_backup, dim3(m->d.T), dim3(kWave), lds, (hipStream_t)stream, dp, m->d, logp, values,
                     prior_mode);
  return launch_check("k_expand_backup");
}

int bk_mcts_root_policy(bk_mcts* m, const void* roots, const int32_t* active, double temperature, int32_t* ids,
                        double* pi, int cap, int32_t* counts, void* stream) {
  BK_REQUIRE(m && roots && ids && pi && counts && cap > 0 && temperature >= 0.0, "bad argument");
  hipLaunchKernelGGL(k_root, dim3(m->d.T), dim3(kWave), 0, (hipStream_t)stream, m->d, (const uint32_t*)roots,
                     active, temperature, 0, ids, pi, (uint32_t*)nullptr, (double*)nullptr, (float*)nullptr, cap,
                     counts);
  return launch_check("k_root policy");
}

int bk_mcts_root_stats(bk_mcts* m, const void* roots, const int32_t* active, int32_t* ids, uint32_t* n, double* q,
                       float* p, int cap, int32_t* counts, void* stream) {
  BK_REQUIRE(m && roots && ids && n && q && p && counts && cap > 0, "bad argument");
  hipLaunchKernelGGL(k_root, dim3(m->d.T), dim3(kWave), 0, (hipStream_t)stream, m->d, (const uint32_t*)roots,
                     active, 1.0, 1, ids, (double*)nullptr, n, q, p, cap, counts);
  return launch_check("k_root stats");
}

int bk_mcts_leaf_info(bk_mcts* m, void* leaf_states, int32_t* depths, void* stream) {
  BK_REQUIRE(m && leaf_states && depths, "bad argument");
  int rc = hip_check(hipMemcpyAsync(leaf_states, m->d.leaf_state, (size_t)m->d.T * kStateBytes,
                                    hipMemcpyDeviceToDevice, (hipStream_t)stream), "copy leaf states");
  if (!rc) rc = hip_check(hipMemcpyAsync(depths, m->d.depth, (size_t)m->d.T * sizeof(int32_t),
                                         hipMemcpyDeviceToDevice, (hipStream_t)stream), "copy depths");
  return rc;
}

int bk_mcts_counters(bk_mcts* m, int64_t* out, void* stream) {
  BK_REQUIRE(m && out, "bad argument");
  unsigned long long c[8];
  int rc = hip_check(hipMemcpyAsync(c, m->d.counters, sizeof(c), hipMemcpyDeviceToHost, (hipStream_t)stream),
                     "copy counters");
  if (!rc) rc = hip_check(hipStreamSynchronize((hipStream_t)stream), "sync counters");
  if (rc) return rc;
  std::vector<int32_t> nodes(m->d.T);
  std::vector<int64_t> ch(m->d.T);
  rc = hip_check(hipMemcpy(nodes.data(), m->d.tree_nodes, sizeof(int32_t) * m->d.T, hipMemcpyDeviceToHost),
                 "copy nodes");
  if (!rc) rc = hip_check(hipMemcpy(ch.data(), m->d.tree_children, sizeof(int64_t) * m->d.T,
                                    hipMemcpyDeviceToHost), "copy children");
  if (rc) return rc;
  std::vector<unsigned long long> tcs((size_t)m->d.T * 8);
  rc = hip_check(hipMemcpy(tcs.data(), m->d.tree_ctr, sizeof(unsigned long long) * tcs.size(), hipMemcpyDeviceToHost),
                 "copy tree counters");
  if (rc) return rc;
  int64_t tn = 0, tc = 0;
  for (int t = 0; t < m->d.T; ++t) {
    tn += nodes[t];
    tc += ch[t];
    for (int k = 2; k < 8; ++k) c[k] += tcs[(size_t)t * 8 + k];  // per-tree parts (k_err stays global)
  }
  out[0] = tn;
  out[1] = tc;
  for (int k = 2; k < 8; ++k) out[k] = (int64_t)c[k];
  return BK_OK;
}

}  // extern "C"
