// sims.hip — whole MCTS simulations in one launch (bk_mcts_simulate_resnet / _const).
//
// The batched search runs a simulation as four launches over all T trees: k_select -> the leaf
// ResNet (k_tower_wino) -> k_leaf_logits -> k_expand_backup (mcts.hip, conv.hip). Every stage
// touches only its own tree and board, so no stage needs the whole grid to have finished the one
// before. Here one workgroup (4 waves, one per SIMD; one per CU, the tower's LDS) owns one tree
// and runs `nsims` simulations of it back to back in a single launch; per simulation
//   select_tree       wave 0: descent from the root to a new or terminal board, the leaf's
//                     state, legal bitmask and observation (mcts.py:37-66)
//   tower_forward     4 waves: stem conv, the Winograd residual tower, the heads' 1x1 convs and
//                     the value MLP of the leaf (models/blokus_nnet.py:135-151, BN folded)
//   leaf_logits_tree  4 waves: the policy Linear over the leaf's legal ids only
//   expand_tree       wave 0: priors (softmax over the legal ids), the new node, the backup
//                     (mcts.py:50-70)
// The stages are the per-stage kernels' own device functions with the same arithmetic, so the
// trees come out bitwise identical (tests/test_sims_gpu.py). What the fusion removes is the
// grid-wide step between stages: the dependent-launch gaps, and every stage waiting for the
// slowest tree of the stage before — here each tree goes at its own pace, and the per-tree spread
// in descent depth and legal-move count averages out over the nsims simulations.
// Handoff between stages (data one wave wrote, others of the CU read): the writers wait for their
// stores (vmcnt 0), workgroup barrier, L1 invalidate.
#define BK_BOARD_SYNC() ::bk::wave_lds_sync()  // select / expand run on one wave
#include "../../include/blokus_engine.h"
#include "ctx.h"
#include "legal_rows.h"
#include "mcts_dev.h"
#include "tower_dev.h"

namespace bk {
namespace {

// the leaf net's operands (those of bk_resnet_stem_tower_heads + the policy Linear) and the
// per-tree scratch rows
struct SimNet {
  TowerHeads hd;  // heads and stem weights; the pf [T][2NN], v [T][P], obs [T][8][N][N] scratch
  const float* u2all;
  const float* biasall;
  int nlayers;
  const float* W;     // policy Linear [A][2NN]
  const float* bias;  // [A]
  float* x0;          // activations [T][N][N][64]
  float* hA;
  float* hB;
};

// stores of one wave visible to the others of the workgroup (and to its own later loads)
__device__ __forceinline__ void wg_handoff() {
  __builtin_amdgcn_s_waitcnt(0x0F70);           // vmcnt(0): this wave's stores are done
  __syncthreads();
  asm volatile("buffer_inv sc0" ::: "memory");  // no stale L1 lines of what the others wrote
}
__device__ __forceinline__ void wave_handoff() {
  __builtin_amdgcn_s_waitcnt(0x0F70);
  wave_lds_sync();
  asm volatile("buffer_inv sc0" ::: "memory");
}

// The search stages as out-of-line calls inside k_sims: inlined next to the tower they pushed the
// kernel's register allocation into 3 KB/lane of scratch (the tower's U array is 256 AGPRs).
__device__ __noinline__ int sims_select(const DevPreset& dp, const DevMcts& m, int t, const uint32_t* roots,
                                        const int32_t* active, double cpuct, float* obs, uint32_t* lds) {
  return select_tree(dp, m, t, roots, active, cpuct, nullptr, obs, nullptr, lds);
}
__device__ __noinline__ void sims_leaf_logits(const DevPreset& dp, const DevMcts& m, int t, const float* feat, int F,
                                              const float* W, const float* bias, uint32_t* lds) {
  leaf_logits_tree<2>(dp, m, t, 0, 1, feat, F, F, W, bias, lds);
}
__device__ __noinline__ void sims_expand(const DevPreset& dp, const DevMcts& m, int t, const float* values,
                                         uint32_t* lds) {
  expand_tree(dp, m, t, nullptr, values, 2, lds);
}

template <int N>
__device__ __noinline__ void sims_tower(float* lds, const SimNet& net) {
  tower_forward<N, true, true>(lds, net.x0, net.hA, net.hB, nullptr, net.u2all, net.biasall, net.nlayers, net.hd);
}

template <int N>
__global__ __launch_bounds__(kW2Threads, 1) void k_sims(DevPreset dp, DevMcts m, const uint32_t* __restrict__ roots,
                                                        const int32_t* __restrict__ active, double cpuct, int nsims,
                                                        SimNet net) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];  // the tower's; the search stages reuse it
  __shared__ int status_sh;
  const int t = blockIdx.x, wave = threadIdx.x >> 6;
  float* lds = reinterpret_cast<float*>(lds32);
  constexpr int F = 2 * N * N;
  for (int sim = 0; sim < nsims; ++sim) {
    if (wave == 0) {
      const int st = sims_select(dp, m, t, roots, active, cpuct, const_cast<float*>(net.hd.obs), lds32);
      if (threadIdx.x == 0) status_sh = st;
    }
    wg_handoff();
    const int status = status_sh;
    if (status == 1) {
      sims_tower<N>(lds, net);
      wg_handoff();
      sims_leaf_logits(dp, m, t, net.hd.pf, F, net.W, net.bias, lds32);
      wg_handoff();
    }
    if (wave == 0 && status != 0) sims_expand(dp, m, t, net.hd.v, lds32);
    wg_handoff();
  }
}

// Uninformed search (DumbNet, compare_arena.py:87-95: the same logp [T][A] and values [T][P] for
// every leaf of tree t): select + expand/backup with dense priors, nsims times, one wave per tree.
__global__ __launch_bounds__(64) void k_sims_const(DevPreset dp, DevMcts m, const uint32_t* __restrict__ roots,
                                                   const int32_t* __restrict__ active, double cpuct, int nsims,
                                                   const float* __restrict__ logp, const float* __restrict__ values) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  uint32_t* lds = lds32;
  const int t = blockIdx.x;
  for (int sim = 0; sim < nsims; ++sim) {
    const int st = select_tree(dp, m, t, roots, active, cpuct, nullptr, nullptr, nullptr, lds);
    wave_handoff();
    if (st != 0) expand_tree(dp, m, t, logp, values, 0, lds);
    wave_handoff();
  }
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" int bk_mcts_simulate_resnet(bk_mcts* m, const void* roots, const int32_t* active, double cpuct, int nsims,
                                       int nlayers, const float* wstem, const float* bstem, const float* u2all,
                                       const float* biasall, const float* wp, const float* bp, const float* wv,
                                       const float* bv, const float* w1t, const float* b1, const float* w2,
                                       const float* b2, const float* policy_w, const float* policy_b, float* obs,
                                       float* x0, float* hA, float* hB, float* pf, float* v, void* stream) {
  BK_REQUIRE(m && roots && nsims >= 0 && nlayers >= 1, "bad argument");
  BK_REQUIRE(wstem && bstem && u2all && biasall && wp && bp && wv && bv && w1t && b1 && w2 && b2 && policy_w &&
                 policy_b && obs && x0 && hA && hB && pf && v,
             "bad argument");
  const DevPreset& dp = m->ctx->dp;
  const int N = dp.N, F = 2 * N * N;
  BK_REQUIRE((N == 14 || N == 20) && 2 * dp.P == kStemCin,
             "bk_mcts_simulate_resnet: 14x14 or 20x20 boards with 4 players (the 8-plane stem)");
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  BK_REQUIRE(a16(x0) && a16(hA) && a16(hB) && a16(u2all) && a16(biasall) && a16(wp) && a16(wv) && a16(policy_w) &&
                 a16(obs) && a16(pf),
             "bk_mcts_simulate_resnet: 16-byte aligned buffers");
  // the tower's LDS (V buffers + the heads' partials); the search stages run inside it
  const size_t lds = sizeof(float) * (2 * (size_t)kW2VBuf + (size_t)N * N * 12);
  BK_REQUIRE(sizeof(uint32_t) * ((size_t)kStateWords + 2 * kMaxN + dp.W32pad) <= lds &&
                 sizeof(uint32_t) * ((size_t)dp.W32pad + kLeafCap + F) <= lds &&
                 sizeof(uint32_t) * ((size_t)dp.W32pad + kExpandLdsIds) <= lds && F <= kMaxFeat &&
                 F <= 64 * kLeafQ,
             "bk_mcts_simulate_resnet: stage buffers exceed the LDS");
  {
    const void* fns[2] = {(const void*)k_sims<14>, (const void*)k_sims<20>};
    if (set_max_dynamic_lds(fns, 2, (int)(sizeof(float) * (2 * kW2VBuf + 20 * 20 * 12))) != BK_OK) return BK_EHIP;
  }
  if (nsims == 0) return BK_OK;
  SimNet net{};
  net.hd = TowerHeads{wp, bp, wv, bv, w1t, b1, w2, b2, dp.P, pf, v, 0, obs, wstem, bstem};
  net.u2all = u2all;
  net.biasall = biasall;
  net.nlayers = nlayers;
  net.W = policy_w;
  net.bias = policy_b;
  net.x0 = x0;
  net.hA = hA;
  net.hB = hB;
  hipStream_t s = (hipStream_t)stream;
  if (N == 20)
    hipLaunchKernelGGL((k_sims<20>), dim3(m->d.T), dim3(kW2Threads), lds, s, dp, m->d, (const uint32_t*)roots, active,
                       cpuct, nsims, net);
  else
    hipLaunchKernelGGL((k_sims<14>), dim3(m->d.T), dim3(kW2Threads), lds, s, dp, m->d, (const uint32_t*)roots, active,
                       cpuct, nsims, net);
  return launch_check("k_sims");
}

extern "C" int bk_mcts_simulate_const(bk_mcts* m, const void* roots, const int32_t* active, double cpuct, int nsims,
                                      const float* logp, const float* values, void* stream) {
  BK_REQUIRE(m && roots && logp && values && nsims >= 0, "bad argument");
  const DevPreset& dp = m->ctx->dp;
  const size_t a = (size_t)kStateWords + 2 * kMaxN + dp.W32pad, b = (size_t)dp.W32pad + kExpandLdsIds;
  const size_t lds = sizeof(uint32_t) * (a > b ? a : b);
  if (nsims == 0) return BK_OK;
  hipLaunchKernelGGL(k_sims_const, dim3(m->d.T), dim3(kWave), lds, (hipStream_t)stream, dp, m->d,
                     (const uint32_t*)roots, active, cpuct, nsims, logp, values);
  return launch_check("k_sims_const");
}
