// env.hip — batched Blokus rules engine on gfx950 + the env half of the C-ABI
// (include/blokus_engine.h). One 64-lane wave per board; see common.h.
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <utility>

#include <cstdlib>

#include "../../include/blokus_engine.h"
#include "ctx.h"
#include "legal_rows.h"

namespace bk {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return BK_OK;
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  return BK_EHIP;
}
int launch_check(const char* what) { return hip_check(hipGetLastError(), what); }

int set_max_dynamic_lds(const void* const* fns, int n, int bytes) {
  // The attribute belongs to the kernel on the current device: remember (device, kernel) pairs
  // already raised, under a lock (several host threads may launch on several devices).
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  if (hip_check(hipGetDevice(&dev), "hipGetDevice") != BK_OK) return BK_EHIP;
  std::lock_guard<std::mutex> lock(mu);
  for (int i = 0; i < n; ++i) {
    if (done.count({dev, fns[i]})) continue;
    if (hip_check(hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize, bytes),
                  "hipFuncSetAttribute") != BK_OK)
      return BK_EHIP;
    done.insert({dev, fns[i]});
  }
  return BK_OK;
}

namespace {

__global__ void k_init_states(DevPreset dp, uint32_t* states, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * kStateWords) return;
  const int w = i % kStateWords;
  uint32_t v = 0;
  if (w >= kWPieces && w < kWPieces + kMaxP) v = (w - kWPieces) < dp.P ? dp.full_pieces : 0u;
  if (w == kWHash) v = 0x7F4A7C15u;      // hash of the empty board = the seed
  if (w == kWHash + 1) v = 0x9E3779B9u;
  states[i] = v;
}

// Legal-move bitmask of B boards. Grid = B blocks of one wave.
__global__ __launch_bounds__(64) void k_legal_mask(DevPreset dp, const uint32_t* __restrict__ states,
                                                   const int32_t* __restrict__ players, int B,
                                                   uint64_t* __restrict__ masks, int32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* s = lds;                                   // 96 words
  uint64_t* fa = reinterpret_cast<uint64_t*>(lds + kStateWords);  // 20 u64
  uint32_t* m32 = lds + kStateWords + 2 * kMaxN;       // W32pad words
  const int b = blockIdx.x;
  const int l = lane_id();
  load_state(s, states + (size_t)b * kStateWords);
  __syncthreads();
  int q = players ? players[b] : -1;
  if (q < 0) q = (int)s[kWToMove];
  build_mask(dp, s, q, fa, m32);
  int cnt = 0;
  uint64_t* out = masks + (size_t)b * dp.W64;
  for (int j = l; j < dp.W64; j += kWave) {
    const uint64_t w = (uint64_t)m32[2 * j] | ((uint64_t)m32[2 * j + 1] << 32);
    cnt += __popcll(w);
    out[j] = w;
  }
  cnt = wave_sum(cnt);
  if (counts && l == 0) counts[b] = cnt;
}

__global__ __launch_bounds__(64) void k_legal_ids(DevPreset dp, const uint32_t* __restrict__ states,
                                                  const int32_t* __restrict__ players, int B, int32_t* ids,
                                                  int cap, int32_t* counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* s = lds;
  uint64_t* fa = reinterpret_cast<uint64_t*>(lds + kStateWords);
  uint32_t* m32 = lds + kStateWords + 2 * kMaxN;
  const int b = blockIdx.x;
  load_state(s, states + (size_t)b * kStateWords);
  __syncthreads();
  int q = players ? players[b] : -1;
  if (q < 0) q = (int)s[kWToMove];
  build_mask(dp, s, q, fa, m32);
  const int K = compact_ids(dp, m32, ids + (size_t)b * cap, cap);
  if (lane_id() == 0) counts[b] = K <= cap ? K : -K;
}

__global__ __launch_bounds__(64) void k_next_state(DevPreset dp, const uint32_t* __restrict__ in,
                                                   const int32_t* __restrict__ actions, int B, uint32_t* out,
                                                   int32_t* next_players, int32_t* status) {
  __shared__ __attribute__((aligned(16))) uint32_t s[kStateWords];
  __shared__ uint64_t fa[kMaxN];
  const int b = blockIdx.x;
  load_state(s, in + (size_t)b * kStateWords);
  __syncthreads();
  const int a = actions[b];
  int st = 0;
  if (a >= 0) st = apply_action(dp, s, a, fa);
  store_state(out + (size_t)b * kStateWords, s);
  if (lane_id() == 0) {
    if (next_players) next_players[b] = (int)s[kWToMove];
    if (status) status[b] = st;
  }
}

__global__ void k_game_ended(DevPreset dp, const uint32_t* __restrict__ states, int B, int32_t* ended,
                             double* scores) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint32_t* s = states + (size_t)b * kStateWords;
  const bool over = s[kWFlags] & kFlagOver;
  if (ended) ended[b] = over ? 1 : 0;
  if (!scores) return;
  double sc[kMaxP];
  if (over) {
    terminal_scores(dp, s, sc);
  } else {
    for (int k = 0; k < kMaxP; ++k) sc[k] = 0.0;
  }
  for (int k = 0; k < dp.P; ++k) scores[(size_t)b * dp.P + k] = sc[k];
}

__global__ void k_square_counts(DevPreset dp, const uint32_t* __restrict__ states, int B, int32_t* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint32_t* s = states + (size_t)b * kStateWords;
  for (int k = 0; k < dp.P; ++k) out[(size_t)b * dp.P + k] = squares_of(dp, s, k);
}

// Observation planes [2P][N][N] f32 (Board.canonical_board, blokus_wrapper.py:146): one block
// of 256 threads per board, each thread a run of cells.
__global__ __launch_bounds__(256) void k_observe(DevPreset dp, const uint32_t* __restrict__ states, int B,
                                                 float* __restrict__ obs) {
  const int b = blockIdx.x;
  const uint32_t* s = states + (size_t)b * kStateWords;
  const int NN = dp.N * dp.N;
  const int total = 2 * dp.P * NN;
  const int tm = (int)s[kWToMove];
  float* o = obs + (size_t)b * total;
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int plane = i / NN, cell = i - plane * NN;
    float v;
    if (plane < dp.P) {
      const int r = cell / dp.N, c = cell - r * dp.N;
      v = (float)((s[plane * kMaxN + r] >> c) & 1u);
    } else {
      v = (plane - dp.P) == tm ? 1.0f : 0.0f;
    }
    o[i] = v;
  }
}

}  // namespace
}  // namespace bk

using namespace bk;

static size_t mask_lds_bytes(const DevPreset& dp) {
  return sizeof(uint32_t) * (size_t)(kStateWords + 2 * kMaxN + dp.W32pad);
}

extern "C" {

const char* bk_last_error(void) { return g_last_error.c_str(); }
int bk_version(void) { return 1; }
int bk_state_bytes(void) { return BK_STATE_BYTES; }

int bk_ctx_create(int board_size, int num_players, int max_piece_cells, int device, bk_ctx** out) {
  BK_REQUIRE(out, "out is null");
  *out = nullptr;
  bk_ctx* c = new bk_ctx();
  if (!build_preset(board_size, num_players, max_piece_cells, &c->pre)) {
    delete c;
    set_error("unsupported preset");
    return BK_EINVAL;
  }
  c->device = device;
  const Preset& p = c->pre;
  DevPreset& d = c->dp;
  d.N = p.N; d.P = p.P; d.A = p.A; d.W64 = p.mask_words; d.W32 = p.mask_words32;
  d.W32pad = 4 * ((p.mask_words + 1) / 2);  // 16-B aligned rows of u32 in LDS
  d.num_items = p.num_items; d.num_pieces = p.num_pieces;
  d.full_pieces = p.full_pieces;
  d.full_row = (1u << p.N) - 1u;
  d.corner_r4 = d.corner_c4 = 0u;
  for (int k = 0; k < kMaxP; ++k) {
    d.corner_r4 |= (uint32_t)(p.corner_r[k] & 0xFF) << (8 * k);
    d.corner_c4 |= (uint32_t)(p.corner_c[k] & 0xFF) << (8 * k);
  }
  for (int i = 0; i <= kNumPieces; ++i) d.piece_item_off[i] = (int16_t)p.piece_item_off[i];
  // the unrolled kernel's compile-time orientations must be the host tables' orientations
  bool same = (int)p.orients.size() <= kNumOrient;
  for (size_t o = 0; same && o < p.orients.size(); ++o) {
    const std::vector<int>& od = p.orients[o];
    const OrientC& k = kOrient[o];
    same = od[0] == k.piece && od[1] == k.h && od[2] == k.w && od[3] == k.n;
    for (int q = 0; same && q < 5; ++q) same = od[4 + q] == k.dr[q] && od[9 + q] == k.dc[q];
  }
  if (!same) {
    delete c;
    set_error("orient_table.h disagrees with the host orientation tables (re-run gen_orient.py)");
    return BK_EINVAL;
  }
  {
    const char* e = std::getenv("BK_LEGAL_KERNEL");
    c->legal_items_kernel = e && std::string(e) == "items";
    const char* w = std::getenv("BK_LEGAL_WPB");  // waves per workgroup (A/B knob)
    c->legal_wpb = w ? std::atoi(w) : 1;
  }
  if (device < 0) {  // host-only context: tables, no device memory (CPU tests, tooling)
    *out = c;
    return BK_OK;
  }
  int rc = hip_check(hipSetDevice(device), "hipSetDevice");
  if (rc) { delete c; return rc; }
  rc = hip_check(hipMalloc(&c->d_items, sizeof(uint64_t) * p.items.size()), "hipMalloc items");
  std::vector<uint4> act_it(p.act.size());
  for (size_t a = 0; a < p.act.size(); ++a) {
    const uint64_t it = p.items[p.act[a] & 0xFFFFu];
    act_it[a] = make_uint4((uint32_t)it, (uint32_t)(it >> 32), p.act[a], 0u);
  }
  if (!rc) rc = hip_check(hipMalloc(&c->d_act_it, sizeof(uint4) * act_it.size()), "hipMalloc act_it");
  if (!rc) rc = hip_check(hipMemcpy(c->d_items, p.items.data(), sizeof(uint64_t) * p.items.size(),
                                    hipMemcpyHostToDevice), "copy items");
  if (!rc) rc = hip_check(hipMemcpy(c->d_act_it, act_it.data(), sizeof(uint4) * act_it.size(),
                                    hipMemcpyHostToDevice), "copy act_it");
  if (!rc) {
    // k_legal_mask_staged's pack table: u32 word k of the mask is the OR over the fields
    // overlapping it of hi32(field << sh), field (O, r) at stage slot O * kStageRows + r starting
    // at bit S = base(O) + r * W, sh = S - 32k + 32; entries 18 bits (slot | sh << 12), 3 per u64.
    // Presets whose narrowest field is short enough that a word can overlap > 3 fields (N < 20)
    // have no table: the staged variant falls back to the atomic kernel there.
    std::vector<uint64_t> ent(2 * (size_t)p.mask_words, 0ull);
    std::vector<int> used(2 * (size_t)p.mask_words, 0);
    int64_t base = 0;
    bool fits = true;
    for (size_t o = 0; o < p.orients.size() && fits; ++o) {
      const int h = p.orients[o][1], w = p.orients[o][2];
      const int R = p.N - h + 1, W = p.N - w + 1;
      for (int r = 0; r < R && fits; ++r) {
        const int64_t S = base + (int64_t)r * W;
        for (int64_t k = S / 32; k <= (S + W - 1) / 32; ++k) {
          const int sh = (int)(S - 32 * k + 32);
          const int64_t slot = (int64_t)o * kStageRows + r;
          if (k >= (int64_t)ent.size() || used[k] >= 3 || sh < 1 || sh > 63 || slot >= 4096) {
            fits = false;
            break;
          }
          ent[k] |= ((uint64_t)slot | ((uint64_t)sh << 12)) << (18 * used[k]++);
        }
      }
      base += (int64_t)R * W;
    }
    if (fits && base == p.A) {
      rc = hip_check(hipMalloc(&c->d_pack, sizeof(uint64_t) * ent.size()), "hipMalloc pack");
      if (!rc) rc = hip_check(hipMemcpy(c->d_pack, ent.data(), sizeof(uint64_t) * ent.size(), hipMemcpyHostToDevice),
                              "copy pack");
    }
  }
  if (rc) { bk_ctx_destroy(c); return rc; }
  d.items = c->d_items;
  d.act_it = c->d_act_it;
  *out = c;
  return BK_OK;
}

int bk_ctx_destroy(bk_ctx* c) {
  if (!c) return BK_OK;
  if (c->d_items) (void)hipFree(c->d_items);
  if (c->d_act_it) (void)hipFree(c->d_act_it);
  if (c->d_pack) (void)hipFree(c->d_pack);
  delete c;
  return BK_OK;
}

int bk_action_size(const bk_ctx* c) { return c ? c->pre.A : BK_EINVAL; }
int bk_mask_words(const bk_ctx* c) { return c ? c->pre.mask_words : BK_EINVAL; }
int bk_num_pieces(const bk_ctx* c) { return c ? c->pre.num_pieces : BK_EINVAL; }

int bk_action_table(const bk_ctx* c, int32_t* out) {
  BK_REQUIRE(c && out, "null argument");
  std::memcpy(out, c->pre.act_table.data(), sizeof(int32_t) * c->pre.act_table.size());
  return BK_OK;
}

int bk_action_cells(const bk_ctx* c, int16_t* out) {
  BK_REQUIRE(c && out, "null argument");
  std::memcpy(out, c->pre.act_cells.data(), sizeof(int16_t) * c->pre.act_cells.size());
  return BK_OK;
}

int bk_init_states(bk_ctx* c, void* states, int B, void* stream) {
  BK_REQUIRE(c && states && B >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  if (B == 0) return BK_OK;
  const int n = B * kStateWords;
  hipLaunchKernelGGL(k_init_states, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, c->dp,
                     (uint32_t*)states, B);
  return launch_check("k_init_states");
}

int bk_legal_mask(bk_ctx* c, const void* states, const int32_t* players, int B, uint64_t* mask_words,
                  int32_t* counts, void* stream) {
  BK_REQUIRE(c && states && mask_words && B >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  if (B == 0) return BK_OK;
  if (c->legal_items_kernel) {  // A/B reference: the item-loop kernel (BK_LEGAL_KERNEL=items)
    hipLaunchKernelGGL(k_legal_mask, dim3(B), dim3(kWave), mask_lds_bytes(c->dp), (hipStream_t)stream, c->dp,
                       (const uint32_t*)states, players, B, mask_words, counts);
    return launch_check("k_legal_mask");
  }
  const int bpw = kWave / c->dp.N;
  const size_t lds = sizeof(uint32_t) * (size_t)bpw * (size_t)c->dp.W32pad;
  const dim3 grid((B + bpw - 1) / bpw);
  const hipStream_t st = (hipStream_t)stream;
  const uint32_t* sp = (const uint32_t*)states;
#define BK_LEGAL_LAUNCH(W, S) \
  hipLaunchKernelGGL((k_legal_mask_rows<W, S>), grid, dim3(64 * W), lds, st, c->dp, sp, players, B, mask_words, counts)
#define BK_LEGAL_LAUNCH_NT(W, S)                                                                      \
  hipLaunchKernelGGL((k_legal_mask_rows<W, S, 0, 20>), grid, dim3(64 * W), lds, st, c->dp, sp, players, B, \
                     mask_words, counts)
  const bool classic = c->dp.N == 20 && c->dp.num_pieces == kNumPieces && c->dp.W64 == kClassicW64 &&
                       c->dp.W32pad == kClassicW32pad;
  switch (c->legal_wpb) {
    case 2: BK_LEGAL_LAUNCH(2, 0); break;
    case 4: BK_LEGAL_LAUNCH(4, 0); break;
    case 8: BK_LEGAL_LAUNCH(8, 0); break;
    case 12: BK_LEGAL_LAUNCH(2, 1); break;
    case 14: BK_LEGAL_LAUNCH(4, 1); break;
    case 21:  // two boards per wave (balanced grid at B = 4096)
      if (c->dp.N * 2 <= kWave) {
        hipLaunchKernelGGL((k_legal_mask_rows<1, 0, 2>), dim3((B + 1) / 2), dim3(64),
                           sizeof(uint32_t) * 2 * (size_t)c->dp.W32pad, st, c->dp, sp, players, B, mask_words, counts);
        break;
      }
      BK_LEGAL_LAUNCH(1, 0);
      break;
    case 31: {  // staged: no LDS atomics (legal_rows.h)
      if (!c->d_pack || kWave / c->dp.N > kStageMaxBoards) { BK_LEGAL_LAUNCH(1, 0); break; }
      const int bytes = legal_stage_lds_bytes(c->dp.N);
      static const void* fns[] = {(const void*)k_legal_mask_staged<kStageMaxBoards>};
      if (int rc = set_max_dynamic_lds(fns, 1, bytes)) return rc;
      hipLaunchKernelGGL(k_legal_mask_staged<kStageMaxBoards>, grid, dim3(64), bytes, st, c->dp, sp, players, B,
                         (const uint4*)c->d_pack, mask_words, counts);
      return launch_check("k_legal_mask_staged");
    }
    case 11: BK_LEGAL_LAUNCH(1, 1); break;  // even/odd origin rows in separate LDS atomics: 15.1 vs 12.1 us
    case 40: BK_LEGAL_LAUNCH(1, 0); break;  // the round-4 step: bit-reversed rows, row/column masks
    // lean steps on 2 / 3 waves per group (each wave every 2nd / 3rd orientation)
    case 45: if (classic) BK_LEGAL_LAUNCH_NT(3, 3); else BK_LEGAL_LAUNCH(1, 3); break;
    case 46: if (classic) BK_LEGAL_LAUNCH_NT(2, 3); else BK_LEGAL_LAUNCH(1, 3); break;
    default:  // 1: one wave per group of 3 boards, the lean step (validity folded into the rows, which
              // are in board order), at the compile-time size on the classic board
      if (classic) BK_LEGAL_LAUNCH_NT(1, 3); else BK_LEGAL_LAUNCH(1, 3);
      break;
  }
#undef BK_LEGAL_LAUNCH
#undef BK_LEGAL_LAUNCH_NT
  return launch_check("k_legal_mask_rows");
}

int bk_legal_ids(bk_ctx* c, const void* states, const int32_t* players, int B, int32_t* ids, int cap,
                 int32_t* counts, void* stream) {
  BK_REQUIRE(c && states && ids && counts && B >= 0 && cap > 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_legal_ids, dim3(B), dim3(kWave), mask_lds_bytes(c->dp), (hipStream_t)stream, c->dp,
                     (const uint32_t*)states, players, B, ids, cap, counts);
  return launch_check("k_legal_ids");
}

int bk_next_state(bk_ctx* c, const void* states_in, const int32_t* actions, int B, void* states_out,
                  int32_t* next_players, int32_t* status, void* stream) {
  BK_REQUIRE(c && states_in && actions && states_out && B >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  BK_REQUIRE(states_in != states_out, "states_out must not alias states_in");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_next_state, dim3(B), dim3(kWave), 0, (hipStream_t)stream, c->dp,
                     (const uint32_t*)states_in, actions, B, (uint32_t*)states_out, next_players, status);
  return launch_check("k_next_state");
}

int bk_game_ended(bk_ctx* c, const void* states, int B, int32_t* ended, double* scores, void* stream) {
  BK_REQUIRE(c && states && B >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_game_ended, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, c->dp,
                     (const uint32_t*)states, B, ended, scores);
  return launch_check("k_game_ended");
}

int bk_square_counts(bk_ctx* c, const void* states, int B, int32_t* out, void* stream) {
  BK_REQUIRE(c && states && out && B >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_square_counts, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, c->dp,
                     (const uint32_t*)states, B, out);
  return launch_check("k_square_counts");
}

int bk_observe(bk_ctx* c, const void* states, int B, float* obs, void* stream) {
  BK_REQUIRE(c && states && obs && B >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_observe, dim3(B), dim3(256), 0, (hipStream_t)stream, c->dp, (const uint32_t*)states, B,
                     obs);
  return launch_check("k_observe");
}

}  // extern "C"
