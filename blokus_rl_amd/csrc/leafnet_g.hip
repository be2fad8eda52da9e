// leafnet_g.hip — k_leafnet_x3g: the leaf ResNet of k_leafnet_x3 (models/blokus_nnet.py:88-151, BN
// folded; the same split-f16 products, operand scaling, packed weights, pixel map and stem) with the
// residual tower's convolutions GROUP-MAJOR.
//
// Why: k_leafnet_x3 runs each conv chunk-major — every K chunk over all 25 pixel groups, the 25
// accumulators in AGPRs — so all groups finish together and the epilogue (scale, bias, ReLU, split,
// the grid writes: 5.1k cycles a layer) runs with the matrix cores idle, between two barriers; the
// layer takes 31k cycles against a 21.6k-cycle MFMA floor. Here a wave keeps its 16 output channels'
// weights for the whole conv in registers (18 chunks x hi/lo = 144 VGPRs, the next conv's loading
// into a second set under this one), and runs the groups one after another: group g's 54 MFMAs
// (18 chunks x 3 products) carry, between them, the epilogue of group g-1 and the grid writes of
// group g-4. The tower is one stream of 25 x nlayers group steps with a workgroup barrier between
// steps; no step waits for a whole layer.
//
// In place: a group's outputs overwrite its input pixels in the grid. Group g reads the pixels of
// groups g-3..g+3 (the pixel map's read radius, checked at compile time), so its outputs are held
// back kGD = 4 steps (in registers) and written after the barrier that ends step g+3, mid-step,
// when every read of those pixels issued by any wave is hundreds of cycles old. The next conv's
// first groups read pixels written >= 20 steps earlier. The per-layer operand scale needs the
// previous layer's board maximum: its last group's epilogue runs at the next layer's first step,
// posts the wave maxima, and the next step (after the barrier) reads them — just before the new
// layer's first epilogue needs them.
//
// The last conv writes y (fp32, + x0 from the global workspace, ReLU) into the grid as raw floats
// (a lane's 4 channels in the 16-B slot of its channel half), and a post-pass takes the heads'
// 1x1 convs per pixel from there (as k_leafnet_wx3), then the value MLP (as k_leafnet_x3).
#include "../../include/blokus_engine.h"
#include "ctx.h"

#include "leafnet_common.h"

namespace bk {
namespace {

#ifndef BK_X3G_PROBE
#define BK_X3G_PROBE 0  // timing probes only (wrong results): 1 no step barriers, 2 no B reads in the
                        // tower, 3 no epilogue / writes / weight loads, 4 no MFMAs in the tower
#endif
#ifndef BK_X3G_SGB
#define BK_X3G_SGB 1  // A/B knob: the step scheduled by sched_group_barrier (0: a memory fence per chunk)
#endif
constexpr int kGN = 20, kGNN = kGN * kGN, kGNG = ln_groups(kGN);
constexpr int kGU = 5;       // group steps per unrolled iteration: the period of the acc / output / base rings
constexpr int kGD = 4;       // a group's outputs go into the grid kGD steps after its MFMAs
constexpr int kGC = 9;       // K chunks of 32 per wave and group (half of the 18)
constexpr int kGRing = 3;    // B fragments of local chunk c in ring slot c % kGRing
constexpr int kGPf = 2;      // B reads run kGPf chunks ahead of their MFMAs, on into the next group
constexpr int kGWrite = 5;   // the chunk after which a step writes its delayed outputs
static_assert(kGNG == 25 && kGNG % kGU == 0 && kGC % kGRing == 0 && kGPf < kGRing && kGD < kGU, "x3g rings");

// read radius of the pixel map: the largest |g' - g| over a pixel of group g and a 3x3 neighbour in
// group g'
constexpr int x3g_read_radius() {
  constexpr int RS = ln_row(kGN);
  LnPixMap<kGN> mp{};
  int grp[kGNN] = {};
  for (int i = 0; i < kGNG * 16; ++i) {
    const int sl = mp.slot[i];
    grp[(sl / RS - 1) * kGN + sl % RS - 1] = i / 16;
  }
  int r = 0;
  for (int p = 0; p < kGNN; ++p)
    for (int dr = -1; dr <= 1; ++dr)
      for (int dc = -1; dc <= 1; ++dc) {
        const int rr = p / kGN + dr, cc = p % kGN + dc;
        if (rr < 0 || rr >= kGN || cc < 0 || cc >= kGN) continue;
        const int d = grp[rr * kGN + cc] - grp[p];
        r = d > r ? d : (-d > r ? -d : r);
      }
  return r;
}
static_assert(x3g_read_radius() + 1 <= kGD, "x3g: the output delay must exceed the pixel map's read radius");

#if BK_LN_STAMP
// diagnostic build: s_memtime at the chunk boundaries of one group step (conv 1, group 10) per wave
__device__ unsigned long long g_x3g_stamps[256 * 4 * 16];
__device__ unsigned long long g_x3g_steps[256 * 4 * 64];  // step starts of convs 1 and 2 (50 steps)
#endif

// c ? a : b element by element (a whole-vector select of two array elements became a scratch
// array indexed at run time)
__device__ __forceinline__ f32x4 sel4(int c, f32x4 a, f32x4 b) {
  return f32x4{c ? a[0] : b[0], c ? a[1] : b[1], c ? a[2] : b[2], c ? a[3] : b[3]};
}

template <int N>
__global__ __launch_bounds__(kLnThreads, 1) void k_leafnet_x3g(const float* __restrict__ obs,
                                                               const h16x8* __restrict__ wstem,
                                                               const float* __restrict__ sstem,
                                                               const float* __restrict__ bstem,
                                                               const h16x8* __restrict__ wt,
                                                               const float* __restrict__ st,
                                                               const float* __restrict__ bt,
                                                               const float* __restrict__ bounds, int nlayers,
                                                               LnHeads hd, float* __restrict__ x0ws,
                                                               float* __restrict__ xout) {
  static_assert(N == kGN, "k_leafnet_x3g: 20x20");
  constexpr int NN = N * N, RS = ln_row(N), NG = kGNG, PIX_IT = (NN + kLnThreads - 1) / kLnThreads;
  constexpr int PL = ln_plane(N);
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* act = lds;            // 16 planes [hi q | lo q][(N+2) x RS slots][16 B]
  unsigned char* sin = lds + 16 * PL;  // 2 planes: the stem input hi, lo (the heads' scratch after the tower)
  float* red = reinterpret_cast<float*>(lds + 18 * PL);  // [0..7]: layer maxima by parity, [8..11]: the observation
  int* bases = reinterpret_cast<int*>(lds + 18 * PL + 64);  // [NG][64]: every lane's B-read base per group
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oc = 16 * wave + 4 * ks;
  const size_t b = blockIdx.x;

  // ---- the observation, the halos, the stem: k_leafnet_x3's
  const float* ob = obs + b * kStemCinX3 * NN;
  float xin[PIX_IT][kStemCinX3];
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
#pragma unroll
    for (int c = 0; c < kStemCinX3; ++c) xin[it][c] = p < NN ? ob[c * NN + p] : 0.0f;
  }
  {
    constexpr int kHaloCols = RS - N, kHalo = 2 * RS + N * kHaloCols;
    for (int i = tid; i < 18 * kHalo; i += kLnThreads) {
      const int plane = i / kHalo, k = i - plane * kHalo;
      int row, col;
      if (k < 2 * RS) {
        row = k < RS ? 0 : N + 1;
        col = k < RS ? k : k - RS;
      } else {
        const int h = k - 2 * RS, c = h % kHaloCols;
        row = 1 + h / kHaloCols;
        col = c == 0 ? 0 : N + c;
      }
      *reinterpret_cast<u32x4*>(lds + plane * PL + (row * RS + col) * 16) = u32x4{0u, 0u, 0u, 0u};
    }
  }
  constexpr int kBias = (RS + 1) * 16;
  // the lane's B-read base in group g: its slot + its k-group's plane block, less kBias (the tower
  // reads the slots from LDS: a global table load would put a vmcnt wait in every group step)
  int ab[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) ab[g] = kLnPixMap<N>.slot[16 * g + n] * 16 + ks * 4 * PL - kBias;
  if (wave == 0)
    for (int g = 0; g < NG; ++g) bases[64 * g + l] = ab[g];
  // (a whole base per lane: the value is used as loaded, first by the prefetch at chunk 18 - kGPf,
  // so the wait for it is a counted one behind the ring reads issued after it)
  auto read_base = [&](int g) { return bases[64 * g + l]; };

  // the tower weights: W[set][chunk][part], set = layer parity; layer 0's in flight under the stem
  constexpr int kLayerBlocks = 18 * 4 * 2;
  const __amdgpu_buffer_rsrc_t wrs = ln_rsrc(wt, (unsigned)nlayers * kLayerBlocks * 1024u);
  // the tower: wave w = 2 mh + kh (below); its weights W[set][local chunk][m][part] (set = conv
  // parity) for output blocks 2mh + m and chunks 9kh + j; layer 0's in flight under the stem
  const int kh = wave & 1;
  auto wload2 = [&](int layer, int c, int mb, int p) {
    return __builtin_bit_cast(h16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                         wrs, l * 16, ((layer * kLayerBlocks + c * 8 + mb * 2 + p) * 64) * 16, 0));
  };
  h16x8 W[2][kGC][2][2];
#pragma unroll
  for (int c = 0; c < kGC; ++c)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      W[0][c][m][0] = wload2(0, kGC * kh + c, wave ^ m, 0);
      W[0][c][m][1] = wload2(0, kGC * kh + c, wave ^ m, 1);
    }
  h16x8 wsa[3][2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    wsa[j][0] = wstem[((j * 4 + wave) * 2) * 64 + l];
    wsa[j][1] = wstem[((j * 4 + wave) * 2 + 1) * 64 + l];
  }
  const f32x4 s_stem = *reinterpret_cast<const f32x4*>(sstem + oc), b_stem = *reinterpret_cast<const f32x4*>(bstem + oc);

  float m = 0.0f;
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it)
#pragma unroll
    for (int c = 0; c < kStemCinX3; ++c) m = fmaxf(m, fabsf(xin[it][c]));
  const float max_obs = block_max(m, red + 8, wave, l);
  int ex = scale_exp(max_obs);  // the scale of the current conv input
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
    if (p < NN) {
      unsigned h[4], o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split2(ldexpf(xin[it][2 * q], ex), ldexpf(xin[it][2 * q + 1], ex), h[q], o[q]);
      unsigned char* dst = sin + ((p / N + 1) * RS + p % N + 1) * 16;
      *reinterpret_cast<u32x4*>(dst) = u32x4{h[0], h[1], h[2], h[3]};
      *reinterpret_cast<u32x4*>(dst + PL) = u32x4{o[0], o[1], o[2], o[3]};
    }
  }
  __syncthreads();
  // per-lane byte offsets (from the slot) of the two 8-B stores of a group's outputs: split halves
  // (hi plane, lo plane of the lane's octet, its half of the slot), or raw floats (the last conv:
  // the slot of the plane of the lane's channel half)
  const int o8 = 2 * wave + (ks >> 1);
  const int hiplane = ((o8 & 3) * 4 + (o8 >> 2) * 2) * PL;
  const int ws0 = hiplane + (ks & 1) * 8, ws1 = ws0 + PL;
  const int wr0 = hiplane + (ks & 1) * PL, wr1 = wr0 + 8;
  auto slot_of = [&](int base) { return base - ks * 4 * PL + kBias; };  // read base -> the slot's byte offset
  {
    f32x4 sacc[NG];
    h16x8 rbs[kLnSlots][2];
    auto toff = [&](int j) {
      const int t = 4 * j + ks < 9 ? 4 * j + ks : 8;
      return ((t / 3 - 1) * RS + (t % 3 - 1)) * 16 + kBias - ks * 4 * PL;
    };
    ln_prime<NG, PL>(rbs, sin, ab, toff(0));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j == 0)
        ln_chunk<NG, true, PL>(sacc, wsa[0][0], wsa[0][1], sin, ab, toff(0), toff(1), rbs);
      else
        ln_chunk<NG, false, PL>(sacc, wsa[j][0], wsa[j][1], sin, ab, toff(j), toff(j < 2 ? j + 1 : j), rbs);
    }
    ln_mfma_drain(sacc);
    // stem epilogue (k_leafnet_x3's arithmetic): x0 = relu(acc s 2^-ex + b) -> the workspace
    // (unscaled, for the final residual), and scaled by 2^ex0 and split -> the grid
    const int ex0 = scale_exp(bounds[0] * max_obs + bounds[1]);
    const f32x2 s01{ldexpf(s_stem.x, -ex), ldexpf(s_stem.y, -ex)}, s23{ldexpf(s_stem.z, -ex), ldexpf(s_stem.w, -ex)};
    const f32x2 b01{b_stem.x, b_stem.y}, b23{b_stem.z, b_stem.w};
    const float up = ldexpf(1.0f, ex0);
    float mx = 0.0f;
    f32x4* x0b = reinterpret_cast<f32x4*>(x0ws) + b * NN * 16;  // [pixel][channel quad]
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      f32x2 y01 = pk_fma(f32x2{sacc[g][0], sacc[g][1]}, s01, b01);
      f32x2 y23 = pk_fma(f32x2{sacc[g][2], sacc[g][3]}, s23, b23);
      y01 = f32x2{max_bits(y01.x, 0), max_bits(y01.y, 0)};
      y23 = f32x2{max_bits(y23.x, 0), max_bits(y23.y, 0)};
      mx = max3_abs(max3_abs(mx, y01.x, y01.y), y23.x, y23.y);
      const int sl = slot_of(ab[g]) / 16;
      x0b[((sl / RS - 1) * N + sl % RS - 1) * 16 + oc / 4] = f32x4{y01.x, y01.y, y23.x, y23.y};
      unsigned h0, h1, l0, l1;
      split2(y01.x * up, y01.y * up, h0, l0);
      split2(y23.x * up, y23.y * up, h1, l1);
      unsigned char* dst = act + slot_of(ab[g]);
      *reinterpret_cast<u32x2*>(dst + ws0) = u32x2{h0, h1};
      *reinterpret_cast<u32x2*>(dst + ws1) = u32x2{l0, l1};
    }
    // the tower's first conv reads the stem's board maximum from the parity-0 slots
    mx = wave_max_f(mx);
    if (l == 0) red[wave] = mx;
    __syncthreads();  // the grid and the maxima complete
    ex = ex0;
  }

  // ---- the residual tower, group-major, K split over wave pairs (file comment): wave w = 2 mh + kh
  // accumulates output blocks w (m = 0) and w^1 (m = 1, its partner's; 16 channels each) over chunks
  // 9kh..9kh+8, hands its partial sums of block w^1 to the partner through LDS and finishes block w
  // (= its stem block) as the sum of the two halves' partial sums
  float4* xch = reinterpret_cast<float4*>(sin);  // [group parity 2][wave 4][64 lanes]: partial sums
  // rings indexed by the step's position u in its iteration of kGU (static in the unrolled code)
  f32x4 acc[kGU][2];  // indexed by compile-time constants only (a wave-uniform kh index would put it in scratch)
  u32x4 pend[kGU];
  int abr[kGU];
  h16x8 rb[kGRing][2];
  // the epilogue state of the conv whose groups are being finished
  f32x2 e_s01{0.f, 0.f}, e_s23{0.f, 0.f}, e_b01{0.f, 0.f}, e_b23{0.f, 0.f};
  int e_floor = 0, e_k = 0;
  bool e_last = false;
  float mx = 0.0f;
#pragma unroll
  for (int u = 0; u < kGU; ++u) {
    acc[u][0] = acc[u][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    pend[u] = u32x4{0u, 0u, 0u, 0u};
  }
  abr[0] = ab[0];
  // chunk c = (tap c/2, channel half c%2): a compile-time offset from the read base (per half kh)
  auto coff_of = [&](int c) {
    const int t = c >> 1;
    return 2 * (c & 1) * PL + ((t / 3 - 1) * RS + (t % 3 - 1)) * 16 + kBias;
  };
  // the wave's local chunk j is global chunk kGC kh + j
  auto lcoff = [&](int j) { return coff_of(kh ? kGC + j : j); };
#pragma unroll
  for (int c = 0; c < kGPf; ++c) ln_load<PL>(rb[c % kGRing], act, abr[0], lcoff(c));
  f32x4 sv{0.f, 0.f, 0.f, 0.f}, bv{0.f, 0.f, 0.f, 0.f};

  // the epilogue of one group: y = acc s + b, floor (ReLU or none), the lane maximum, and the packed
  // outputs (split halves, or raw floats after the last conv, whose residual and ReLU the heads'
  // pass applies)
  auto epi = [&](f32x4 a) {
    f32x2 y01 = pk_fma(f32x2{a[0], a[1]}, e_s01, e_b01);
    f32x2 y23 = pk_fma(f32x2{a[2], a[3]}, e_s23, e_b23);
    y01 = f32x2{max_bits(y01.x, e_floor), max_bits(y01.y, e_floor)};
    y23 = f32x2{max_bits(y23.x, e_floor), max_bits(y23.y, e_floor)};
    mx = max3_abs(max3_abs(mx, y01.x, y01.y), y23.x, y23.y);
    unsigned h0, h1, l0, l1;
    split2(y01.x, y01.y, h0, l0);
    split2(y23.x, y23.y, h1, l1);
    // bit_cast whole vectors: hipcc's bit_cast of an ext_vector element reads element 0 (ROCm 7.2)
    const u32x2 r01 = __builtin_bit_cast(u32x2, y01), r23 = __builtin_bit_cast(u32x2, y23);
    const u32x4 raw{r01.x, r01.y, r23.x, r23.y};
    return e_last ? raw : u32x4{h0, h1, l0, l1};
  };
  // a group's finished block: the two K halves' partial sums, kh 0 first whichever wave adds
  auto partner = [&](int par) {  // the partner's partial sums of this wave's block
    const float4 o = xch[(par * 4 + (wave ^ 1)) * 64 + l];
    return f32x4{o.x, o.y, o.z, o.w};
  };
  auto finish = [&](f32x4 own, f32x4 other) { return add4(own, other); };  // (IEEE addition commutes)
  auto post = [&](f32x4 a, int par) {  // this wave's partial sums of its partner's block
    xch[(par * 4 + wave) * 64 + l] = make_float4(a[0], a[1], a[2], a[3]);
  };
  auto write_out = [&](u32x4 v, int base, int off0, int off1) {
    unsigned char* dst = act + slot_of(base);
    *reinterpret_cast<u32x2*>(dst + off0) = u32x2{v.x, v.y};
    *reinterpret_cast<u32x2*>(dst + off1) = u32x2{v.z, v.w};
  };
  auto set_epilogue = [&](int layer) {
    // conv `layer`'s epilogue state, from the board maximum of its input
    const bool last = layer + 1 == nlayers;
    const float max_in = fmaxf(fmaxf(red[4 * (layer & 1)], red[4 * (layer & 1) + 1]),
                               fmaxf(red[4 * (layer & 1) + 2], red[4 * (layer & 1) + 3]));
    const int ex_out = scale_exp(bounds[2 * (layer + 1)] * max_in + bounds[2 * (layer + 1) + 1]);
    const int ko = last ? 0 : ex_out;
    e_s01 = f32x2{ldexpf(sv.x, ko - ex), ldexpf(sv.y, ko - ex)};
    e_s23 = f32x2{ldexpf(sv.z, ko - ex), ldexpf(sv.w, ko - ex)};
    e_b01 = f32x2{ldexpf(bv.x, ko), ldexpf(bv.y, ko)};
    e_b23 = f32x2{ldexpf(bv.z, ko), ldexpf(bv.w, ko)};
    e_floor = (!(layer & 1) && !last) ? 0 : (int)0x80000000u;
    e_k = ko;
    e_last = last;
    ex = ex_out;
  };

  // one group step of conv `layer` (weight set P, group g = 5 i + U of the layer; FIRST: i == 0):
  // the group's MFMAs; under them the partial-sum hand-off of group g-1, the epilogue of group g-2,
  // the delayed grid writes of group g-4 and (FIRST) a fifth of the next conv's weights
  auto step = [&](auto pc, auto fc, auto uc, int layer, int g) {
    constexpr int P = decltype(pc)::value;
    constexpr bool FIRST = decltype(fc)::value;
    constexpr int U = decltype(uc)::value, UP = (U + kGU - 1) % kGU, UP2 = (U + kGU - 2) % kGU, UN = (U + 1) % kGU;
    const bool last = layer + 1 == nlayers;
    const int tau = layer * NG + g;
    if (FIRST && U == 2) set_epilogue(layer);
    // the write offsets of the group written this step (a group of the previous conv at the first
    // kGD steps of a conv: never the last conv)
    const bool wraw = !(FIRST && U < kGD) && last;
    const int w0 = wraw ? wr0 : ws0, w1 = wraw ? wr1 : ws1;
    const bool wvalid = !(FIRST && U < kGD) || layer > 0;
    const int gn = g + 1 < NG ? g + 1 : 0;
    int nbase = 0;
    f32x4 xo{0.f, 0.f, 0.f, 0.f};
#if BK_LN_STAMP
    unsigned long long tst[kGC + 1] = {};
    const bool stamp = P == 1 && !FIRST && U == 0 && layer == 1 && g == 10;
    if (stamp) asm volatile("s_memtime %0" : "=s"(tst[0]));
    if ((layer == 1 || layer == 2) && l == 0 && blockIdx.x < 256) {
      unsigned long long ts;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts) :: "memory");
      g_x3g_steps[(blockIdx.x * 4 + wave) * 64 + (layer - 1) * NG + g] = ts;
    }
#endif
#pragma unroll
    for (int c = 0; c < kGC; ++c) {
      const int cc = c + kGPf;
      if (BK_X3G_PROBE != 2) {
        if (cc < kGC)
          ln_load<PL>(rb[cc % kGRing], act, abr[U], lcoff(cc));
        else
          ln_load<PL>(rb[cc % kGRing], act, abr[UN], lcoff(cc - kGC));
      }
#if !BK_X3G_SGB
      // the reads stay at their chunk (the scheduler would sink them next to their MFMAs)
      asm volatile("" ::: "memory");
#endif
      const h16x8 bh = rb[c % kGRing][0], bl = rb[c % kGRing][1];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        f32x4 a = c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[U][m];
        a = mfma16(W[P][c][m][0], bh, a);
        a = mfma16(W[P][c][m][1], bh, a);
        a = mfma16(W[P][c][m][0], bl, a);
        acc[U][m] = a;
      }
      if (c == 0) {
        nbase = read_base(gn);
        xo = partner((tau - 2) & 1);  // read here, used at chunk 2: a counted wait behind the ring
      }
      if (c == 1) post(acc[UP][1], (tau - 1) & 1);  // group g-1's partial sums for the partner
      if (c == 2) {
        // group g-2 finished (at a conv's first two steps: the previous conv's last groups, then
        // its wave maxima for this conv's bound)
        if (FIRST && U < 2) {
          if (layer > 0) {
            pend[UP2] = epi(finish(acc[UP2][0], xo));
            if (U == 1) {
              const float wm = wave_max_f(ldexpf(mx, -e_k));
              if (l == 0) red[4 * (layer & 1) + wave] = wm;
            }
          }
          if (U == 1) mx = 0.0f;
        } else {
          pend[UP2] = epi(finish(acc[UP2][0], xo));
        }
      }
      if (FIRST && c >= 1) {
        // the next conv's weights into the other set, a fifth per step (the last conv reloads its
        // own: unconditional loads keep the wait counts static)
        constexpr int k0 = 4 * kGC * U / kGU, k1 = 4 * kGC * (U + 1) / kGU;
        const int nl = last ? layer : layer + 1;
#pragma unroll
        for (int k = k0 + 2 * (c - 1); k < k1 && k < k0 + 2 * c; ++k)
          W[1 - P][k >> 2][(k >> 1) & 1][k & 1] = wload2(nl, kGC * kh + (k >> 2), wave ^ ((k >> 1) & 1), k & 1);
      }
      if (c == kGWrite) {
        if (FIRST && U < kGD) {
          if (wvalid) write_out(pend[UN], abr[UN], w0, w1);
        } else {
          write_out(pend[UN], abr[UN], w0, w1);
        }
        abr[UN] = nbase;
      }
#if BK_LN_STAMP
      if (stamp) asm volatile("s_memtime %0" : "=s"(tst[c + 1]));
#endif
    }
#if BK_X3G_SGB
    // the step's schedule: per chunk its two B reads, then each MFMA followed by one VALU op
#pragma unroll
    for (int c = 0; c < kGC; ++c) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, 1, 0);
      }
    }
#endif
#if BK_LN_STAMP
    if (stamp && l == 0 && blockIdx.x < 256) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k <= kGC; ++k) g_x3g_stamps[(blockIdx.x * 4 + wave) * 16 + k] = tst[k];
    }
#endif
    if (BK_X3G_PROBE != 1) asm volatile("s_barrier" ::: "memory");
  };
  auto iteration = [&](auto pc, auto fc, int layer, int i) {
    step(pc, fc, std::integral_constant<int, 0>{}, layer, 5 * i + 0);
    step(pc, fc, std::integral_constant<int, 1>{}, layer, 5 * i + 1);
    step(pc, fc, std::integral_constant<int, 2>{}, layer, 5 * i + 2);
    step(pc, fc, std::integral_constant<int, 3>{}, layer, 5 * i + 3);
    step(pc, fc, std::integral_constant<int, 4>{}, layer, 5 * i + 4);
  };
  auto conv = [&](auto pc, int layer) {
    sv = *reinterpret_cast<const f32x4*>(st + layer * 64 + oc);
    bv = *reinterpret_cast<const f32x4*>(bt + layer * 64 + oc);
    iteration(pc, std::true_type{}, layer, 0);
    for (int i = 1; i < NG / kGU; ++i) iteration(pc, std::false_type{}, layer, i);
  };
  for (int layer = 0; layer < nlayers; layer += 2) {
    conv(std::integral_constant<int, 0>{}, layer);
    if (layer + 1 < nlayers) conv(std::integral_constant<int, 1>{}, layer + 1);
  }
  // drain (the steps after the last conv's group 24 = position 4): its partial sums and the
  // epilogue of group 23, then group 24's, then (every read of the grid done) groups 21..24 out
  {
    const int tau = nlayers * NG;  // the step after the last
    post(acc[kGU - 1][1], (tau - 1) & 1);
    pend[kGU - 2] = epi(finish(acc[kGU - 2][0], partner((tau - 2) & 1)));
    __syncthreads();
    pend[kGU - 1] = epi(finish(acc[kGU - 1][0], partner((tau - 1) & 1)));
    __syncthreads();
#pragma unroll
    for (int u = 1; u < kGU; ++u) write_out(pend[u], abr[u], wr0, wr1);
    __syncthreads();
  }

  // ---- heads (blokus_nnet.py:146-150, BN folded): the tower output y is in the grid as raw floats
  // (channel quad q of a pixel: the slot of plane ((q/2)%4) 4 + (q/8) 2 + q%2); per pixel the two
  // policy and one value 1x1 convs, a quad per lane summed over 16 lanes
  float* vfeat = reinterpret_cast<float*>(sin);
  float* part = vfeat + NN;
  float* hsum = part + 256;  // [NN][3]
  {
    const int nb = tid >> 4, cb = tid & 15;
    const int oq = cb >> 1;
    const int qplane = ((oq & 3) * 4 + (oq >> 2) * 2 + (cb & 1)) * PL;
    const f32x4 hw0 = *reinterpret_cast<const f32x4*>(hd.wp + 4 * cb);
    const f32x4 hw1 = *reinterpret_cast<const f32x4*>(hd.wp + 64 + 4 * cb);
    const f32x4 hwv = *reinterpret_cast<const f32x4*>(hd.wv + 4 * cb);
    const f32x4* x0b = reinterpret_cast<const f32x4*>(x0ws) + b * NN * 16 + cb;
    for (int i = nb; i < NN; i += kLnThreads / 16) {
      const int slot = (i / N + 1) * RS + i % N + 1;
      // the tower output: relu(y + x0) (blokus_nnet.py:140-141), as k_leafnet_x3's last epilogue
      const f32x4 y = *reinterpret_cast<const f32x4*>(act + qplane + slot * 16);
      const f32x4 x0 = x0b[i * 16];
      const f32x2 s01 = pk_add(f32x2{y[0], y[1]}, f32x2{x0[0], x0[1]});
      const f32x2 s23 = pk_add(f32x2{y[2], y[3]}, f32x2{x0[2], x0[3]});
      const f32x4 v{max_bits(s01.x, 0), max_bits(s01.y, 0), max_bits(s23.x, 0), max_bits(s23.y, 0)};
      float d0 = v.x * hw0.x + v.y * hw0.y + v.z * hw0.z + v.w * hw0.w;
      float d1 = v.x * hw1.x + v.y * hw1.y + v.z * hw1.z + v.w * hw1.w;
      float dv = v.x * hwv.x + v.y * hwv.y + v.z * hwv.z + v.w * hwv.w;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        d0 += __shfl_xor(d0, o);
        d1 += __shfl_xor(d1, o);
        dv += __shfl_xor(dv, o);
      }
      if (cb == 0) {
        hsum[3 * i] = d0;
        hsum[3 * i + 1] = d1;
        hsum[3 * i + 2] = dv;
      }
      if (xout) *reinterpret_cast<f32x4*>(xout + (b * NN + i) * 64 + 4 * cb) = v;
    }
  }
  __syncthreads();
  for (int i = tid; i < NN; i += kLnThreads) {
    const float p0 = hsum[3 * i], p1 = hsum[3 * i + 1], pv = hsum[3 * i + 2];
    hd.pf[b * 2 * NN + i] = fmaxf(p0 + hd.bp[0], 0.0f);
    hd.pf[b * 2 * NN + NN + i] = fmaxf(p1 + hd.bp[1], 0.0f);
    vfeat[i] = fmaxf(pv + hd.bv[0], 0.0f);
  }
  __syncthreads();
  {
    constexpr int Q = NN / 4;
    const int q0 = Q * wave;
    float w[Q];
#pragma unroll
    for (int k = 0; k < Q; ++k) w[k] = hd.w1t[(size_t)(q0 + k) * 64 + l];
    float a0 = 0.f, a1 = 0.f;
    int k = 0;
#pragma unroll
    for (; k + 10 <= Q; k += 10) {
#pragma unroll
      for (int u = 0; u < 10; u += 2) {
        a0 += w[k + u] * vfeat[q0 + k + u];
        a1 += w[k + u + 1] * vfeat[q0 + k + u + 1];
      }
    }
#pragma unroll
    for (; k < Q; ++k) a0 += w[k] * vfeat[q0 + k];
    part[wave * 64 + l] = a0 + a1;
  }
  __syncthreads();
  if (wave == 0) {
    const float h = fmaxf(((part[l] + part[64 + l]) + (part[128 + l] + part[192 + l])) + hd.b1[l], 0.0f);
    for (int q = 0; q < hd.P; ++q) {
      const float sum = wave_sum_f(hd.w2[q * 64 + l] * h);
      if (l == 0) hd.v[b * hd.P + q] = tanhf(sum + hd.b2[q]);
    }
  }
}

constexpr int x3g_lds_bytes() { return ln_lds_bytes(kGN) + kGNG * 64 * 4; }
static_assert(x3g_lds_bytes() <= 160 * 1024, "k_leafnet_x3g: LDS");
static_assert(3 * kGNN * 4 + kGNN * 4 + 256 * 4 <= 2 * ln_plane(kGN), "k_leafnet_x3g: heads scratch");

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_leafnet_x3g_supported(int N) { return N == kGN; }

#if BK_LN_STAMP
int bk_x3g_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x3g_stamps), sizeof(g_x3g_stamps)) == hipSuccess ? 0 : -1;
}
int bk_x3g_steps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x3g_steps), sizeof(g_x3g_steps)) == hipSuccess ? 0 : -1;
}
#endif

int bk_leafnet_x3g(const float* obs, int B, int N, int cin, const void* wstem, const float* sstem, const float* bstem,
                   int nlayers, const void* wtower, const float* stower, const float* btower, const float* bounds,
                   const float* wp, const float* bp, const float* wv, const float* bv, const float* w1t,
                   const float* b1, const float* w2, const float* b2, int P, float* pf, float* vout, float* x0ws,
                   float* out, void* stream) {
  BK_REQUIRE(obs && wstem && sstem && bstem && wtower && stower && btower && bounds && B >= 0, "bad argument");
  BK_REQUIRE(wp && bp && wv && bv && w1t && b1 && w2 && b2 && pf && vout && x0ws && P > 0, "bad argument");
  BK_REQUIRE(cin == kStemCinX3, "bk_leafnet_x3g: the stem takes 8 observation planes");
  BK_REQUIRE(nlayers >= 1, "bk_leafnet_x3g: at least one tower conv");
  BK_REQUIRE(bk_leafnet_x3g_supported(N), "bk_leafnet_x3g: N must be 20");
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  BK_REQUIRE(a16(wstem) && a16(wtower) && a16(sstem) && a16(bstem) && a16(stower) && a16(btower) && a16(wp) &&
                 a16(wv) && a16(x0ws) && a16(out),
             "bk_leafnet_x3g: 16-byte aligned buffers");
  if (B == 0) return BK_OK;
  {
    const void* fns[1] = {(const void*)k_leafnet_x3g<kGN>};
    if (set_max_dynamic_lds(fns, 1, x3g_lds_bytes()) != BK_OK) return BK_EHIP;
  }
  const LnHeads h{wp, bp, wv, bv, w1t, b1, w2, b2, P, pf, vout};
  hipLaunchKernelGGL(k_leafnet_x3g<kGN>, dim3(B), dim3(kLnThreads), x3g_lds_bytes(), (hipStream_t)stream, obs,
                     reinterpret_cast<const h16x8*>(wstem), sstem, bstem, reinterpret_cast<const h16x8*>(wtower),
                     stower, btower, bounds, nlayers, h, x0ws, out);
  return launch_check("k_leafnet_x3g");
}

}  // extern "C"
