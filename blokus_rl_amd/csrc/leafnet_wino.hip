// leafnet_wino.hip — the leaf ResNet (models/blokus_nnet.py:88-151, eval-mode BN folded) of one
// 20x20 board per workgroup with its residual tower as Winograd F(2x2,3x3) convolutions on
// split-f16 MFMA products ("wx3"): fp32-class accuracy at 2.25x fewer matrix products than the
// direct form of leafnet.hip (k_leafnet_x3).
//
// Arithmetic. Per 64->64 conv and 2x2 output tile: V = B^T d B (the tile's 4x4 input window d,
// per input channel, in fp32), M_xi = sum_c U_xi[o][c] V_xi[c] for the 16 positions xi = (xi1, xi2)
// of the 4x4 transform domain, y = A^T M A (F(2x2,3x3): B^T, G, A^T as in Lavin & Gray). U =
// G g G^T is computed on the host in fp64 (nets.pack_wx3), scaled per output channel by a power
// of two into [2^14, 2^15) and split into f16 hi + lo; V is split on the device after the
// transform (the layer input is stored scaled by 2^e so that |V| <= 4 max|d| < 2^15). Each
// product is hi*hi + lo*hi + hi*lo on v_mfma_f32_16x16x32_f16 (exact f16 products, f32
// accumulation), as in k_leafnet_x3; the scalings are undone exactly in the epilogue.
//
// Decomposition (one workgroup of 4 waves per board, one wave per SIMD): wave q owns the row
// xi1 = q of the transform domain for ALL 64 output channels — its U (64 x 64 channels x 4 xi2 x
// hi/lo) in 256 AGPRs for the layer — so a wave's B operands are its own: each lane reads the
// two window rows its B^T row combines (tile n = lane % 16, 8 input channels of a K chunk) from
// the activation grid in LDS and transforms and splits them in registers. The transform domain
// never goes through LDS. The 100 tiles form 7 groups of 16 (the MFMA columns; the last has 4
// spare). Per group a wave reduces its rows of M to the A^T row sums R_q (2 values per output
// channel and tile) and writes them to LDS; after a barrier every thread (one tile x 4 output
// channels) adds the four waves' R into the 2x2 outputs y = sum_q A^T[.][q] R_q, applies the
// epilogue and holds y until every wave has read the next group's windows (the grid is updated
// in place): two barriers per group. The stem (8 -> 64) stays the direct x3 conv of
// leafnet_common.h; x0 waits in a global workspace for the final residual.
#include "leafnet_common.h"

namespace bk {
namespace {

#if BK_LN_STAMP
constexpr int kWxStamps = 64;
__device__ unsigned long long g_wx_stamps[256 * 4 * kWxStamps];
#define WXSTAMP(i)                                                                                          \
  do {                                                                                                      \
    if (l == 0 && blockIdx.x < 256)                                                                         \
      g_wx_stamps[(blockIdx.x * 4 + wave) * kWxStamps + (i)] = __builtin_amdgcn_s_memtime();                \
  } while (0)
#else
#define WXSTAMP(i) \
  do {             \
  } while (0)
#endif

constexpr int kWxN = 20;                            // the 20x20 preset
constexpr int kWxNN = kWxN * kWxN;
constexpr int kWxT = kWxN / 2;                      // tiles per row
constexpr int kWxTiles = kWxT * kWxT;               // 100 output tiles of 2x2 pixels
constexpr int kWxTG = (kWxTiles + 15) / 16;         // 7 tile groups of 16
constexpr int kWxGR = kWxN + 2;                     // activation grid: 1-pixel zero halo
constexpr int kWxActBytes = kWxGR * kWxGR * 256;    // [22][22] pixels x 64 channels fp32
constexpr int kWxRBytes = 4 * 2 * 16 * 256;         // R: [wave q][r 2][tile 16][64 channels] f32
constexpr int kWxROff = kWxActBytes;
constexpr int kWxRedOff = kWxActBytes + kWxRBytes;
constexpr int kWxLds = kWxRedOff + 64;
constexpr int kWxLayerBlocks = 256;                 // (q, m, xi2, chunk, half) blocks of 1 KB per conv
static_assert(kWxLds <= 160 * 1024, "k_leafnet_wx3: LDS");
static_assert(2 * ln_plane(kWxN) <= kWxRBytes, "k_leafnet_wx3: the stem input planes live in the R buffer");

// activation grid: pixel (gr, gc) at (gr * 22 + gc) * 256, channel quad s (channels 4s..4s+3)
// at 16-B slot s ^ wx_g(gr, gc). A window read (lane: tile n = lane % 16, quad slot wx_slot) of 8
// lanes of one k-group hits 8 consecutive tiles, so 8 distinct (t + const) & 7; the two k-groups of
// a ds_read_b128 lane group differ in slot bit 3 (wx_slot): conflict-free. The epilogue's 8-lane
// store groups (one pixel, 8 quads) likewise.
__device__ __forceinline__ int wx_g(int gr, int gc) { return (10 * (gr >> 1) + (gc >> 1)) & 7; }
// the grid slot of the B-operand channels of k-group ks, K chunk ch, half h (elements 4h..4h+3 of
// the lane's 8): the K index 8 ks + e of chunk ch is channel 4 wx_slot(ks, ch, e / 4) + e % 4
__host__ __device__ constexpr int wx_slot(int ks, int ch, int h) { return 8 * (ks & 1) + 4 * (ks >> 1) + 2 * ch + h; }

// one MFMA step: acc (+)= ah*bh + al*bh + ah*bl. Inline asm pins the operands' register files —
// U (A) in AGPRs, the accumulator in VGPRs — which the builtin left to a register allocator that
// split U over both files and spilled. hipcc pads nothing inside asm: the s_nop 1 covers a B
// operand the transform has just written (VALU write -> MFMA read); the accumulator's readers
// wait behind wx_drain.
#ifndef BK_WX_PROBE
#define BK_WX_PROBE 0  // timing probes (tools): 1 no MFMAs, 2 no transform VALU
#endif
#ifndef BK_WX_ASM
#define BK_WX_ASM 1  // A/B knob: 0 = the MFMA builtin (the compiler allocates and schedules)
#endif
#if BK_WX_ASM
template <bool INIT>
__device__ __forceinline__ void wx_mfma(f32x4& acc, const h16x8& ah, const h16x8& al, const h16x8& bh,
                                        const h16x8& bl) {
  if (INIT)
    asm volatile(
        "s_nop 1\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %2, 0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
        : "=&v"(acc)
        : "a"(ah), "v"(bh), "a"(al), "v"(bl));
  else
    asm volatile(
        "s_nop 1\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
        : "+v"(acc)
        : "a"(ah), "v"(bh), "a"(al), "v"(bl));
}
#else
template <bool INIT>
__device__ __forceinline__ void wx_mfma(f32x4& acc, const h16x8& ah, const h16x8& al, const h16x8& bh,
                                        const h16x8& bl) {
  f32x4 c = INIT ? f32x4{0.f, 0.f, 0.f, 0.f} : acc;
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
}
#endif
// the last MFMAs' results -> VALU reads (16-pass-class XDL write -> VALU read: 12+ wait states);
// the empty asm on each accumulator keeps its readers below the wait
__device__ __forceinline__ void wx_drain(f32x4 (&acc)[4][4]) {
#if BK_WX_ASM
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int m = 0; m < 4; ++m) asm volatile("" : "+v"(acc[x][m]));
#else
  (void)acc;
#endif
}

__device__ __forceinline__ f32x4 relu4(f32x4 y) {
  return f32x4{max_bits(y.x, 0), max_bits(y.y, 0), max_bits(y.z, 0), max_bits(y.w, 0)};
}

// (x, y) -> packed f16 hi halves and lo halves of 4 values: h16x8 element order (a.x..a.w, b.x..b.w)
__device__ __forceinline__ void split8(f32x4 a, f32x4 b, h16x8& hi, h16x8& lo) {
  unsigned h[4], o[4];
  split2(a.x, a.y, h[0], o[0]);
  split2(a.z, a.w, h[1], o[1]);
  split2(b.x, b.y, h[2], o[2]);
  split2(b.z, b.w, h[3], o[3]);
  hi = __builtin_bit_cast(h16x8, u32x4{h[0], h[1], h[2], h[3]});
  lo = __builtin_bit_cast(h16x8, u32x4{o[0], o[1], o[2], o[3]});
}

__device__ __forceinline__ float sum16(float a) {  // sum over the 16 lanes of a DPP row
  a += __shfl_xor(a, 1);
  a += __shfl_xor(a, 2);
  a += __shfl_xor(a, 4);
  a += __shfl_xor(a, 8);
  return a;
}

__global__ __launch_bounds__(kLnThreads, 1) void k_leafnet_wx3(const float* __restrict__ obs,
                                                               const h16x8* __restrict__ wstem,
                                                               const float* __restrict__ sstem,
                                                               const float* __restrict__ bstem,
                                                               const h16x8* __restrict__ ut,
                                                               const float* __restrict__ su,
                                                               const float* __restrict__ bt,
                                                               const float* __restrict__ bounds, int nlayers,
                                                               LnHeads hd, float* __restrict__ x0ws,
                                                               float* __restrict__ xout) {
  constexpr int N = kWxN, NN = kWxNN, RS = ln_row(N), NG = ln_groups(N), PIX_IT = (NN + kLnThreads - 1) / kLnThreads;
  constexpr int PL = ln_plane(N);
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* act = lds;
  unsigned char* rbuf = lds + kWxROff;
  unsigned char* sin = rbuf;  // the stem's input planes (hi, lo), before the tower uses the R buffer
  float* red = reinterpret_cast<float*>(lds + kWxRedOff);
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oc = 16 * wave + 4 * ks;
  const size_t b = blockIdx.x;
  WXSTAMP(0);

  // ---- the observation, the halos, the stem (as k_leafnet_x3)
  const float* ob = obs + b * kStemCinX3 * NN;
  float xin[PIX_IT][kStemCinX3];
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
#pragma unroll
    for (int c = 0; c < kStemCinX3; ++c) xin[it][c] = p < NN ? ob[c * NN + p] : 0.0f;
  }
  {
    // the stem planes' halo
    constexpr int kHaloCols = RS - N, kHalo = 2 * RS + N * kHaloCols;
    for (int i = tid; i < 2 * kHalo; i += kLnThreads) {
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
      *reinterpret_cast<u32x4*>(sin + plane * PL + (row * RS + col) * 16) = u32x4{0u, 0u, 0u, 0u};
    }
    // the activation grid's halo: rows 0, 21 and columns 0, 21 (84 pixels x 16 quads)
    constexpr int kHaloPix = 2 * kWxGR + 2 * N;
    for (int i = tid; i < kHaloPix * 16; i += kLnThreads) {
      const int k = i >> 4, s = i & 15;
      int gr, gc;
      if (k < 2 * kWxGR) {
        gr = k < kWxGR ? 0 : kWxGR - 1;
        gc = k < kWxGR ? k : k - kWxGR;
      } else {
        const int h = k - 2 * kWxGR;
        gr = 1 + (h >> 1);
        gc = (h & 1) ? kWxGR - 1 : 0;
      }
      *reinterpret_cast<u32x4*>(act + (gr * kWxGR + gc) * 256 + s * 16) = u32x4{0u, 0u, 0u, 0u};
    }
  }
  constexpr int kBias = (RS + 1) * 16;
  int ab[NG];
  unsigned valid = 0;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int sl = kLnPixMap<N>.slot[16 * g + n];
    ab[g] = (sl >= 0 ? sl : RS + 1) * 16 + ks * 4 * PL - kBias;
    valid |= (sl >= 0 ? 1u : 0u) << g;
  }
  auto is_valid = [&](int g) { return NN % 16 == 0 || ((valid >> g) & 1u); };
  auto slot_b = [&](int g) { return ab[g] - ks * 4 * PL + kBias; };
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
  const int ex_obs = scale_exp(max_obs);
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
    if (p < NN) {
      unsigned h[4], o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        split2(ldexpf(xin[it][2 * q], ex_obs), ldexpf(xin[it][2 * q + 1], ex_obs), h[q], o[q]);
      unsigned char* dst = sin + ((p / N + 1) * RS + p % N + 1) * 16;
      *reinterpret_cast<u32x4*>(dst) = u32x4{h[0], h[1], h[2], h[3]};
      *reinterpret_cast<u32x4*>(dst + PL) = u32x4{o[0], o[1], o[2], o[3]};
    }
  }
  __syncthreads();
  f32x4 sacc[NG];
  {
    h16x8 rb[kLnSlots][2];
    auto toff = [&](int j) {
      const int t = 4 * j + ks < 9 ? 4 * j + ks : 8;
      return ((t / 3 - 1) * RS + (t % 3 - 1)) * 16 + kBias - ks * 4 * PL;
    };
    ln_prime<NG, PL>(rb, sin, ab, toff(0));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j == 0)
        ln_chunk<NG, true, PL>(sacc, wsa[0][0], wsa[0][1], sin, ab, toff(0), toff(1), rb);
      else
        ln_chunk<NG, false, PL>(sacc, wsa[j][0], wsa[j][1], sin, ab, toff(j), toff(j < 2 ? j + 1 : j), rb);
    }
  }
  ln_mfma_drain(sacc);

  // stem epilogue: x0 = relu(conv + b) -> the global workspace (unscaled, for the final residual)
  // and, scaled by 2^ex so that the first conv's V fits f16 (|V| <= 4 max|d|), the grid (natural
  // channel quads: slot oc/4, swizzled)
  float max_in;
  int ex;  // the scale of the activation grid's contents
  {
    ex = scale_exp(4.0f * (bounds[0] * max_obs + bounds[1]));
    const f32x4 sv{ldexpf(s_stem.x, -ex_obs), ldexpf(s_stem.y, -ex_obs), ldexpf(s_stem.z, -ex_obs),
                   ldexpf(s_stem.w, -ex_obs)};
    const float up = ldexpf(1.0f, ex);
    float mx = 0.0f;
    float* x0b = x0ws + b * NN * 64;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const f32x4 y = relu4(sacc[g] * sv + b_stem);
      if (is_valid(g)) {
        mx = max3_abs(max3_abs(mx, y.x, y.y), y.z, y.w);
        const int px = ln_pixel<N>(slot_b(g) / 16);
        *reinterpret_cast<f32x4*>(x0b + px * 64 + oc) = y;
        const int gr = px / N + 1, gc = px % N + 1;
        *reinterpret_cast<f32x4*>(act + (gr * kWxGR + gc) * 256 + (((4 * wave + ks) ^ wx_g(gr, gc)) * 16)) = y * up;
      }
    }
    max_in = block_max(mx, red, wave, l);  // the barrier also completes the grid
  }

  // ---- the residual tower
  // U of one conv: [q 4][m 4][xi2 4][chunk 2][half 2][lane 64][8 f16]: wave q, lane (ks, n) holds
  // U[16m + n][channel of K index 8 ks + e of the chunk][q][xi2] (wx_slot order)
  const __amdgpu_buffer_rsrc_t urs = ln_rsrc(ut, (unsigned)nlayers * kWxLayerBlocks * 1024u);
  h16x8 Ua[4][4][2][2];  // [m][xi2][chunk][half]
  auto uload = [&](int layer, int ch) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int blk = (((wave * 4 + m) * 4 + x) * 2 + ch) * 2 + h;
          Ua[m][x][ch][h] = __builtin_bit_cast(
              h16x8, __builtin_amdgcn_raw_buffer_load_b128(urs, l * 16, (layer * kWxLayerBlocks + blk) * 1024, 0));
        }
  };
  uload(0, 0);
  uload(0, 1);
  WXSTAMP(1);

  // the wave's B^T row: t = d[rA] + sgn d[rB] (xi1 = 0: d0 - d2, 1: d1 + d2, 2: d2 - d1, 3: d1 - d3)
  const int rA = wave == 0 ? 0 : wave == 3 ? 1 : wave;  // 0, 1, 2, 1
  const int rB = wave == 0 ? 2 : wave == 1 ? 2 : wave == 2 ? 1 : 3;
  const f32x2 sgn = wave == 1 ? f32x2{1.0f, 1.0f} : f32x2{-1.0f, -1.0f};
  // the phase-B thread: tile nb of the group, output channel quad cb
  const int nb = tid >> 4, cb = tid & 15;

  for (int layer = 0; layer < nlayers; ++layer) {
    const bool LAST = layer + 1 == nlayers;
    const int rfloor = (!(layer & 1) || LAST) ? 0 : (int)0x80000000u;  // max_bits floor: ReLU or identity
    const f32x4 suv = *reinterpret_cast<const f32x4*>(su + layer * 64 + 4 * cb);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bt + layer * 64 + 4 * cb);
    const int ex_out = scale_exp(4.0f * (bounds[2 * (layer + 1)] * max_in + bounds[2 * (layer + 1) + 1]));
    const int ko = LAST ? 0 : ex_out;
    const f32x4 sc{ldexpf(suv.x, ko - ex), ldexpf(suv.y, ko - ex), ldexpf(suv.z, ko - ex), ldexpf(suv.w, ko - ex)};
    const f32x4 bc{ldexpf(bv.x, ko), ldexpf(bv.y, ko), ldexpf(bv.z, ko), ldexpf(bv.w, ko)};
    float mx = 0.0f;
    f32x4 yv[2][2];  // phase B: the group's outputs, held until they may go into the grid
    int ystore = -1;  // the group whose yv waits to be stored

    // phase B's deferred store of group tg's outputs (grid, or the heads' sums after the last conv)
    auto store_y = [&](int tg) {
      const int t = 16 * tg + nb;
      if (t >= kWxTiles) return;
      const int ti = (t * 205) >> 11, tj = t - ti * kWxT;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int gr = 2 * ti + 1 + ii, gc = 2 * tj + 1 + jj;
          unsigned char* px = act + (gr * kWxGR + gc) * 256;
          *reinterpret_cast<f32x4*>(px + ((cb ^ wx_g(gr, gc)) * 16)) = yv[ii][jj];
        }
    };

    // the window rows of a (group, chunk): rows rA and rB x 4 pixels x the lane's 2 channel quads.
    // Addresses: the slot swizzle (t + const) & 7 is the same for tiles t and t + 16, so the
    // per-(row, column pair, chunk, half) offsets are fixed for the layer; the tile's window base
    // steps by 56 or 80 pixels from one group to the next (wbase, set by wbase_at).
    f32x4 W[2][4][2];  // [row A/B][pixel column][half]
    int woff[2][2][2][2];  // [row A/B][column pair][chunk][half] byte offsets from the window base
    {
      const int t0 = n;
#pragma unroll
      for (int ab = 0; ab < 2; ++ab)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
          const int r = ab ? rB : rA;
          const int g = (t0 + 10 * (r >> 1) + cc) & 7;
#pragma unroll
          for (int ch = 0; ch < 2; ++ch)
#pragma unroll
            for (int h = 0; h < 2; ++h) woff[ab][cc][ch][h] = (r * kWxGR + 2 * cc) * 256 + ((wx_slot(ks, ch, h) ^ g) * 16);
        }
    }
    auto wbase_at = [&](int tg) {
      int t = 16 * tg + n;
      t = t < kWxTiles ? t : n;  // spare columns (tg 6) read the window of tile n (same swizzle class)
      const int ti = (t * 205) >> 11, tj = t - ti * kWxT;
      return (2 * ti * kWxGR + 2 * tj) * 256;
    };
    int wbase = wbase_at(0);
    auto wload = [&](int base, int ch) {
      const unsigned char* p = act + base;
#pragma unroll
      for (int ab = 0; ab < 2; ++ab)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            W[ab][c][h] = *reinterpret_cast<const f32x4*>(p + woff[ab][c >> 1][ch][h] + (c & 1) * 256);
    };
    f32x4 Rv[4][2];  // the A^T row sums of the 4 waves for the phase-B thread (read after barrier Y)
    // phase B: y of group tg from Rv (tile nb, channels 4cb..4cb+3): epilogue into yv / hsum
    auto phase_b = [&](int tg) {
      const int tb = 16 * tg + nb;
      const int tbi = (tb * 205) >> 11, tbj = tb - tbi * kWxT;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        yv[0][jj] = add4(Rv[0][jj], add4(Rv[1][jj], Rv[2][jj]));
        yv[1][jj] = sub4(sub4(Rv[1][jj], Rv[2][jj]), Rv[3][jj]);
      }
      const bool real = tb < kWxTiles;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          f32x4 v = fma4(yv[ii][jj], sc, bc);
          const int px = (2 * tbi + ii) * N + 2 * tbj + jj;
          if (LAST && real) v = add4(v, *reinterpret_cast<const f32x4*>(x0ws + (b * NN + px) * 64 + 4 * cb));
          v = f32x4{max_bits(v.x, rfloor), max_bits(v.y, rfloor), max_bits(v.z, rfloor), max_bits(v.w, rfloor)};
          if (real) mx = max3_abs(max3_abs(mx, v.x, v.y), v.z, v.w);
          yv[ii][jj] = v;
          if (LAST && xout && real) *reinterpret_cast<f32x4*>(xout + (b * NN + px) * 64 + 4 * cb) = v;
        }
      ystore = tg;
    };

    wload(wbase, 0);
    for (int tg = 0; tg < kWxTG; ++tg) {
      const int wnext = tg + 1 < kWxTG ? wbase_at(tg + 1) : wbase;
      // ---- phase A: this wave's row q of the transform domain for the group's 16 tiles; the
      // next chunk's window rows load under this chunk's MFMAs
      f32x4 acc[4][4];  // [xi2][m]
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        // t = d[rA] + sgn d[rB] per pixel column (the wave's B^T row)
        f32x4 tt[4][2];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x2 lo = pk_fma(f32x2{W[1][c][h].x, W[1][c][h].y}, sgn, f32x2{W[0][c][h].x, W[0][c][h].y});
            const f32x2 hi = pk_fma(f32x2{W[1][c][h].z, W[1][c][h].w}, sgn, f32x2{W[0][c][h].z, W[0][c][h].w});
            tt[c][h] = f32x4{lo.x, lo.y, hi.x, hi.y};
          }
        // the previous group's outputs from the four waves' row sums (read after its barrier Y;
        // acc is not live yet, so Rv costs no MFMA-phase registers)
        if (ch == 0 && tg > 0) phase_b(tg - 1);
        h16x8 bfh[4], bfl[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          if (x == 0) {
            // the B operands of all four xi2: V = the wave's B^T row times B, split (tt dead after)
#pragma unroll
            for (int xx = 0; xx < 4; ++xx) {
              f32x4 v[2];
#pragma unroll
              for (int h = 0; h < 2; ++h)
                v[h] = xx == 0 ? sub4(tt[0][h], tt[2][h]) : xx == 1 ? add4(tt[1][h], tt[2][h])
                     : xx == 2 ? sub4(tt[2][h], tt[1][h]) : sub4(tt[1][h], tt[3][h]);
#if BK_WX_PROBE == 2  // timing probe only (wrong results): no transform / split VALU
              bfh[xx] = __builtin_bit_cast(h16x8, tt[xx][0]);
              bfl[xx] = __builtin_bit_cast(h16x8, tt[xx][1]);
              (void)v;
#else
              split8(v[0], v[1], bfh[xx], bfl[xx]);
#endif
            }
          }
          if (x == 0) {
            // tt is dead: the next chunk's window rows load under this chunk's 48 MFMAs
            if (ch == 0)
              wload(wbase, 1);
            else if (tg + 1 < kWxTG)
              wload(wnext, 0);
          }
          const h16x8 bh = bfh[x], bl = bfl[x];
#if BK_WX_PROBE == 1  // timing probe only (wrong results): no MFMAs
          acc[x][0] += __builtin_bit_cast(f32x4, bh) + __builtin_bit_cast(f32x4, bl);
          continue;
#endif
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            if (ch == 0)
              wx_mfma<true>(acc[x][m], Ua[m][x][0][0], Ua[m][x][0][1], bh, bl);
            else
              wx_mfma<false>(acc[x][m], Ua[m][x][1][0], Ua[m][x][1][1], bh, bl);
          }
        }
        // the last group's U chunk is free once its MFMAs are issued: the next conv's
        if (tg == kWxTG - 1 && !LAST) uload(layer + 1, ch);
      }
      // A^T row sums of this wave's row: R_q[jj] = sum_xi2 M[q][xi2] A[xi2][jj]
      wx_drain(acc);
      f32x4 r0[4], r1[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        r0[m] = add4(add4(acc[0][m], acc[1][m]), acc[2][m]);
        r1[m] = sub4(sub4(acc[1][m], acc[2][m]), acc[3][m]);
      }
      if (layer == 1) WXSTAMP(2 + 3 * tg);
      __syncthreads();  // X: every wave has read this group's windows and the previous R
      if (ystore >= 0) store_y(ystore);
      ystore = -1;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int quad = 4 * m + ks;
        *reinterpret_cast<f32x4*>(rbuf + ((wave * 2 + 0) * 16 + n) * 256 + ((quad ^ (n & 7)) * 16)) = r0[m];
        *reinterpret_cast<f32x4*>(rbuf + ((wave * 2 + 1) * 16 + n) * 256 + ((quad ^ (n & 7)) * 16)) = r1[m];
      }
      if (layer == 1) WXSTAMP(3 + 3 * tg);
      __syncthreads();  // Y: the group's row sums are complete
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 2; ++r)
          Rv[q][r] = *reinterpret_cast<const f32x4*>(rbuf + ((q * 2 + r) * 16 + nb) * 256 + ((cb ^ (nb & 7)) * 16));
      if (layer == 1) WXSTAMP(4 + 3 * tg);
      wbase = wnext;
    }
    phase_b(kWxTG - 1);
    __syncthreads();  // phase B of the last group done everywhere (its windows were read long ago)
    store_y(ystore);
    if (layer == 1) WXSTAMP(30);
    if (!LAST) {
      // the grid complete and the next conv's output bound (A max|x| + B, nets.pack_x3)
      max_in = block_max(mx * ldexpf(1.0f, -ko), red + 4 * (layer & 1), wave, l);
      ex = ex_out;
    } else {
      __syncthreads();  // the tower output is in the grid
    }
  }

  // ---- heads (blokus_nnet.py:146-150, BN folded): the tower output is in the grid; per pixel
  // the two policy and one value 1x1 convs (a quad of channels per lane, summed over 16 lanes)
  float* vfeat = reinterpret_cast<float*>(rbuf);
  float* part = vfeat + NN;
  float* hsum = part + 256;  // [NN][3]
  {
    const f32x4 hw0 = *reinterpret_cast<const f32x4*>(hd.wp + 4 * cb);
    const f32x4 hw1 = *reinterpret_cast<const f32x4*>(hd.wp + 64 + 4 * cb);
    const f32x4 hwv = *reinterpret_cast<const f32x4*>(hd.wv + 4 * cb);
    for (int i = nb; i < NN; i += kLnThreads / 16) {
      const int gr = i / N + 1, gc = i % N + 1;
      const f32x4 v = *reinterpret_cast<const f32x4*>(act + (gr * kWxGR + gc) * 256 + ((cb ^ wx_g(gr, gc)) * 16));
      const float d0 = sum16(v.x * hw0.x + v.y * hw0.y + v.z * hw0.z + v.w * hw0.w);
      const float d1 = sum16(v.x * hw1.x + v.y * hw1.y + v.z * hw1.z + v.w * hw1.w);
      const float dv = sum16(v.x * hwv.x + v.y * hwv.y + v.z * hwv.z + v.w * hwv.w);
      if (cb == 0) {
        hsum[3 * i] = d0;
        hsum[3 * i + 1] = d1;
        hsum[3 * i + 2] = dv;
      }
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
  WXSTAMP(31);
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_leafnet_wx3_weight_bytes() { return kWxLayerBlocks * 1024; }

#if BK_LN_STAMP
// stamps of the diagnostic build: [block][wave][64]: 0 start, 1 tower start, 2 + 3 tg: layer 1's
// group tg: its MFMAs done, R written, y computed; 30 layer 1 done, 31 end
int bk_wx_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wx_stamps), sizeof(g_wx_stamps)) == hipSuccess ? 0 : -1;
}
#endif

int bk_leafnet_wx3_supported(int N) { return N == kWxN; }

int bk_leafnet_wx3(const float* obs, int B, int N, int cin, const void* wstem, const float* sstem, const float* bstem,
                   int nlayers, const void* utower, const float* sutower, const float* btower, const float* bounds,
                   const float* wp, const float* bp, const float* wv, const float* bv, const float* w1t,
                   const float* b1, const float* w2, const float* b2, int P, float* pf, float* vout, float* x0ws,
                   float* out, void* stream) {
  BK_REQUIRE(obs && wstem && sstem && bstem && utower && sutower && btower && bounds && B >= 0, "bad argument");
  BK_REQUIRE(wp && bp && wv && bv && w1t && b1 && w2 && b2 && pf && vout && x0ws && P > 0, "bad argument");
  BK_REQUIRE(cin == kStemCinX3, "bk_leafnet_wx3: the stem takes 8 observation planes");
  BK_REQUIRE(nlayers >= 1, "bk_leafnet_wx3: at least one tower conv");
  BK_REQUIRE(bk_leafnet_wx3_supported(N), "bk_leafnet_wx3: N must be 20");
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  BK_REQUIRE(a16(wstem) && a16(utower) && a16(sstem) && a16(bstem) && a16(sutower) && a16(btower) && a16(wp) &&
                 a16(wv) && a16(x0ws) && a16(out),
             "bk_leafnet_wx3: 16-byte aligned buffers");
  if (B == 0) return BK_OK;
  {
    const void* fns[1] = {(const void*)k_leafnet_wx3};
    if (set_max_dynamic_lds(fns, 1, kWxLds) != BK_OK) return BK_EHIP;
  }
  const LnHeads h{wp, bp, wv, bv, w1t, b1, w2, b2, P, pf, vout};
  hipLaunchKernelGGL(k_leafnet_wx3, dim3(B), dim3(kLnThreads), kWxLds, (hipStream_t)stream, obs,
                     reinterpret_cast<const h16x8*>(wstem), sstem, bstem, reinterpret_cast<const h16x8*>(utower),
                     sutower, btower, bounds, nlayers, h, x0ws, out);
  return launch_check("k_leafnet_wx3");
}

}  // extern "C"
