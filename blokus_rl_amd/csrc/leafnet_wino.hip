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
// Decomposition (one workgroup of 4 waves per board, one wave per SIMD): wave w owns output
// channels 16w..16w+15 and holds their U — 16 positions x 64 input channels x (hi, lo) — in 256
// AGPRs for the whole layer (the A operands, read by the MFMAs straight from AGPRs). The 100
// tiles form 7 groups of 16 (the MFMA columns; the last group has 4 spare columns). The
// transform domain of a group is produced a quarter at a time (xi1 = 1, 2, 0, 3: one B^T row
// each) into one of two 16 KB LDS buffers by all 256 threads (thread = one tile x 4 channels),
// while the waves' MFMAs consume the other buffer: per (group, quarter) slot one barrier. The
// accumulators of a quarter are final after its slot; its part of the output transform (A^T row
// sums) runs three slots later under other MFMAs, and a group's outputs go back into the
// activation grid once every window of the next group has been read (the grid is updated in
// place). The stem (8 -> 64) stays the direct x3 conv of leafnet_common.h; the stem output x0
// waits in a global workspace for the tower's final residual; the heads run as in leafnet.hip.
#include "leafnet_common.h"

namespace bk {
namespace {

constexpr int kWxN = 20;                            // the 20x20 preset
constexpr int kWxNN = kWxN * kWxN;
constexpr int kWxT = kWxN / 2;                      // tiles per row
constexpr int kWxTiles = kWxT * kWxT;               // 100 output tiles of 2x2 pixels
constexpr int kWxTG = (kWxTiles + 15) / 16;         // 7 tile groups of 16
constexpr int kWxGR = kWxN + 2;                     // activation grid: 1-pixel zero halo
constexpr int kWxActBytes = kWxGR * kWxGR * 256;    // [22][22] pixels x 64 channels fp32
constexpr int kWxVBytes = 16384;                    // one quarter: [4 xi2][hi, lo][16 tiles][64 ch] f16
constexpr int kWxVOff = kWxActBytes;
constexpr int kWxRedOff = kWxActBytes + 2 * kWxVBytes;
constexpr int kWxLds = kWxRedOff + 64;
constexpr int kWxLayerBlocks = 256;                 // (xi1, xi2, chunk, wave, half) blocks of 1 KB per conv
static_assert(kWxLds <= 160 * 1024, "k_leafnet_wx3: LDS");
static_assert(2 * ln_plane(kWxN) <= 2 * kWxVBytes, "k_leafnet_wx3: the stem input planes live in the V buffers");

// xi1 of the four quarters of a tile group, in slot order: 1 and 2 need window rows 1, 2; then 0
// (rows 0, 2) and 3 (rows 1, 3)
__host__ __device__ constexpr int wx_q(int qi) { return qi == 0 ? 1 : qi == 1 ? 2 : qi == 2 ? 0 : 3; }

// activation grid: pixel (gr, gc) at (gr * 22 + gc) * 256, its 16-B channel quad s at slot
// s ^ wx_sw(gr, gc): the epilogue's 8-lane store groups (8 tiles, one quad) spread over the
// banks; the window reads (16 lanes = one pixel's 16 quads) stay conflict-free
__device__ __forceinline__ int wx_sw(int gr, int gc) { return (((gr + 1) >> 1) * 2 + ((gc + 1) >> 1)) & 3; }
// V buffer: tile row n (128 B = 64 channels f16) holds its 16-B channel octet o at slot o ^ wx_vf(n)
// (the MFMA B-operand reads of a ds_read_b128 lane group hit 16 distinct bank groups)
__device__ __forceinline__ int wx_vf(int n) { return (n >> 1) & 7; }

// one MFMA step: acc (+)= ah*bh + al*bh + ah*bl. BK_WX_ASM=1: inline asm with the A operands
// from AGPRs and a 2-state pad for operands the compiler has just copied in; 0 (default): the
// builtin (the compiler allocates, pads and schedules)
#ifndef BK_WX_ASM
#define BK_WX_ASM 0
#endif
template <bool INIT>
__device__ __forceinline__ void wx_mfma(f32x4& acc, const h16x8& ah, const h16x8& al, const h16x8& bh,
                                        const h16x8& bl) {
#if BK_WX_ASM
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
#else
  f32x4 c = INIT ? f32x4{0.f, 0.f, 0.f, 0.f} : acc;
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
#endif
}

__device__ __forceinline__ f32x4 relu4(f32x4 y) {
  return f32x4{max_bits(y.x, 0), max_bits(y.y, 0), max_bits(y.z, 0), max_bits(y.w, 0)};
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
  unsigned char* vb = lds + kWxVOff;
  unsigned char* sin = vb;  // the stem's input planes (hi, lo), before the tower uses the V buffers
  float* red = reinterpret_cast<float*>(lds + kWxRedOff);
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oc = 16 * wave + 4 * ks;
  const size_t b = blockIdx.x;

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
  // and, scaled by 2^ex so that the first conv's V fits f16 (|V| <= 4 max|d|), the grid
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
        *reinterpret_cast<f32x4*>(act + (gr * kWxGR + gc) * 256 + (((4 * wave + ks) ^ wx_sw(gr, gc)) * 16)) = y * up;
      }
    }
    max_in = block_max(mx, red, wave, l);  // the barrier also completes the grid
  }

  // ---- the residual tower
  // U of one conv: [xi1 4][xi2 4][chunk 2][wave 4][half 2][lane 64][8 f16]; wave `wave` reads its
  // quarter q as 16 blocks (xi2, chunk, half) of 16 B per lane
  const __amdgpu_buffer_rsrc_t urs = ln_rsrc(ut, (unsigned)nlayers * kWxLayerBlocks * 1024u);
  auto uload = [&](int layer, int q, h16x8 (&dst)[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int xi2 = i >> 2, ch = (i >> 1) & 1, h = i & 1;
      const int blk = (((q * 4 + xi2) * 2 + ch) * 4 + wave) * 2 + h;
      dst[i] = __builtin_bit_cast(h16x8, __builtin_amdgcn_raw_buffer_load_b128(urs, l * 16,
                                                                               (layer * kWxLayerBlocks + blk) * 1024, 0));
    }
  };
  h16x8 Ua[4][16];
#pragma unroll
  for (int q = 0; q < 4; ++q) uload(0, q, Ua[q]);

  // the transform thread: tile nt of the group, channel quad c4
  const int nt = tid >> 4, c4 = tid & 15;
  // V write base (a quarter buffer's tile row nt, quad c4) and the lane's B-read bases (chunk 0, 1)
  const int vw = kWxVOff + nt * 128 + (((c4 >> 1) ^ wx_vf(nt)) * 16) + (c4 & 1) * 8;
  const int vr0 = kWxVOff + n * 128 + ((ks ^ wx_vf(n)) * 16);
  const int vr1 = kWxVOff + n * 128 + (((4 + ks) ^ wx_vf(n)) * 16);

  for (int layer = 0; layer < nlayers; ++layer) {
    const bool last = layer + 1 == nlayers, more = !last;
    const bool relu = !(layer & 1) || last;
    const f32x4 suv = *reinterpret_cast<const f32x4*>(su + layer * 64 + oc);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bt + layer * 64 + oc);
    const int ex_out = scale_exp(4.0f * (bounds[2 * (layer + 1)] * max_in + bounds[2 * (layer + 1) + 1]));
    const int ko = last ? 0 : ex_out;
    const f32x4 sc{ldexpf(suv.x, ko - ex), ldexpf(suv.y, ko - ex), ldexpf(suv.z, ko - ex), ldexpf(suv.w, ko - ex)};
    const f32x4 bc{ldexpf(bv.x, ko), ldexpf(bv.y, ko), ldexpf(bv.z, ko), ldexpf(bv.w, ko)};
    const float down = ldexpf(1.0f, -ko);  // the lane maximum back to the unscaled output
    float mx = 0.0f;

    // the transform thread's window bases for tile group tg (spare tiles read tile 0's window)
    int pb[4];
    auto set_tile = [&](int tg) {
      int t = 16 * tg + nt;
      t = t < kWxTiles ? t : 0;
      const int ti = t / kWxT, tj = t - ti * kWxT;
      const int base = (2 * ti * kWxGR + 2 * tj) * 256, s0 = 2 * ti + tj;
#pragma unroll
      for (int k = 0; k < 4; ++k) pb[k] = base + ((c4 ^ ((s0 + k) & 3)) * 16);
    };
    // window row r of the current tile: 4 pixels x 4 channels
    auto load_row = [&](f32x4 (&R)[4], int r) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = 2 * ((r + 1) >> 1) + ((c + 1) >> 1);
        R[c] = *reinterpret_cast<const f32x4*>(act + pb[k & 3] + (r * kWxGR + c) * 256);
      }
    };
    f32x4 Ra[4], Rb[4];
    // quarter xi1 = q of the current tile's transform -> V buffer `buf` (Ra, Rb hold the rows)
    auto transform = [&](int q, int buf) {
      f32x4 t[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) t[c] = q == 1 ? Ra[c] + Rb[c] : q == 2 ? Rb[c] - Ra[c] : Ra[c] - Rb[c];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = j == 0 ? t[0] - t[2] : j == 1 ? t[1] + t[2] : j == 2 ? t[2] - t[1] : t[1] - t[3];
        unsigned h0, l0, h1, l1;
        split2(v.x, v.y, h0, l0);
        split2(v.z, v.w, h1, l1);
        unsigned char* dst = lds + vw + buf * kWxVBytes + j * 4096;
        *reinterpret_cast<u32x2*>(dst) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(dst + 2048) = u32x2{l0, l1};
      }
    };

    f32x4 acc[4][4];
    f32x4 y[2][2];
    // the output transform's A^T row sums of quarter q (final accumulators) into y
    auto partial = [&](int q) {
      f32x4 r0, r1;
      r0 = acc[q][0] + acc[q][1] + acc[q][2];
      r1 = acc[q][1] - acc[q][2] - acc[q][3];
      if (q == 1) {
        y[0][0] = r0;
        y[0][1] = r1;
        y[1][0] = r0;
        y[1][1] = r1;
      } else if (q == 2) {
        y[0][0] += r0;
        y[0][1] += r1;
        y[1][0] -= r0;
        y[1][1] -= r1;
      } else if (q == 0) {
        y[0][0] += r0;
        y[0][1] += r1;
      } else {
        y[1][0] -= r0;
        y[1][1] -= r1;
      }
    };
    // group tg's outputs (complete in y): scale, bias, (x0,) ReLU -> the grid (scaled by
    // 2^ex_out) or, after the last conv, the heads' per-pixel partial dot products
    auto finish = [&](int tg) {
      const int t = 16 * tg + n;
      if (t >= kWxTiles) return;
      const int ti = t / kWxT, tj = t - ti * kWxT;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int gr = 2 * ti + 1 + ii, gc = 2 * tj + 1 + jj, px = (gr - 1) * N + gc - 1;
          f32x4 v = y[ii][jj] * sc + bc;
          if (last) v += *reinterpret_cast<const f32x4*>(x0ws + (b * NN + px) * 64 + oc);
          if (relu) v = relu4(v);
          mx = max3_abs(max3_abs(mx, v.x, v.y), v.z, v.w);
          y[ii][jj] = v;
          if (!last) {
            *reinterpret_cast<f32x4*>(act + (gr * kWxGR + gc) * 256 + (((4 * wave + ks) ^ wx_sw(gr, gc)) * 16)) = v;
          } else if (xout) {
            *reinterpret_cast<f32x4*>(xout + (b * NN + px) * 64 + oc) = v;
          }
        }
      if (last) {
        // the heads' 1x1 convs: per pixel the dot products over this wave's 16 channels
        const f32x4 wp0 = *reinterpret_cast<const f32x4*>(hd.wp + oc);
        const f32x4 wp1 = *reinterpret_cast<const f32x4*>(hd.wp + 64 + oc);
        const f32x4 wvv = *reinterpret_cast<const f32x4*>(hd.wv + oc);
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const f32x4 v = y[ii][jj];
            float d[3];
            const f32x4* w[3] = {&wp0, &wp1, &wvv};
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              const float a = v.x * (*w[k]).x + v.y * (*w[k]).y + v.z * (*w[k]).z + v.w * (*w[k]).w;
              const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
              const float a16 = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
              const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a16), __float_as_uint(a16), false, false);
              d[k] = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
            }
            if (ks == 0) {
              // into the grid pixel itself (its input values are no longer read): wave w's 3 floats
              const int gr = 2 * ti + 1 + ii, gc = 2 * tj + 1 + jj;
              float* dst = reinterpret_cast<float*>(act + (gr * kWxGR + gc) * 256 + wave * 16);
              dst[0] = d[0];
              dst[1] = d[1];
              dst[2] = d[2];
            }
          }
      }
    };

    // the B fragments of one MFMA step (xi2, chunk) of the quarter in buffer `buf`
    auto bload = [&](h16x8 (&r)[2], int buf, int xi2, int ch) {
      const int base = (ch ? vr1 : vr0) + buf * kWxVBytes + xi2 * 4096;
      r[0] = *reinterpret_cast<const h16x8*>(lds + base);
      r[1] = *reinterpret_cast<const h16x8*>(lds + base + 2048);
    };

    // prologue: group 0's first quarter
    set_tile(0);
    load_row(Ra, 1);
    load_row(Rb, 2);
    transform(wx_q(0), 0);
    __syncthreads();

    for (int tg = 0; tg < kWxTG; ++tg) {
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        const int q = wx_q(qi), buf = qi & 1;
        if (tg > 0 || qi > 0) __syncthreads();
        // the previous group's outputs go out once every window of this group has been read
        if (qi == 3 && tg > 0) finish(tg - 1);
        // the next conv's U quarter (registers free since the previous slot's MFMAs)
        if (tg == kWxTG - 1 && qi > 0 && more) {
          asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
          uload(layer + 1, wx_q(qi - 1), Ua[wx_q(qi - 1)]);
        }
        h16x8 bf[2][2];
        bload(bf[0], buf, 0, 0);
        // the next slot's window rows
        const bool tnext = qi < 3 || tg + 1 < kWxTG;
        if (tnext) {
          if (qi == 1) load_row(Ra, 0);
          if (qi == 2) {
            load_row(Ra, 1);
            load_row(Rb, 3);
          }
          if (qi == 3) {
            set_tile(tg + 1);
            load_row(Ra, 1);
            load_row(Rb, 2);
          }
        }
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const int xi2 = st >> 1, ch = st & 1;
          if (st + 1 < 8) bload(bf[(st + 1) & 1], buf, (st + 1) >> 1, (st + 1) & 1);
          const h16x8* u = &Ua[q][(xi2 * 2 + ch) * 2];
          if (ch == 0)
            wx_mfma<true>(acc[q][xi2], u[0], u[1], bf[st & 1][0], bf[st & 1][1]);
          else
            wx_mfma<false>(acc[q][xi2], u[0], u[1], bf[st & 1][0], bf[st & 1][1]);
          if (st == 1) {
            // three slots back: that quarter's accumulators are final (48 MFMAs since)
            const int qp = wx_q((qi + 1) & 3);
            if (tg > 0 || qi == 3) {
#if BK_WX_ASM
#pragma unroll
              for (int x = 0; x < 4; ++x) asm volatile("" : "+v"(acc[qp][x]));
#endif
              partial(qp);
            }
          }
          if (st == 3 && tnext) transform(wx_q((qi + 1) & 3), buf ^ 1);
        }
      }
    }
    // tail: the last group's quarters 1..3 (slots 25..27), its outputs, the next conv's last U quarter
#if BK_WX_ASM
    // the MFMA writes of the last slots -> VALU reads (hipcc does not see the asm MFMAs' latency)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int x = 0; x < 4; ++x) asm volatile("" : "+v"(acc[q][x]));
#endif
    partial(wx_q(1));
    partial(wx_q(2));
    partial(wx_q(3));
    finish(kWxTG - 1);
    if (more) uload(layer + 1, wx_q(3), Ua[wx_q(3)]);
    if (more) {
      max_in = block_max(mx * down, red + 4 * (layer & 1), wave, l);  // completes the grid too
      ex = ex_out;
    } else {
      __syncthreads();  // the heads' partial sums are in the grid
    }
  }

  // ---- heads (blokus_nnet.py:146-150, BN folded): per pixel the 4 waves' partial sums
  float* vfeat = reinterpret_cast<float*>(vb);
  float* part = vfeat + NN;
  for (int i = tid; i < NN; i += kLnThreads) {
    const int gr = i / N + 1, gc = i % N + 1;
    const float* q = reinterpret_cast<const float*>(act + (gr * kWxGR + gc) * 256);
    const float p0 = ((q[0] + q[4]) + q[8]) + q[12], p1 = ((q[1] + q[5]) + q[9]) + q[13],
                pv = ((q[2] + q[6]) + q[10]) + q[14];
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

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_leafnet_wx3_weight_bytes() { return kWxLayerBlocks * 1024; }

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
