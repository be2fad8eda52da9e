// trainconv.hip — the learner's 3x3 convolutions 64 -> 64 (models/blokus_nnet.py:103-112, the
// residual tower the reference trains in neural_network.py:52-85) on split-f16 MFMA products:
// the leaf net's "x3" arithmetic (leafnet.hip) as one launch per conv and direction, so that a
// training step's forward (y = conv(x) + b) and its input gradient (dx = conv(dy, w flipped and
// transposed)) leave the fp32 MFMA / MIOpen path for the f16 matrix cores at fp32-class accuracy.
//
// One workgroup per CU walking boards b = blockIdx.x, += gridDim.x (4 waves, wave w = output
// channels 16w..16w+15), each board as k_leafnet_x3's tower layer: the next board's NHWC input is
// loaded into registers under the current board's MFMAs; a board's input is scaled by a power of two so that its
// largest magnitude lies in [2^14, 2^15) (the board maximum: a block reduction), split into f16
// halves and written into the zero-haloed LDS planes of leafnet_common.h; the 18 K-chunks (9 taps
// x 2 halves of 32 input channels) then run the same ring-fed MFMA loop (ln_chunk), and the
// epilogue unscales (the per-output-channel weight scale x 2^-ex), adds the bias and stores NHWC.
// bk_conv_x3_pack splits the weights on the device (one launch per step: no host round trip).
#include "../../include/blokus_engine.h"
#include "ctx.h"

#include "leafnet_common.h"

#ifndef BK_CONV_IL
#define BK_CONV_IL 1  // k_conv_x3: ln_chunk_il (the B-fragment reads between the MFMAs)
#endif

namespace bk {
namespace {

template <int N>
__global__ __launch_bounds__(kLnThreads, 1) void k_conv_x3(const float* __restrict__ x, const h16x8* __restrict__ w,
                                                           const float* __restrict__ inv,
                                                           const float* __restrict__ bias, float* __restrict__ y, int B) {
  constexpr int NN = N * N, RS = ln_row(N), NG = ln_groups(N), PL = ln_plane(N);
  constexpr int QN = NN * 16, QIT = (QN + kLnThreads - 1) / kLnThreads;  // float4 quads of the board
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* act = lds;  // 16 planes [hi q | lo q][(N+2) x RS slots][16 B]
  float* red = reinterpret_cast<float*>(lds + 16 * PL);
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oc = 16 * wave + 4 * ks;

  // a board's input into registers (issued one board ahead: its HBM latency under the MFMAs)
  f32x4 xv[QIT];
  auto load = [&](int b) {
    const f32x4* xb = reinterpret_cast<const f32x4*>(x + (size_t)b * NN * 64);
#pragma unroll
    for (int i = 0; i < QIT; ++i) {
      const int q = tid + i * kLnThreads;
      xv[i] = q < QN ? __builtin_nontemporal_load(xb + q) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  int b = blockIdx.x;
  if (b < B) load(b);
  {  // zero the halo of the 16 planes once (k_leafnet_x3's map): every board writes only interiors
    constexpr int kHaloCols = RS - N, kHalo = 2 * RS + N * kHaloCols;
    for (int i = tid; i < 16 * kHalo; i += kLnThreads) {
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
  const __amdgpu_buffer_rsrc_t wrs = ln_rsrc(w, 18u * 8u * 1024u);
  auto wload = [&](int c, int p) {
    return __builtin_bit_cast(h16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, l * 16, ((c * 8 + wave * 2 + p) * 64) * 16, 0));
  };
  const f32x4 sv = *reinterpret_cast<const f32x4*>(inv + oc);
  const f32x4 bv = bias ? *reinterpret_cast<const f32x4*>(bias + oc) : f32x4{0.f, 0.f, 0.f, 0.f};
  auto coff_of = [&](int c) {
    const int t = c >> 1;
    return 2 * (c & 1) * PL + ((t / 3 - 1) * RS + (t % 3 - 1)) * 16 + kBias;
  };

  for (; b < B; b += gridDim.x) {
    h16x8 wq[kLnWpf + 1][2];
#pragma unroll
    for (int c = 0; c < kLnWpf; ++c) {
      wq[c][0] = wload(c, 0);
      wq[c][1] = wload(c, 1);
    }
    // scale by the board maximum, split, into the planes: quad q of pixel p = channels 4q..4q+3,
    // octet q/2 (hi plane 4 (o % 4) + 2 (o / 4), lo the next), half q % 2 of the octet's 16-B slot
    float m = 0.0f;
#pragma unroll
    for (int i = 0; i < QIT; ++i) m = max3_abs(max3_abs(m, xv[i].x, xv[i].y), xv[i].z, xv[i].w);
    // the barrier in block_max also orders the halo zeroing and the previous board's grid reads
    const float max_in = block_max(m, red + 4 * ((b / gridDim.x) & 1), wave, l);
    const int ex = scale_exp(max_in);
#pragma unroll
    for (int i = 0; i < QIT; ++i) {
      const int q = tid + i * kLnThreads;
      if (q < QN) {
        const int p = q >> 4, qq = q & 15, o = qq >> 1;
        unsigned h0, h1, l0, l1;
        split2(ldexpf(xv[i].x, ex), ldexpf(xv[i].y, ex), h0, l0);
        split2(ldexpf(xv[i].z, ex), ldexpf(xv[i].w, ex), h1, l1);
        unsigned char* d = act + ((o & 3) * 4 + (o >> 2) * 2) * PL + ((p / N + 1) * RS + p % N + 1) * 16 + (qq & 1) * 8;
        *reinterpret_cast<u32x2*>(d) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(d + PL) = u32x2{l0, l1};
      }
    }
    if (b + (int)gridDim.x < B) load(b + gridDim.x);  // the next board, in flight under this one's MFMAs
    __syncthreads();

    // the 18 chunks (tap c/2, channel half c%2), weights kLnWpf chunks ahead
    f32x4 acc[NG];
    h16x8 rb[kLnSlots][2];
    ln_prime<NG, PL>(rb, act, ab, coff_of(0));
#pragma unroll
    for (int c = 0; c < 18; ++c) {
      const int cn = c + kLnWpf, sn = cn % (kLnWpf + 1);
      if (cn < 18) {
        wq[sn][0] = wload(cn, 0);
        wq[sn][1] = wload(cn, 1);
      }
      const h16x8* wc = wq[c % (kLnWpf + 1)];
#if BK_CONV_IL
      // the B-fragment reads between each triple's MFMAs (leafnet_common.h ln_chunk_il)
      if (c == 0)
        ln_chunk_il<NG, true, PL>(acc, wc[0], wc[1], act, ab, coff_of(0), coff_of(1), rb);
      else
        ln_chunk_il<NG, false, PL>(acc, wc[0], wc[1], act, ab, coff_of(c), coff_of(c + 1 < 18 ? c + 1 : c), rb);
#else
      if (c == 0)
        ln_chunk<NG, true, PL>(acc, wc[0], wc[1], act, ab, coff_of(0), coff_of(1), rb);
      else
        ln_chunk<NG, false, PL>(acc, wc[0], wc[1], act, ab, coff_of(c), coff_of(c + 1 < 18 ? c + 1 : c), rb);
#endif
    }
#if BK_CONV_IL
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last chunk's untracked read-ahead
#endif
    ln_mfma_drain(acc);

    // y = acc * inv * 2^-ex + bias, NHWC
    const f32x2 s01{ldexpf(sv.x, -ex), ldexpf(sv.y, -ex)}, s23{ldexpf(sv.z, -ex), ldexpf(sv.w, -ex)};
    const f32x2 b01{bv.x, bv.y}, b23{bv.z, bv.w};
    float* yb = y + (size_t)b * NN * 64;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (is_valid(g)) {
        const f32x2 y01 = pk_fma(f32x2{acc[g][0], acc[g][1]}, s01, b01);
        const f32x2 y23 = pk_fma(f32x2{acc[g][2], acc[g][3]}, s23, b23);
        __builtin_nontemporal_store(f32x4{y01.x, y01.y, y23.x, y23.y},
                                    reinterpret_cast<f32x4*>(yb + ln_pixel<N>(slot_b(g) / 16) * 64 + oc));
      }
    }
  }
}

static_assert(ln_lds_bytes(20) <= 160 * 1024, "k_conv_x3<20>: LDS");

// Weights [64 o][64 c][3][3] f32 (flip: use w[c][o][2-ky][2-kx], the input-gradient conv) -> the
// split A fragments of k_conv_x3: GEMM row o, column k = tap * 64 + c (tap = 3 ky + kx), row scaled
// by 2^e_o (largest |w| of the row in [2^14, 2^15)), hi = f16, lo = f16(x - hi); fragment order
// [chunk 18][wave 4][part 2][k-group 4][row 16][8] (nets.pack_x3's); inv[o] = 2^-e_o.
// One 64-lane workgroup per row o.
__global__ __launch_bounds__(64) void k_conv_x3_pack(const float* __restrict__ wt, int flip,
                                                    _Float16* __restrict__ out, float* __restrict__ inv) {
  const int o = blockIdx.x, l = threadIdx.x;
  float a[9];
  float m = 0.0f;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int k = l + 64 * j, tap = k >> 6, c = k & 63;
    const int ky = tap / 3, kx = tap % 3;
    a[j] = flip ? wt[((c * 64 + o) * 3 + (2 - ky)) * 3 + (2 - kx)] : wt[((o * 64 + c) * 3 + ky) * 3 + kx];
    m = fmaxf(m, fabsf(a[j]));
  }
  m = wave_max_f(m);
  int e = 0;
  if (m > 0.0f && m < __builtin_inff()) {
    int fe;
    (void)frexpf(m, &fe);
    e = 15 - fe;
  }
  const int wv = o >> 4, row = o & 15;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int k = l + 64 * j, chunk = k >> 5, kg = (k >> 3) & 3, el = k & 7;
    const float s = ldexpf(a[j], e);
    const _Float16 hi = (_Float16)s;
    const _Float16 lo = (_Float16)(s - (float)hi);
    const size_t base = ((((size_t)chunk * 4 + wv) * 2) * 4 + kg) * 16 + row;  // part 0
    out[base * 8 + el] = hi;
    out[(base + 4 * 16) * 8 + el] = lo;  // part 1: + one (k-group x row) block of 4 x 16 x 8
  }
  if (l == 0) inv[o] = ldexpf(1.0f, -e);
}

// ---- the weight gradient: dW[o][c][tap] = sum over boards b and pixels p of
// dy[b][p][o] * x[b][p + off(tap)][c] (zero padding), a GEMM of M = 64 (o) x N = 576 (tap, c) over
// K = B x N x N pixels. Each workgroup (8 waves, one per CU) walks its boards (b = blockIdx.x,
// += gridDim.x) in bands of 4 rows; per band the dy rows and the x rows around them (one halo
// row above and below) are scaled, split and stored pixel-major per channel ("transposed": the
// MFMA K is the pixel) in LDS — dy at k = row * 24 + col (cols 20..23 zero), x in a 24-wide
// zero-haloed grid, so tap (dy, dx) of pixel k is x grid element k + 24 dy + dx. The next band's
// global loads are issued into registers before this band's MFMAs (their HBM latency hides
// under the matrix work). Wave w owns input channels 16 (w % 4).. and output channels 32 (w / 4)..
// for all 9 taps (18 accumulator tiles): per K-chunk of 32 pixels it reads 4 A fragments (dy,
// 2 o-blocks, hi/lo) and, per tap row, two aligned B fragments from which dx = 0, 1, 2 are cut
// (dx = 1: v_alignbit, dx = 2: the next dword), then 54 MFMAs. Operand scaling: one power of two
// per workgroup and operand, lowered (and the accumulators rescaled, exactly) whenever a band
// holds larger values. The workgroup's partial sums go to a workspace in fragment order;
// k_conv_x3_wgrad_reduce adds them up in a fixed order.
constexpr int kWgBand = 4;                     // board rows per band (5 bands)
constexpr int kWgThreads = 512, kWgWaves = 8;
constexpr int kWgGrid = 256;                   // workgroups (at most): one per CU
constexpr int kWgDyStride = kWgBand * 24 + 8;  // 104 f16 per (channel, half): 52 dwords (4 x odd: conflict-free reads)
constexpr int kWgXRows = kWgBand + 3;          // x rows y0-1 .. y0+4, + a zero row (fragment overreach)
constexpr int kWgXStride = kWgXRows * 24;      // 168 f16 (84 dwords)
constexpr int kWgDyBytes = 2 * 64 * kWgDyStride * 2;
constexpr int kWgLds = kWgDyBytes + 2 * 64 * kWgXStride * 2 + 128;
constexpr int kWgTiles = 18;                   // (o-block of the wave's pair, tap) tiles per wave
constexpr int kWgDyItems = kWgBand * 12 * 16, kWgXItems = kWgXRows * 12 * 16;
constexpr int kDyIt = (kWgDyItems + kWgThreads - 1) / kWgThreads, kXIt = (kWgXItems + kWgThreads - 1) / kWgThreads;
static_assert(kWgLds <= 160 * 1024, "k_conv_x3_wgrad: LDS");
static_assert(20 % kWgBand == 0 && kWgBand * 24 % 32 == 0, "k_conv_x3_wgrad: whole bands of whole K-chunks");

__device__ __forceinline__ int wg_exp(float m) {  // the scale exponent of a band maximum (1000: no constraint)
  if (!(m > 0.0f)) return 1000;
  return scale_exp(m);
}

__global__ __launch_bounds__(kWgThreads, 1) void k_conv_x3_wgrad(const float* __restrict__ x, const float* __restrict__ dy,
                                                                 int B, f32x4* __restrict__ part) {
  constexpr int N = 20, NN = N * N, kBands = N / kWgBand;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  _Float16* dyt = reinterpret_cast<_Float16*>(lds);               // [half][64 o][kWgDyStride]
  _Float16* xt = reinterpret_cast<_Float16*>(lds + kWgDyBytes);   // [half][64 c][kWgXStride]
  float* red = reinterpret_cast<float*>(lds + kWgLds - 128);      // [parity][dy 8 | x 8] wave maxima
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = wave & 3, oh = wave >> 2;

  f32x4 acc[kWgTiles];
#pragma unroll
  for (int t = 0; t < kWgTiles; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  int E1 = 1000, E2 = 1000;  // the workgroup's operand exponents so far (1000: no data yet)

  const int a_base = (32 * oh + n) * kWgDyStride + 8 * ks;  // A: dy row o = 32 oh + 16 j + n, k-group ks
  const int b_base = (16 * cb + n) * kWgXStride + 8 * ks;   // B: x row c = 16 cb + n
  constexpr int kHalfDy = 64 * kWgDyStride, kHalfX = 64 * kWgXStride;

  const int nboards = B > (int)blockIdx.x ? (B - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nsteps = nboards * kBands;
  // band data in registers: items (row, column pair m, channel quad q); dy pairs m = 0..11 of
  // columns 2m, 2m + 1 (m >= 10: the zero columns 20..23); x rows r = 0..5 (board row y0 - 1 + r,
  // r = 6 the zero row), grid columns 2m, 2m + 1 = board columns 2m - 1, 2m (outside: zero)
  f32x4 dv[kDyIt][2], xv[kXIt][2];
  auto load = [&](int step) {
    const int b = blockIdx.x + (step / kBands) * gridDim.x, y0 = (step % kBands) * kWgBand;
    const f32x4* dyb = reinterpret_cast<const f32x4*>(dy + (size_t)b * NN * 64);
    const f32x4* xb = reinterpret_cast<const f32x4*>(x + (size_t)b * NN * 64);
#pragma unroll
    for (int i = 0; i < kDyIt; ++i) {
      const int it = tid + i * kWgThreads, q = it & 15, m = (it >> 4) % 12, r = (it >> 4) / 12;
      const bool ok = it < kWgDyItems && m < 10;
      const int p = (y0 + r) * N + 2 * m;
      dv[i][0] = ok ? __builtin_nontemporal_load(dyb + p * 16 + q) : f32x4{0.f, 0.f, 0.f, 0.f};
      dv[i][1] = ok ? __builtin_nontemporal_load(dyb + (p + 1) * 16 + q) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < kXIt; ++i) {
      const int it = tid + i * kWgThreads, q = it & 15, m = (it >> 4) % 12, r = (it >> 4) / 12;
      const int yy = y0 - 1 + r, c0 = 2 * m - 1;
      const bool rowok = it < kWgXItems && r <= kWgBand + 1 && yy >= 0 && yy < N;
      const bool ok0 = rowok && c0 >= 0 && c0 < N, ok1 = rowok && c0 + 1 < N;
      xv[i][0] = ok0 ? xb[(yy * N + c0) * 16 + q] : f32x4{0.f, 0.f, 0.f, 0.f};
      xv[i][1] = ok1 ? xb[(yy * N + c0 + 1) * 16 + q] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (nsteps > 0) load(0);

  for (int step = 0; step < nsteps; ++step) {
    const int par = step & 1;
    float my = 0.0f, mxx = 0.0f;
#pragma unroll
    for (int i = 0; i < kDyIt; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) my = max3_abs(max3_abs(my, dv[i][h].x, dv[i][h].y), dv[i][h].z, dv[i][h].w);
#pragma unroll
    for (int i = 0; i < kXIt; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) mxx = max3_abs(max3_abs(mxx, xv[i][h].x, xv[i][h].y), xv[i][h].z, xv[i][h].w);
    my = wave_max_f(my);
    mxx = wave_max_f(mxx);
    if (l == 0) {  // parity-buffered [par][dy 8 | x 8]: a slow wave may still read the last band's
      red[par * 16 + wave] = my;
      red[par * 16 + 8 + wave] = mxx;
    }
    __syncthreads();  // the previous band's MFMAs are done with the LDS; the maxima are visible
    float ry = 0.0f, rx = 0.0f;
#pragma unroll
    for (int w = 0; w < kWgWaves; ++w) {
      ry = fmaxf(ry, red[par * 16 + w]);
      rx = fmaxf(rx, red[par * 16 + 8 + w]);
    }
    const int n1 = min(E1, wg_exp(ry)), n2 = min(E2, wg_exp(rx));
    if (E1 < 1000 && E2 < 1000 && n1 + n2 != E1 + E2) {  // larger values: rescale what is summed so far
      const float f = ldexpf(1.0f, (n1 + n2) - (E1 + E2));
#pragma unroll
      for (int t = 0; t < kWgTiles; ++t) acc[t] = acc[t] * f;
    }
    E1 = n1;
    E2 = n2;
    const int s1 = E1 < 1000 ? E1 : 0, s2 = E2 < 1000 ? E2 : 0;
    // split and store pixel-major: a pair of pixels of one channel = one u32 per half
#pragma unroll
    for (int i = 0; i < kDyIt; ++i) {
      const int it = tid + i * kWgThreads, q = it & 15, m = (it >> 4) % 12, r = (it >> 4) / 12;
      if (it < kWgDyItems) {
        const float a0[4] = {dv[i][0].x, dv[i][0].y, dv[i][0].z, dv[i][0].w};
        const float a1[4] = {dv[i][1].x, dv[i][1].y, dv[i][1].z, dv[i][1].w};
        const int k = r * 24 + 2 * m;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned h, o;
          split2(ldexpf(a0[j], s1), ldexpf(a1[j], s1), h, o);
          const int ch = 4 * q + j;
          *reinterpret_cast<unsigned*>(dyt + ch * kWgDyStride + k) = h;
          *reinterpret_cast<unsigned*>(dyt + kHalfDy + ch * kWgDyStride + k) = o;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kXIt; ++i) {
      const int it = tid + i * kWgThreads, q = it & 15, m = (it >> 4) % 12, r = (it >> 4) / 12;
      if (it < kWgXItems) {
        const float a0[4] = {xv[i][0].x, xv[i][0].y, xv[i][0].z, xv[i][0].w};
        const float a1[4] = {xv[i][1].x, xv[i][1].y, xv[i][1].z, xv[i][1].w};
        const int k = r * 24 + 2 * m;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned h, o;
          split2(ldexpf(a0[j], s2), ldexpf(a1[j], s2), h, o);
          const int ch = 4 * q + j;
          *reinterpret_cast<unsigned*>(xt + ch * kWgXStride + k) = h;
          *reinterpret_cast<unsigned*>(xt + kHalfX + ch * kWgXStride + k) = o;
        }
      }
    }
    if (step + 1 < nsteps) load(step + 1);  // the next band's loads, in flight under the MFMAs
    __syncthreads();
    // the band's 3 K-chunks of 32 pixels
#pragma unroll
    for (int kc = 0; kc < kWgBand * 24 / 32; ++kc) {
      const int k0 = 32 * kc;
      h16x8 ah[2], al[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        ah[j] = *reinterpret_cast<const h16x8*>(dyt + a_base + 16 * j * kWgDyStride + k0);
        al[j] = *reinterpret_cast<const h16x8*>(dyt + kHalfDy + a_base + 16 * j * kWgDyStride + k0);
      }
#pragma unroll
      for (int dr = 0; dr < 3; ++dr) {
        const int off = b_base + k0 + 24 * dr;
        const u32x4 h0 = *reinterpret_cast<const u32x4*>(xt + off), h1 = *reinterpret_cast<const u32x4*>(xt + off + 8);
        const u32x4 o0 = *reinterpret_cast<const u32x4*>(xt + kHalfX + off);
        const u32x4 o1 = *reinterpret_cast<const u32x4*>(xt + kHalfX + off + 8);
        h16x8 bh[3], bl[3];
        bh[0] = __builtin_bit_cast(h16x8, h0);
        bl[0] = __builtin_bit_cast(h16x8, o0);
        bh[1] = __builtin_bit_cast(h16x8, u32x4{__builtin_amdgcn_alignbit(h0.y, h0.x, 16), __builtin_amdgcn_alignbit(h0.z, h0.y, 16),
                                                __builtin_amdgcn_alignbit(h0.w, h0.z, 16), __builtin_amdgcn_alignbit(h1.x, h0.w, 16)});
        bl[1] = __builtin_bit_cast(h16x8, u32x4{__builtin_amdgcn_alignbit(o0.y, o0.x, 16), __builtin_amdgcn_alignbit(o0.z, o0.y, 16),
                                                __builtin_amdgcn_alignbit(o0.w, o0.z, 16), __builtin_amdgcn_alignbit(o1.x, o0.w, 16)});
        bh[2] = __builtin_bit_cast(h16x8, u32x4{h0.y, h0.z, h0.w, h1.x});
        bl[2] = __builtin_bit_cast(h16x8, u32x4{o0.y, o0.z, o0.w, o1.x});
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int dc = 0; dc < 3; ++dc) {
            f32x4& c = acc[j * 9 + dr * 3 + dc];
            asm volatile(
                "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
                "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
                "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
                : "+a"(c)
                : "v"(ah[j]), "v"(bh[dc]), "v"(al[j]), "v"(bl[dc]));
          }
      }
    }
    ln_mfma_drain(acc);
  }
  // the partial sums, unscaled, in fragment order: part[block][wave][tile][lane]
  const float u = (E1 < 1000 && E2 < 1000) ? ldexpf(1.0f, -(E1 + E2)) : 0.0f;
  f32x4* pb = part + ((size_t)blockIdx.x * kWgWaves + wave) * kWgTiles * 64 + l;
#pragma unroll
  for (int t = 0; t < kWgTiles; ++t) pb[t * 64] = acc[t] * u;
}

// dW[o][c][ky][kx] (PyTorch's layout) = the sum over the G workgroups' partials; one thread per
// (wave, tile, lane, element): 8 independent running sums (g mod 8) combined at the end (a
// fixed order: deterministic)
constexpr int kWgPer = kWgWaves * kWgTiles * 64 * 4;  // floats per workgroup partial (36864)
__global__ __launch_bounds__(256) void k_conv_x3_wgrad_reduce(const float* __restrict__ part, int G, float* __restrict__ dw) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= kWgPer) return;
  const int i = e & 3, l = (e >> 2) & 63, t = (e >> 8) % kWgTiles, w = (e >> 8) / kWgTiles;
  const int o = 32 * (w >> 2) + 16 * (t / 9) + 4 * (l >> 4) + i, c = 16 * (w & 3) + (l & 15), tap = t % 9;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int g = 0;
  for (; g + 8 <= G; g += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += part[(size_t)(g + j) * kWgPer + e];
  }
  for (int j = 0; g < G; ++g, ++j) s[j] += part[(size_t)g * kWgPer + e];
  dw[(o * 64 + c) * 9 + tap] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_conv_x3_wgrad_workspace_floats(int B) {
  const int G = B < kWgGrid ? (B > 0 ? B : 1) : kWgGrid;
  return G * kWgPer;
}

int bk_conv_x3_wgrad(const float* x, const float* dy, int B, int N, float* workspace, float* dw, void* stream) {
  BK_REQUIRE(dw && B >= 0 && (B == 0 || (x && dy && workspace)), "bad argument");
  BK_REQUIRE(N == 20, "bk_conv_x3_wgrad: 20x20 boards");
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  BK_REQUIRE(a16(x) && a16(dy) && a16(workspace), "bk_conv_x3_wgrad: 16-byte aligned buffers");
  hipStream_t s = (hipStream_t)stream;
  const int G = B < kWgGrid ? (B > 0 ? B : 1) : kWgGrid;
  if (B == 0) return hipMemsetAsync(dw, 0, 64 * 64 * 9 * sizeof(float), s) == hipSuccess ? BK_OK : BK_EHIP;
  {
    const void* fns[1] = {(const void*)k_conv_x3_wgrad};
    if (set_max_dynamic_lds(fns, 1, kWgLds) != BK_OK) return BK_EHIP;
  }
  hipLaunchKernelGGL(k_conv_x3_wgrad, dim3(G), dim3(kWgThreads), kWgLds, s, x, dy, B, (f32x4*)workspace);
  if (launch_check("k_conv_x3_wgrad") != BK_OK) return BK_EHIP;
  hipLaunchKernelGGL(k_conv_x3_wgrad_reduce, dim3((kWgPer + 255) / 256), dim3(256), 0, s, workspace, G, dw);
  return launch_check("k_conv_x3_wgrad_reduce");
}

int bk_conv_x3_weight_bytes(void) { return 18 * 4 * 2 * kBlock * 2; }

int bk_conv_x3_pack(const float* w, int flip, void* wsplit, float* inv, void* stream) {
  BK_REQUIRE(w && wsplit && inv, "bad argument");
  BK_REQUIRE(((uintptr_t)wsplit & 15u) == 0 && ((uintptr_t)inv & 15u) == 0, "bk_conv_x3_pack: 16-byte aligned outputs");
  hipLaunchKernelGGL(k_conv_x3_pack, dim3(64), dim3(64), 0, (hipStream_t)stream, w, flip, (_Float16*)wsplit, inv);
  return launch_check("k_conv_x3_pack");
}

int bk_conv_x3(const float* x, int B, int N, const void* wsplit, const float* inv, const float* bias, float* y,
               void* stream) {
  BK_REQUIRE(x && wsplit && inv && y && B >= 0, "bad argument");
  BK_REQUIRE(N == 20, "bk_conv_x3: 20x20 boards");
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  BK_REQUIRE(a16(x) && a16(wsplit) && a16(inv) && a16(y) && (!bias || a16(bias)), "bk_conv_x3: 16-byte aligned buffers");
  if (B == 0) return BK_OK;
  {
    const void* fns[1] = {(const void*)k_conv_x3<20>};
    if (set_max_dynamic_lds(fns, 1, ln_lds_bytes(20)) != BK_OK) return BK_EHIP;
  }
  const int G = B < 256 ? B : 256;  // persistent: one workgroup per CU, boards strided
  hipLaunchKernelGGL(k_conv_x3<20>, dim3(G), dim3(kLnThreads), ln_lds_bytes(20), (hipStream_t)stream, x,
                     (const h16x8*)wsplit, inv, bias, y, B);
  return launch_check("k_conv_x3");
}

}  // extern "C"
