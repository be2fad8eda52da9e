// trainconv.hip — the learner's 3x3 convolutions 64 -> 64 (models/blokus_nnet.py:103-112, the
// residual tower the reference trains in neural_network.py:52-85) on split-f16 MFMA products:
// the leaf net's "x3" arithmetic (leafnet.hip) as one launch per conv and direction, so that a
// training step's forward (y = conv(x) + b) and its input gradient (dx = conv(dy, w flipped and
// transposed)) leave the fp32 MFMA / MIOpen path for the f16 matrix cores at fp32-class accuracy.
//
// One workgroup per board (4 waves, wave w = output channels 16w..16w+15), as k_leafnet_x3's
// tower layer: the board's NHWC input comes from HBM, is scaled by a power of two so that its
// largest magnitude lies in [2^14, 2^15) (the board maximum: a block reduction), split into f16
// halves and written into the zero-haloed LDS planes of leafnet_common.h; the 18 K-chunks (9 taps
// x 2 halves of 32 input channels) then run the same ring-fed MFMA loop (ln_chunk), and the
// epilogue unscales (the per-output-channel weight scale x 2^-ex), adds the bias and stores NHWC.
// bk_conv_x3_pack splits the weights on the device (one launch per step: no host round trip).
#include "../../include/blokus_engine.h"
#include "ctx.h"

#include "leafnet_common.h"

namespace bk {
namespace {

template <int N>
__global__ __launch_bounds__(kLnThreads, 1) void k_conv_x3(const float* __restrict__ x, const h16x8* __restrict__ w,
                                                           const float* __restrict__ inv,
                                                           const float* __restrict__ bias, float* __restrict__ y) {
  constexpr int NN = N * N, RS = ln_row(N), NG = ln_groups(N), PL = ln_plane(N);
  constexpr int QN = NN * 16, QIT = (QN + kLnThreads - 1) / kLnThreads;  // float4 quads of the board
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* act = lds;  // 16 planes [hi q | lo q][(N+2) x RS slots][16 B]
  float* red = reinterpret_cast<float*>(lds + 16 * PL);
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oc = 16 * wave + 4 * ks;
  const size_t b = blockIdx.x;

  // the board's input first (its HBM latency under the halo zeroing and the weight loads)
  const f32x4* xb = reinterpret_cast<const f32x4*>(x + b * NN * 64);
  f32x4 xv[QIT];
#pragma unroll
  for (int i = 0; i < QIT; ++i) {
    const int q = tid + i * kLnThreads;
    xv[i] = q < QN ? __builtin_nontemporal_load(xb + q) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  {  // zero the halo of the 16 planes (k_leafnet_x3's map)
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
  h16x8 wq[kLnWpf + 1][2];
#pragma unroll
  for (int c = 0; c < kLnWpf; ++c) {
    wq[c][0] = wload(c, 0);
    wq[c][1] = wload(c, 1);
  }
  const f32x4 sv = *reinterpret_cast<const f32x4*>(inv + oc);
  const f32x4 bv = bias ? *reinterpret_cast<const f32x4*>(bias + oc) : f32x4{0.f, 0.f, 0.f, 0.f};

  // scale by the board maximum, split, into the planes: quad q of pixel p = channels 4q..4q+3,
  // octet q/2 (hi plane 4 (o % 4) + 2 (o / 4), lo the next), half q % 2 of the octet's 16-B slot
  float m = 0.0f;
#pragma unroll
  for (int i = 0; i < QIT; ++i) m = max3_abs(max3_abs(m, xv[i].x, xv[i].y), xv[i].z, xv[i].w);
  const float max_in = block_max(m, red, wave, l);  // the barrier also orders the halo zeroing
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
  __syncthreads();

  // the 18 chunks (tap c/2, channel half c%2), weights kLnWpf chunks ahead
  f32x4 acc[NG];
  h16x8 rb[kLnSlots][2];
  auto coff_of = [&](int c) {
    const int t = c >> 1;
    return 2 * (c & 1) * PL + ((t / 3 - 1) * RS + (t % 3 - 1)) * 16 + kBias;
  };
  ln_prime<NG, PL>(rb, act, ab, coff_of(0));
#pragma unroll
  for (int c = 0; c < 18; ++c) {
    const int cn = c + kLnWpf, sn = cn % (kLnWpf + 1);
    if (cn < 18) {
      wq[sn][0] = wload(cn, 0);
      wq[sn][1] = wload(cn, 1);
    }
    const h16x8* wc = wq[c % (kLnWpf + 1)];
    if (c == 0)
      ln_chunk<NG, true, PL>(acc, wc[0], wc[1], act, ab, coff_of(0), coff_of(1), rb);
    else
      ln_chunk<NG, false, PL>(acc, wc[0], wc[1], act, ab, coff_of(c), coff_of(c + 1 < 18 ? c + 1 : c), rb);
  }
  ln_mfma_drain(acc);

  // y = acc * inv * 2^-ex + bias, NHWC
  const f32x2 s01{ldexpf(sv.x, -ex), ldexpf(sv.y, -ex)}, s23{ldexpf(sv.z, -ex), ldexpf(sv.w, -ex)};
  const f32x2 b01{bv.x, bv.y}, b23{bv.z, bv.w};
  float* yb = y + b * NN * 64;
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

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

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
  hipLaunchKernelGGL(k_conv_x3<20>, dim3(B), dim3(kLnThreads), ln_lds_bytes(20), (hipStream_t)stream, x,
                     (const h16x8*)wsplit, inv, bias, y);
  return launch_check("k_conv_x3");
}

}  // extern "C"
