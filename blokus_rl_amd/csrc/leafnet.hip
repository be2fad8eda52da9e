// leafnet.hip — the leaf ResNet (models/blokus_nnet.py:88-151, eval-mode BN folded) of one board
// per workgroup, on the f16 matrix cores with fp32-class accuracy ("x3" = three f16 products).
//
// Why: the f32 MFMA (v_mfma_f32_16x16x4_f32) runs at 1/16 of the f16 rate on gfx950 and does not
// overlap the VALU, so the round-1 tower (Winograd on f32 MFMA, conv.hip) was bound at ~57% of a
// low peak. Here every operand x (weights and activations, fp32) is split into two f16 halves
// x = hi + lo (hi = f16(x), lo = f16(x - hi): 22 significant bits) and each product is taken as
// hi*hi + lo*hi + hi*lo on v_mfma_f32_16x16x32_f16 (exact f16 products, f32 accumulation); the
// dropped lo*lo term is below 2^-22 of the product. To keep both halves normal f16 numbers, the
// operands are scaled by powers of two first: the weights per output channel on the host (largest
// |w| in [2^14, 2^15)), the activations per board and layer on the device (the largest |x| of the
// board's layer input in [2^14, 2^15)); the accumulator is unscaled exactly by the inverse powers.
// Measured error against an fp64 forward: tests/test_leafnet_gpu.py (same order as the fp32 kernel).
//
// Convolutions are direct (implicit GEMM): M = 16 output channels per wave (4 waves = 64), N = 16
// pixels per group (NG = ceil(N*N/16) groups cover the board), K = 9 taps x Cin in chunks of 32
// (tap t = c/2, channel half c%2 for Cin = 64; taps 4c..4c+3 x 8 channels for the stem). The
// board's layer input lives in LDS as a zero-haloed (N+2)^2 pixel grid of split halves
// (kPixBytes per pixel: hi[64] | lo[64] | pad): the B fragment of lane l is one ds_read_b128 per
// half at pixel (16g + l%16) shifted by the tap, channels 8(l/16).. of the chunk. The A fragments
// (weights) stream from global memory (L2-resident across the 32 boards of an XCD), one chunk
// ahead. The accumulators of all NG groups stay in registers for the layer; the epilogue applies
// scale, bias, (residual), ReLU, finds the board maximum, splits and writes the next layer input
// in place. The stem output x0 stays in registers for the tower's final residual, and the last
// layer's epilogue feeds the heads' 1x1 convs straight from the registers.
#include "../../include/blokus_engine.h"
#include "ctx.h"

namespace bk {
namespace {

using h16x8 = _Float16 __attribute__((ext_vector_type(8)));
using h16x2 = _Float16 __attribute__((ext_vector_type(2)));
using f32x4 = float __attribute__((ext_vector_type(4)));
using f32x2 = float __attribute__((ext_vector_type(2)));
using u32x4 = unsigned __attribute__((ext_vector_type(4)));
using u32x2 = unsigned __attribute__((ext_vector_type(2)));

constexpr int kLnThreads = 256;
constexpr int kPixBytes = 272;     // hi[64] f16 | lo[64] f16 | 16 B (pixel stride = 17 x 16 B: spreads banks)
constexpr int kStemPixBytes = 32;  // hi[8] f16 | lo[8] f16
constexpr int kStemCinX3 = 8;
constexpr int kBlock = 64 * 8;     // f16 per (chunk, wave, part) block of packed weights: 64 lanes x 8

__host__ __device__ constexpr int ln_chunks(int cin) { return cin == 64 ? 18 : 3; }

// LDS bytes of k_leafnet_x3<N>: the activation grid, the stem's input grid, 4 wave maxima
__host__ __device__ constexpr int ln_lds_bytes(int N) { return (N + 2) * (N + 2) * (kPixBytes + kStemPixBytes) + 64; }

__device__ __forceinline__ f32x4 mfma16(h16x8 a, h16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// x (already scaled) -> packed f16 halves: hi = f16(x) (round to nearest), lo = f16(x - hi)
__device__ __forceinline__ void split2(float x0, float x1, unsigned& hi, unsigned& lo) {
  const h16x2 h = __builtin_convertvector(f32x2{x0, x1}, h16x2);
  const f32x2 hf = __builtin_convertvector(h, f32x2);
  const f32x2 r = f32x2{x0, x1} - hf;
  hi = __builtin_bit_cast(unsigned, h);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector(r, h16x2));
}

// the power of two that brings the largest magnitude m into [2^14, 2^15)
__device__ __forceinline__ int scale_exp(float m) {
  if (!(m > 0.0f) || !(m < __builtin_inff())) return 0;
  int e;
  (void)frexpf(m, &e);  // m = f 2^e, f in [0.5, 1)
  const int s = 15 - e;
  return s < -64 ? -64 : (s > 64 ? 64 : s);
}

// maximum of m over the workgroup (red: 4 floats of LDS); a barrier inside
__device__ __forceinline__ float block_max(float m, float* red, int wave, int l) {
  m = wave_max_f(m);
  if (l == 0) red[wave] = m;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// One K chunk over the board's NG pixel groups: per group the B fragments (hi, lo) from the grid
// (LDS; read two groups ahead) and acc[g] += ah*bh + al*bh + ah*bl. The MFMAs are inline asm with
// the accumulator in place in AGPRs (srcC = vdst: back-to-back accumulation, no copies); INIT
// starts the accumulators from 0. HALF: byte offset of the lo halves from the hi halves.
template <int NG, bool INIT, int PIX, int HALF>
__device__ __forceinline__ void ln_chunk(f32x4 (&acc)[NG], h16x8 ah, h16x8 al, const unsigned char* grid,
                                         const int (&pp)[NG], int coff) {
  h16x8 rb[3][2];
  auto load = [&](int g, int slot) {
    const unsigned char* q = grid + pp[g] * PIX + coff;
    rb[slot][0] = *reinterpret_cast<const h16x8*>(q);
    rb[slot][1] = *reinterpret_cast<const h16x8*>(q + HALF);
  };
  load(0, 0);
  if (NG > 1) load(1, 1);
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (g + 2 < NG) load(g + 2, (g + 2) % 3);
    const h16x8 bh = rb[g % 3][0], bl = rb[g % 3][1];
    if (INIT)
      asm volatile(
          "v_mfma_f32_16x16x32_f16 %0, %1, %2, 0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
          : "=&a"(acc[g])
          : "v"(ah), "v"(bh), "v"(al), "v"(bl));
    else
      asm volatile(
          "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
          : "+a"(acc[g])
          : "v"(ah), "v"(bh), "v"(al), "v"(bl));
  }
}

// the accumulators are written by MFMAs the compiler cannot see: wait out the MFMA write ->
// VALU read latency before the epilogue reads them
__device__ __forceinline__ void ln_mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }

struct LnHeads {
  const float *wp, *bp, *wv, *bv, *w1t, *b1, *w2, *b2;
  int P;
  float* pf;
  float* v;
};

template <int N>
__global__ __launch_bounds__(kLnThreads, 1) void k_leafnet_x3(const float* __restrict__ obs,
                                                              const h16x8* __restrict__ wstem,
                                                              const float* __restrict__ sstem,
                                                              const float* __restrict__ bstem,
                                                              const h16x8* __restrict__ wt,
                                                              const float* __restrict__ st,
                                                              const float* __restrict__ bt, int nlayers,
                                                              LnHeads hd, float* __restrict__ xout) {
  constexpr int NN = N * N, NP = N + 2, NG = (NN + 15) / 16, PIX_IT = (NN + kLnThreads - 1) / kLnThreads;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* act = lds;                                 // [NP*NP][kPixBytes]
  unsigned char* sin = lds + NP * NP * kPixBytes;           // [NP*NP][kStemPixBytes]
  float* red = reinterpret_cast<float*>(sin + NP * NP * kStemPixBytes);
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, n = l & 15, ks = l >> 4;
  const int oc = 16 * wave + 4 * ks;  // the lane's 4 output channels oc..oc+3 in the D fragments
  const size_t b = blockIdx.x;

  // zero both grids (the halo stays zero; interiors are overwritten before they are read)
  for (int i = tid; i < NP * NP * (kPixBytes + kStemPixBytes) / 16; i += kLnThreads)
    reinterpret_cast<u32x4*>(lds)[i] = u32x4{0u, 0u, 0u, 0u};

  // the lane's pixel of each group (clamped to the board for the last group's spare lanes) as a
  // padded-grid index
  int pp[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int p = 16 * g + n < NN ? 16 * g + n : NN - 1;
    pp[g] = (p / N + 1) * NP + p % N + 1;
  }

  // ---- stem input: the planar observation [8][N][N] of the board, scaled by its maximum, split
  const float* ob = obs + b * kStemCinX3 * NN;
  float xin[PIX_IT][kStemCinX3];
  float m = 0.0f;
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
#pragma unroll
    for (int c = 0; c < kStemCinX3; ++c) {
      xin[it][c] = p < NN ? ob[c * NN + p] : 0.0f;
      m = fmaxf(m, fabsf(xin[it][c]));
    }
  }
  int ex = scale_exp(block_max(m, red, wave, l));  // the barrier also orders the zeroing before the writes
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
    if (p < NN) {
      unsigned h[4], o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split2(ldexpf(xin[it][2 * q], ex), ldexpf(xin[it][2 * q + 1], ex), h[q], o[q]);
      const u32x4 hi{h[0], h[1], h[2], h[3]}, lo{o[0], o[1], o[2], o[3]};
      unsigned char* dst = sin + ((p / N + 1) * NP + p % N + 1) * kStemPixBytes;
      *reinterpret_cast<u32x4*>(dst) = hi;
      *reinterpret_cast<u32x4*>(dst + 16) = lo;
    }
  }
  __syncthreads();

  // ---- stem conv: 3 chunks; lane k-group ks of chunk j is tap 4j + ks (taps > 8 carry zero weights)
  f32x4 acc[NG];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int t = 4 * j + ks < 9 ? 4 * j + ks : 8;
    const int toff = ((t / 3 - 1) * NP + (t % 3 - 1)) * kStemPixBytes;
    const h16x8 ah = wstem[((j * 4 + wave) * 2) * 64 + l], al = wstem[((j * 4 + wave) * 2 + 1) * 64 + l];
    if (j == 0)
      ln_chunk<NG, true, kStemPixBytes, 16>(acc, ah, al, sin, pp, toff);
    else
      ln_chunk<NG, false, kStemPixBytes, 16>(acc, ah, al, sin, pp, toff);
  }
  ln_mfma_drain();

  // epilogue of a conv: y = acc * s + bias (+ x0) (ReLU) in place; returns the lane's max |y|
  // over real pixels
  auto epilogue = [&](const float* sv, const float* bv, bool relu, bool residual, const f32x4 (&x0)[NG]) {
    float s[4], bb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[r] = ldexpf(sv[oc + r], -ex);
      bb[r] = bv[oc + r];
    }
    const float floor = relu ? 0.0f : -__builtin_inff();
    float mx = 0.0f;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float y = fmaf(acc[g][r], s[r], bb[r]);
        if (residual) y += x0[g][r];
        y = fmaxf(y, floor);
        acc[g][r] = y;
        if (16 * g + n < NN) mx = fmaxf(mx, fabsf(y));
      }
    }
    return mx;
  };
  // the layer output (acc) scaled by 2^ex and split into the activation grid (after a barrier:
  // every wave has finished reading the grid)
  auto write_act = [&]() {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (16 * g + n < NN) {
        unsigned h0, h1, l0, l1;
        split2(ldexpf(acc[g][0], ex), ldexpf(acc[g][1], ex), h0, l0);
        split2(ldexpf(acc[g][2], ex), ldexpf(acc[g][3], ex), h1, l1);
        unsigned char* dst = act + pp[g] * kPixBytes + 2 * oc;
        *reinterpret_cast<u32x2*>(dst) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(dst + 128) = u32x2{l0, l1};
      }
    }
  };

  f32x4 x0[NG];
  {
    const float mx = epilogue(sstem, bstem, true, false, x0);
#pragma unroll
    for (int g = 0; g < NG; ++g) x0[g] = acc[g];
    ex = scale_exp(block_max(mx, red, wave, l));
    write_act();
    __syncthreads();
  }

  // ---- residual tower: nlayers convs 64 -> 64; ReLU after each block's first conv; the last
  // adds x0 and takes the ReLU (x = relu(x + res_blocks(x)), blokus_nnet.py:140-141)
  constexpr int kLayerBlocks = 18 * 4 * 2;  // (chunk, wave, part) blocks per layer
  for (int layer = 0; layer < nlayers; ++layer) {
    const h16x8* wl = wt + (size_t)layer * kLayerBlocks * 64 + (wave * 2) * 64 + l;
    h16x8 ah = wl[0], al = wl[64];
    auto coff_of = [&](int c) {
      const int t = c >> 1;
      return ((t / 3 - 1) * NP + (t % 3 - 1)) * kPixBytes + (c & 1) * 64 + ks * 16;
    };
    {
      const h16x8 nh = wl[8 * 64], nl = wl[8 * 64 + 64];
      ln_chunk<NG, true, kPixBytes, 128>(acc, ah, al, act, pp, coff_of(0));
      ah = nh;
      al = nl;
    }
    for (int c = 1; c < 18; ++c) {
      h16x8 nh = ah, nl = al;
      if (c + 1 < 18) {
        nh = wl[(c + 1) * 8 * 64];
        nl = wl[(c + 1) * 8 * 64 + 64];
      }
      ln_chunk<NG, false, kPixBytes, 128>(acc, ah, al, act, pp, coff_of(c));
      ah = nh;
      al = nl;
    }
    ln_mfma_drain();
    const bool last = layer + 1 == nlayers;
    const float mx = epilogue(st + layer * 64, bt + layer * 64, last || !(layer & 1), last, x0);
    if (!last) {
      ex = scale_exp(block_max(mx, red, wave, l));
      write_act();
      __syncthreads();
    }
  }

  // ---- outputs: the tower output (optional) and the heads (blokus_nnet.py:146-150, BN folded)
  if (xout) {
#pragma unroll
    for (int g = 0; g < NG; ++g)
      if (16 * g + n < NN)
        *reinterpret_cast<f32x4*>(xout + (b * NN + 16 * g + n) * 64 + oc) = acc[g];
  }
  __syncthreads();  // every wave is done with the activation grid: the heads' scratch reuses it
  float* hp = reinterpret_cast<float*>(act);  // [NN][4 waves][3]
  {
    const f32x4 wp0 = *reinterpret_cast<const f32x4*>(hd.wp + oc);
    const f32x4 wp1 = *reinterpret_cast<const f32x4*>(hd.wp + 64 + oc);
    const f32x4 wvv = *reinterpret_cast<const f32x4*>(hd.wv + oc);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const f32x4 y = acc[g];
      float d[3];
      const f32x4* w[3] = {&wp0, &wp1, &wvv};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float a = y.x * (*w[k]).x + y.y * (*w[k]).y + y.z * (*w[k]).z + y.w * (*w[k]).w;
        a += __shfl_xor(a, 16);
        a += __shfl_xor(a, 32);
        d[k] = a;
      }
      if (ks == 0 && 16 * g + n < NN) {
        float* dst = hp + ((16 * g + n) * 4 + wave) * 3;
        dst[0] = d[0];
        dst[1] = d[1];
        dst[2] = d[2];
      }
    }
  }
  __syncthreads();
  // pf = relu(policy 1x1 conv + bp) (channel-major), vfeat = relu(value 1x1 conv + bv), then
  // v = tanh(W2 relu(W1 vfeat + b1) + b2); the 4 waves sweep quarters of W1's inputs
  float* vfeat = hp + NN * 12;
  float* part = vfeat + NN;
  for (int i = tid; i < NN; i += kLnThreads) {
    const float* q = hp + i * 12;
    const float p0 = ((q[0] + q[3]) + q[6]) + q[9], p1 = ((q[1] + q[4]) + q[7]) + q[10],
                pv = ((q[2] + q[5]) + q[8]) + q[11];
    hd.pf[b * 2 * NN + i] = fmaxf(p0 + hd.bp[0], 0.0f);
    hd.pf[b * 2 * NN + NN + i] = fmaxf(p1 + hd.bp[1], 0.0f);
    vfeat[i] = fmaxf(pv + hd.bv[0], 0.0f);
  }
  __syncthreads();
  {
    const int q0 = (NN * wave) / 4, q1 = (NN * (wave + 1)) / 4;
    float a0 = 0.f, a1 = 0.f;
    int i = q0;
    for (; i + 10 <= q1; i += 10) {
      float w[10];
#pragma unroll
      for (int u = 0; u < 10; ++u) w[u] = hd.w1t[(size_t)(i + u) * 64 + l];
#pragma unroll
      for (int u = 0; u < 10; u += 2) {
        a0 += w[u] * vfeat[i + u];
        a1 += w[u + 1] * vfeat[i + u + 1];
      }
    }
    for (; i < q1; ++i) a0 += hd.w1t[(size_t)i * 64 + l] * vfeat[i];
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

static_assert(ln_lds_bytes(20) <= 160 * 1024, "k_leafnet_x3<20>: LDS");

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_leafnet_x3_weight_bytes(int cin) {
  return cin == 64 || cin == 8 ? ln_chunks(cin) * 4 * 2 * kBlock * 2 : -1;
}

int bk_leafnet_x3_supported(int N) { return N == 14 || N == 20; }

int bk_leafnet_x3(const float* obs, int B, int N, int cin, const void* wstem, const float* sstem, const float* bstem,
                  int nlayers, const void* wtower, const float* stower, const float* btower, const float* wp,
                  const float* bp, const float* wv, const float* bv, const float* w1t, const float* b1,
                  const float* w2, const float* b2, int P, float* pf, float* vout, float* out, void* stream) {
  BK_REQUIRE(obs && wstem && sstem && bstem && wtower && stower && btower && B >= 0, "bad argument");
  BK_REQUIRE(wp && bp && wv && bv && w1t && b1 && w2 && b2 && pf && vout && P > 0, "bad argument");
  BK_REQUIRE(cin == kStemCinX3, "bk_leafnet_x3: the stem takes 8 observation planes");
  BK_REQUIRE(nlayers >= 1, "bk_leafnet_x3: at least one tower conv");
  BK_REQUIRE(bk_leafnet_x3_supported(N), "bk_leafnet_x3: N must be 14 or 20");
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  BK_REQUIRE(a16(wstem) && a16(wtower) && a16(wp) && a16(wv) && a16(out), "bk_leafnet_x3: 16-byte aligned buffers");
  if (B == 0) return BK_OK;
  {
    const void* fns[2] = {(const void*)k_leafnet_x3<14>, (const void*)k_leafnet_x3<20>};
    if (set_max_dynamic_lds(fns, 2, ln_lds_bytes(20)) != BK_OK) return BK_EHIP;
  }
  const LnHeads h{wp, bp, wv, bv, w1t, b1, w2, b2, P, pf, vout};
  hipStream_t s = (hipStream_t)stream;
  const h16x8* ws = reinterpret_cast<const h16x8*>(wstem);
  const h16x8* wt = reinterpret_cast<const h16x8*>(wtower);
  if (N == 20)
    hipLaunchKernelGGL(k_leafnet_x3<20>, dim3(B), dim3(kLnThreads), ln_lds_bytes(20), s, obs, ws, sstem, bstem, wt,
                       stower, btower, nlayers, h, out);
  else
    hipLaunchKernelGGL(k_leafnet_x3<14>, dim3(B), dim3(kLnThreads), ln_lds_bytes(14), s, obs, ws, sstem, bstem, wt,
                       stower, btower, nlayers, h, out);
  return launch_check("k_leafnet_x3");
}

}  // extern "C"
