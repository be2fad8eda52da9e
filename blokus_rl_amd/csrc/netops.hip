// netops.hip — epilogues of the leaf evaluator's convolutions (the ResNet of
// models/blokus_nnet.py:88-151, BN folded for inference).
//
// MIOpen's convolution with a bias writes the conv result, then adds the bias in separate passes,
// and the ReLU / residual add are further passes: four round trips of the 256 x 64 x 20 x 20 f32
// activation (26 MB) per conv. k_bias_act does bias + optional residual + optional ReLU in one
// pass over the bias-free conv output, in place, on the NHWC (channels_last) layout the leaf
// batch uses: y = act(x + b[c] (+ r)). Same arithmetic and order as relu(conv + b (+ r)).
// Bound: HBM (read x (+ r), write y).
#include "../../include/blokus_engine.h"
#include "ctx.h"

#include <algorithm>

namespace bk {
namespace {

template <bool RELU, bool RES>
__global__ __launch_bounds__(256) void k_bias_act4(float4* __restrict__ x, const float* __restrict__ bias,
                                                   const float4* __restrict__ res, int64_t n4, int C) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)((i * 4) % C);
    float4 v = x[i];
    v.x = v.x + bias[c];
    v.y = v.y + bias[c + 1];
    v.z = v.z + bias[c + 2];
    v.w = v.w + bias[c + 3];
    if (RES) {
      const float4 r = res[i];
      v.x = v.x + r.x;
      v.y = v.y + r.y;
      v.z = v.z + r.z;
      v.w = v.w + r.w;
    }
    if (RELU) {
      v.x = fmaxf(v.x, 0.0f);
      v.y = fmaxf(v.y, 0.0f);
      v.z = fmaxf(v.z, 0.0f);
      v.w = fmaxf(v.w, 0.0f);
    }
    x[i] = v;
  }
}

template <bool RELU, bool RES>
__global__ __launch_bounds__(256) void k_bias_act1(float* __restrict__ x, const float* __restrict__ bias,
                                                   const float* __restrict__ res, int64_t n, int C) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = x[i] + bias[i % C];
    if (RES) v = v + res[i];
    if (RELU) v = fmaxf(v, 0.0f);
    x[i] = v;
  }
}

template <bool RELU, bool RES>
void launch(float* x, const float* b, const float* r, int64_t n, int C, hipStream_t s) {
  if (C % 4 == 0 && ((uintptr_t)x & 15u) == 0 && (!r || ((uintptr_t)r & 15u) == 0)) {
    const int64_t n4 = n / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
    hipLaunchKernelGGL((k_bias_act4<RELU, RES>), dim3(blocks), dim3(256), 0, s, (float4*)x, b, (const float4*)r, n4,
                       C);
  } else {
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL((k_bias_act1<RELU, RES>), dim3(blocks), dim3(256), 0, s, x, b, r, n, C);
  }
}

// ResNet heads (blokus_nnet.py:146-150, BN folded), one 256-thread workgroup per board:
//   policy features pf[c*NN + i] = relu(x_i . wp_c + bp_c), c = 0, 1 (the NCHW flatten order the
//   policy Linear expects), and the value MLP v = tanh(W2 relu(W1 relu(x . wv + bv) + b1) + b2).
// Phase 1: 16 lanes read one pixel's 64-channel row (256 B contiguous, NHWC tower output),
// several rows in flight per lane, and reduce their partial dot products within the 16-lane row. Phase 2 (fc1): lane o
// of each wave owns hidden unit o and sweeps a quarter of the NN inputs over the transposed
// weights w1t [NN][64] (coalesced), the 4 waves' partial sums meet in LDS. Phase 3: one wave.
constexpr int kHeadC = 64;
__global__ __launch_bounds__(256) void k_resnet_heads(const float* __restrict__ x, int NN,
                                                      const float* __restrict__ wp, const float* __restrict__ bp,
                                                      const float* __restrict__ wv, const float* __restrict__ bv,
                                                      const float* __restrict__ w1t, const float* __restrict__ b1,
                                                      const float* __restrict__ w2, const float* __restrict__ b2,
                                                      int P, float* __restrict__ pf, float* __restrict__ vout) {
  extern __shared__ float vfeat[];  // [NN] value features, then [4][64] fc1 partial sums
  float* part = vfeat + NN;
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int sub = t & 15, grp = t >> 4;  // 16 pixel groups of 16 lanes
  const float4 wp0 = reinterpret_cast<const float4*>(wp)[sub];
  const float4 wp1 = reinterpret_cast<const float4*>(wp + kHeadC)[sub];
  const float4 wvv = reinterpret_cast<const float4*>(wv)[sub];
  const float* xb = x + (size_t)b * NN * kHeadC;
  constexpr int kIn = 5;  // rows in flight per lane
  for (int i0 = 0; i0 < NN; i0 += 16 * kIn) {
    float4 xv[kIn];
#pragma unroll
    for (int u = 0; u < kIn; ++u) {
      const int i = i0 + 16 * u + grp;
      xv[u] = i < NN ? reinterpret_cast<const float4*>(xb + (size_t)i * kHeadC)[sub] : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kIn; ++u) {
      const int i = i0 + 16 * u + grp;
      float d0 = xv[u].x * wp0.x + xv[u].y * wp0.y + xv[u].z * wp0.z + xv[u].w * wp0.w;
      float d1 = xv[u].x * wp1.x + xv[u].y * wp1.y + xv[u].z * wp1.z + xv[u].w * wp1.w;
      float dv = xv[u].x * wvv.x + xv[u].y * wvv.y + xv[u].z * wvv.z + xv[u].w * wvv.w;
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) {
        d0 += __shfl_xor(d0, o, 16);
        d1 += __shfl_xor(d1, o, 16);
        dv += __shfl_xor(dv, o, 16);
      }
      if (sub == 0 && i < NN) {
        pf[(size_t)b * 2 * NN + i] = fmaxf(d0 + bp[0], 0.0f);
        pf[(size_t)b * 2 * NN + NN + i] = fmaxf(d1 + bp[1], 0.0f);
        vfeat[i] = fmaxf(dv + bv[0], 0.0f);
      }
    }
  }
  __syncthreads();
  const int wave = t >> 6, l = t & 63;
  const int q0 = (NN * wave) / 4, q1 = (NN * (wave + 1)) / 4;
  // 10 independent loads in flight per lane, two accumulators (the fc1 sweep is latency-bound)
  float acc0 = 0.f, acc1 = 0.f;
  int i = q0;
  for (; i + 10 <= q1; i += 10) {
    float w[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) w[u] = w1t[(size_t)(i + u) * kHeadC + l];
#pragma unroll
    for (int u = 0; u < 10; u += 2) {
      acc0 += w[u] * vfeat[i + u];
      acc1 += w[u + 1] * vfeat[i + u + 1];
    }
  }
  for (; i < q1; ++i) acc0 += w1t[(size_t)i * kHeadC + l] * vfeat[i];
  part[wave * kHeadC + l] = acc0 + acc1;
  __syncthreads();
  if (wave == 0) {
    const float h = fmaxf(((part[l] + part[kHeadC + l]) + (part[2 * kHeadC + l] + part[3 * kHeadC + l])) + b1[l], 0.0f);
    for (int q = 0; q < P; ++q) {
      const float s = wave_sum_f(w2[q * kHeadC + l] * h);
      if (l == 0) vout[(size_t)b * P + q] = tanhf(s + b2[q]);
    }
  }
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_bias_act(float* x, int64_t n, int C, const float* bias, const float* residual, int relu, void* stream) {
  BK_REQUIRE(x && bias && n >= 0 && C > 0 && n % C == 0, "bad argument");
  if (n == 0) return BK_OK;
  hipStream_t s = (hipStream_t)stream;
  if (relu) {
    if (residual) launch<true, true>(x, bias, residual, n, C, s);
    else launch<true, false>(x, bias, nullptr, n, C, s);
  } else {
    if (residual) launch<false, true>(x, bias, residual, n, C, s);
    else launch<false, false>(x, bias, nullptr, n, C, s);
  }
  return launch_check("k_bias_act");
}

int bk_resnet_heads(const float* x, int B, int NN, const float* wp, const float* bp, const float* wv, const float* bv,
                    const float* w1t, const float* b1, const float* w2, const float* b2, int P, float* pf,
                    float* vout, void* stream) {
  BK_REQUIRE(x && wp && bp && wv && bv && w1t && b1 && w2 && b2 && pf && vout && B >= 0 && NN > 0 && P > 0,
             "bad argument");
  BK_REQUIRE(((uintptr_t)x & 15u) == 0 && ((uintptr_t)wp & 15u) == 0 && ((uintptr_t)wv & 15u) == 0,
             "bk_resnet_heads: 16-byte aligned x, wp, wv");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_resnet_heads, dim3(B), dim3(256), sizeof(float) * (NN + 4 * kHeadC), (hipStream_t)stream, x, NN,
                     wp, bp, wv, bv, w1t, b1, w2, b2, P, pf, vout);
  return launch_check("k_resnet_heads");
}

}  // extern "C"
