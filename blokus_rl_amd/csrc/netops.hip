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

}  // extern "C"
