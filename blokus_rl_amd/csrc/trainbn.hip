// trainbn.hip — the learner's train-mode batch norm over 64-channel NHWC activations
// (nn.BatchNorm2d(64) of models/blokus_nnet.py:99-112 as neural_network.py:52-85 trains it):
// batch statistics, the running-stat update, the normalisation, and the backward pass, in
// fewer HBM passes than the framework's kernels (the statistics and the backward reduction are
// one streaming read each, summed in fp64 per workgroup and combined in a fixed order).
//
// x, y, dy, dx: [M][64] f32 (M = batch x pixels, channels innermost: a channels_last [B, 64, H, W]).
#include "../../include/blokus_engine.h"
#include "ctx.h"

namespace bk {
namespace {

using f32x4 = float __attribute__((ext_vector_type(4)));
constexpr int kBnThreads = 256, kBnRows = kBnThreads / 16;  // 16 channel quads x 16 rows per pass
constexpr int kBnGrid = 512;
constexpr int kBnAxGrid = 2048;  // k_bn_axpb's workgroups (grid-stride)

// per workgroup: sum over its rows of a[r][c] (and of a[r][c] * (b[r][c] - mb[c]) when b != null,
// else of a[r][c]^2) in fp64 -> part[c][g][2] (channel-major: each finalize workgroup then reads
// its channel's G partials contiguously)
// (rp, rq non-null, the fused ReLU's backward: a counts only where b rp + rq > 0, i.e. where the
// forward's batch-norm output was positive)
__global__ __launch_bounds__(kBnThreads) void k_bn_reduce(const float* __restrict__ a, const float* __restrict__ b,
                                                          const float* __restrict__ mb, int64_t M,
                                                          double* __restrict__ part, const float* __restrict__ rp,
                                                          const float* __restrict__ rq) {
  __shared__ double red[kBnRows][64][2];
  const int tid = threadIdx.x, q = tid & 15, rl = tid >> 4;
  const f32x4* a4 = reinterpret_cast<const f32x4*>(a);
  const f32x4* b4 = reinterpret_cast<const f32x4*>(b);
  f32x4 m4 = {0.f, 0.f, 0.f, 0.f}, p4 = {0.f, 0.f, 0.f, 0.f}, q4 = {0.f, 0.f, 0.f, 0.f};
  if (b) m4 = reinterpret_cast<const f32x4*>(mb)[q];
  if (rp) {
    p4 = reinterpret_cast<const f32x4*>(rp)[q];
    q4 = reinterpret_cast<const f32x4*>(rq)[q];
  }
  double s[4] = {0, 0, 0, 0}, t[4] = {0, 0, 0, 0};
  for (int64_t r = (int64_t)blockIdx.x * kBnRows + rl; r < M; r += (int64_t)gridDim.x * kBnRows) {
    const f32x4 v = __builtin_nontemporal_load(a4 + r * 16 + q);
    float vv[4] = {v.x, v.y, v.z, v.w};
    if (b) {
      const f32x4 w = __builtin_nontemporal_load(b4 + r * 16 + q);
      if (rp) {
        const f32x4 z = w * p4 + q4;
        vv[0] = z.x > 0.f ? vv[0] : 0.f;
        vv[1] = z.y > 0.f ? vv[1] : 0.f;
        vv[2] = z.z > 0.f ? vv[2] : 0.f;
        vv[3] = z.w > 0.f ? vv[3] : 0.f;
      }
      const float ww[4] = {w.x - m4.x, w.y - m4.y, w.z - m4.z, w.w - m4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] += (double)vv[j];
        t[j] += (double)vv[j] * (double)ww[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] += (double)vv[j];
        t[j] += (double)vv[j] * (double)vv[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[rl][4 * q + j][0] = s[j];
    red[rl][4 * q + j][1] = t[j];
  }
  __syncthreads();
  if (tid < 128) {
    const int c = tid >> 1, k = tid & 1;
    double acc = 0;
#pragma unroll
    for (int i = 0; i < kBnRows; ++i) acc += red[i][c][k];
    part[((size_t)c * gridDim.x + blockIdx.x) * 2 + k] = acc;
  }
}

// the per-workgroup partial sums part[c][g][NV] (NV = 2 values, or 1: the second sum is 0) added
// over g for channel c = blockIdx.x (one workgroup per channel: 256 threads each take g = tid,
// tid + 256, ... in order, then a fixed LDS tree); every thread gets the channel's two totals
constexpr int kBnFinThreads = 256;
template <int NV = 2>
__device__ __forceinline__ void bn_sum_parts(const double* __restrict__ part, int G, double& s0, double& s1) {
  __shared__ double red[kBnFinThreads][2];
  const int c = blockIdx.x, t = threadIdx.x;
  double a = 0, b = 0;
  const double* pc = part + (size_t)c * G * NV;
  for (int g = t; g < G; g += kBnFinThreads) {
    a += pc[(size_t)g * NV];
    if (NV == 2) b += pc[(size_t)g * NV + 1];
  }
  red[t][0] = a;
  red[t][1] = b;
  __syncthreads();
  for (int h = kBnFinThreads / 2; h > 0; h >>= 1) {
    if (t < h) {
      red[t][0] += red[t + h][0];
      red[t][1] += red[t + h][1];
    }
    __syncthreads();
  }
  s0 = red[0][0];
  s1 = red[0][1];
}

// forward statistics -> mean, invstd, scale = gamma invstd, shift = beta - mean scale (f32), and
// the running statistics (PyTorch's update: r = (1 - m) r + m v, the variance unbiased)
__global__ __launch_bounds__(kBnFinThreads) void k_bn_finalize_fwd(const double* __restrict__ part, int G, int64_t M,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         float* __restrict__ rmean, float* __restrict__ rvar, float momentum,
                                                         float eps, float* __restrict__ stats) {
  const int c = blockIdx.x;
  double s, ss;
  bn_sum_parts(part, G, s, ss);
  if (threadIdx.x != 0) return;
  const double mean = s / (double)M;
  double var = ss / (double)M - mean * mean;
  var = var > 0 ? var : 0;
  const double inv = 1.0 / sqrt(var + (double)eps);
  const float g = gamma ? gamma[c] : 1.0f, bt = beta ? beta[c] : 0.0f;
  stats[c] = (float)mean;
  stats[64 + c] = (float)inv;
  stats[128 + c] = (float)((double)g * inv);
  stats[192 + c] = (float)((double)bt - mean * (double)g * inv);
  if (rmean) rmean[c] = (1.0f - momentum) * rmean[c] + momentum * (float)mean;
  if (rvar) rvar[c] = (1.0f - momentum) * rvar[c] + momentum * (float)(M > 1 ? var * (double)M / (double)(M - 1) : var);
}

// backward statistics -> dgamma, dbeta, and dx = k1 dy + k3 x + k2 per channel
__global__ __launch_bounds__(kBnFinThreads) void k_bn_finalize_bwd(const double* __restrict__ part, int G, int64_t M,
                                                         const float* __restrict__ gamma, const float* __restrict__ stats,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                         float* __restrict__ coef) {
  const int c = blockIdx.x;
  double sd, sdx;  // sum dy, sum dy (x - mean)
  bn_sum_parts(part, G, sd, sdx);
  if (threadIdx.x != 0) return;
  const double mean = stats[c], inv = stats[64 + c], g = gamma ? gamma[c] : 1.0f;
  if (dgamma) dgamma[c] = (float)(sdx * inv);
  if (dbeta) dbeta[c] = (float)sd;
  const double k1 = g * inv, k3 = -g * inv * inv * inv * sdx / (double)M;
  const double k2 = -g * inv * sd / (double)M - k3 * mean;
  coef[c] = (float)k1;
  coef[64 + c] = (float)k2;
  coef[128 + c] = (float)k3;
}

// out = a * p[c] + q[c] (+ b * r[c]) over [M][64] (forward: y = x scale + shift; backward:
// dx = dy k1 + k2 + x k3). relu: out = max(out, 0) (the fused ReLU of the forward). mp / mq
// non-null (the fused ReLU's backward): a counts only where b mp + mq > 0. colsum non-null: the
// workgroup's per-channel sums of out in fp64 -> colsum[c][g] (the bias gradient of the conv that
// feeds the batch norm, k_colsum_finalize adds them up in a fixed order).
__global__ __launch_bounds__(256) void k_bn_axpb(const float* __restrict__ a, const float* __restrict__ b,
                                                 const float* __restrict__ p, const float* __restrict__ q,
                                                 const float* __restrict__ rr, int64_t n4, float* __restrict__ out,
                                                 int relu, const float* __restrict__ mp, const float* __restrict__ mq,
                                                 double* __restrict__ colsum) {
  const f32x4* a4 = reinterpret_cast<const f32x4*>(a);
  const f32x4* b4 = reinterpret_cast<const f32x4*>(b);
  const int cq = threadIdx.x & 15;  // the channel quad is fixed per thread: the stride is a multiple of 16
  const f32x4 pv = reinterpret_cast<const f32x4*>(p)[cq], qv = reinterpret_cast<const f32x4*>(q)[cq];
  f32x4 rv = {0.f, 0.f, 0.f, 0.f}, mpv = {0.f, 0.f, 0.f, 0.f}, mqv = {0.f, 0.f, 0.f, 0.f};
  if (b) rv = reinterpret_cast<const f32x4*>(rr)[cq];
  if (mp) {
    mpv = reinterpret_cast<const f32x4*>(mp)[cq];
    mqv = reinterpret_cast<const f32x4*>(mq)[cq];
  }
  double cs[4] = {0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 av = __builtin_nontemporal_load(a4 + i);
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if (b) bv = __builtin_nontemporal_load(b4 + i);
    if (mp) {
      const f32x4 z = bv * mpv + mqv;
      av.x = z.x > 0.f ? av.x : 0.f;
      av.y = z.y > 0.f ? av.y : 0.f;
      av.z = z.z > 0.f ? av.z : 0.f;
      av.w = z.w > 0.f ? av.w : 0.f;
    }
    f32x4 v = av * pv + qv;
    if (b) v += bv * rv;
    if (relu) {
      v.x = v.x > 0.f ? v.x : 0.f;
      v.y = v.y > 0.f ? v.y : 0.f;
      v.z = v.z > 0.f ? v.z : 0.f;
      v.w = v.w > 0.f ? v.w : 0.f;
    }
    if (colsum) {
      cs[0] += (double)v.x;
      cs[1] += (double)v.y;
      cs[2] += (double)v.z;
      cs[3] += (double)v.w;
    }
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(out) + i);
  }
  if (colsum) {  // workgroup-uniform
    __shared__ double red[16][64];
    const int rl = threadIdx.x >> 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) red[rl][4 * cq + j] = cs[j];
    __syncthreads();
    if (threadIdx.x < 64) {
      double acc = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc += red[i][threadIdx.x];
      colsum[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = acc;
    }
  }
}

// colsum partials [64][G] -> out[c] (f32), in bn_sum_parts' fixed order (64 workgroups)
__global__ __launch_bounds__(kBnFinThreads) void k_colsum_finalize(const double* __restrict__ part, int G,
                                                                   float* __restrict__ outc) {
  double s0, s1;
  bn_sum_parts<1>(part, G, s0, s1);
  if (threadIdx.x == 0) outc[blockIdx.x] = (float)s0;
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_bn_workspace_doubles(void) { return kBnGrid * 64 * 2; }

int bk_bn_workspace2_doubles(void) { return kBnAxGrid * 64 * 2; }

int bk_bn_forward_ex(const float* x, int64_t M, const float* gamma, const float* beta, float* running_mean,
                     float* running_var, float momentum, float eps, double* workspace, float* stats, float* y, int relu,
                     void* stream) {
  BK_REQUIRE(x && workspace && stats && y && M > 0, "bad argument");
  BK_REQUIRE(((uintptr_t)x & 15u) == 0 && ((uintptr_t)y & 15u) == 0 && ((uintptr_t)stats & 15u) == 0,
             "bk_bn_forward: 16-byte aligned buffers");
  hipStream_t s = (hipStream_t)stream;
  const int64_t blocks = (M + kBnRows - 1) / kBnRows;
  const int G = blocks < kBnGrid ? (int)blocks : kBnGrid;
  hipLaunchKernelGGL(k_bn_reduce, dim3(G), dim3(kBnThreads), 0, s, x, (const float*)nullptr, (const float*)nullptr, M,
                     workspace, (const float*)nullptr, (const float*)nullptr);
  hipLaunchKernelGGL(k_bn_finalize_fwd, dim3(64), dim3(kBnFinThreads), 0, s, workspace, G, M, gamma, beta, running_mean, running_var,
                     momentum, eps, stats);
  const int64_t n4 = M * 16;
  const int64_t ab = (n4 + 255) / 256;
  hipLaunchKernelGGL(k_bn_axpb, dim3(ab < kBnAxGrid ? (int)ab : kBnAxGrid), dim3(256), 0, s, x, (const float*)nullptr,
                     stats + 128, stats + 192, (const float*)nullptr, n4, y, relu, (const float*)nullptr,
                     (const float*)nullptr, (double*)nullptr);
  return launch_check("bk_bn_forward");
}

int bk_bn_forward(const float* x, int64_t M, const float* gamma, const float* beta, float* running_mean,
                  float* running_var, float momentum, float eps, double* workspace, float* stats, float* y,
                  void* stream) {
  return bk_bn_forward_ex(x, M, gamma, beta, running_mean, running_var, momentum, eps, workspace, stats, y, 0, stream);
}

int bk_bn_backward_ex(const float* dy, const float* x, int64_t M, const float* gamma, const float* stats,
                      double* workspace, float* coef, float* dgamma, float* dbeta, float* dx, int relu, float* dsum,
                      double* workspace2, void* stream) {
  BK_REQUIRE(dy && x && stats && workspace && coef && dx && M > 0, "bad argument");
  BK_REQUIRE(!dsum || workspace2, "bk_bn_backward_ex: dsum needs workspace2");
  BK_REQUIRE(((uintptr_t)dy & 15u) == 0 && ((uintptr_t)x & 15u) == 0 && ((uintptr_t)dx & 15u) == 0 &&
                 ((uintptr_t)coef & 15u) == 0 && ((uintptr_t)stats & 15u) == 0,
             "bk_bn_backward: 16-byte aligned buffers");
  hipStream_t s = (hipStream_t)stream;
  const int64_t blocks = (M + kBnRows - 1) / kBnRows;
  const int G = blocks < kBnGrid ? (int)blocks : kBnGrid;
  const float* mp = relu ? stats + 128 : nullptr;
  const float* mq = relu ? stats + 192 : nullptr;
  hipLaunchKernelGGL(k_bn_reduce, dim3(G), dim3(kBnThreads), 0, s, dy, x, stats, M, workspace, mp, mq);
  hipLaunchKernelGGL(k_bn_finalize_bwd, dim3(64), dim3(kBnFinThreads), 0, s, workspace, G, M, gamma, stats, dgamma, dbeta, coef);
  const int64_t n4 = M * 16;
  const int64_t ab = (n4 + 255) / 256;
  const int GA = ab < kBnAxGrid ? (int)ab : kBnAxGrid;
  hipLaunchKernelGGL(k_bn_axpb, dim3(GA), dim3(256), 0, s, dy, x, coef, coef + 64, coef + 128, n4, dx, 0, mp, mq,
                     dsum ? workspace2 : (double*)nullptr);
  if (dsum) hipLaunchKernelGGL(k_colsum_finalize, dim3(64), dim3(kBnFinThreads), 0, s, workspace2, GA, dsum);
  return launch_check("bk_bn_backward");
}

int bk_bn_backward(const float* dy, const float* x, int64_t M, const float* gamma, const float* stats, double* workspace,
                   float* coef, float* dgamma, float* dbeta, float* dx, void* stream) {
  return bk_bn_backward_ex(dy, x, M, gamma, stats, workspace, coef, dgamma, dbeta, dx, 0, nullptr, nullptr, stream);
}

}  // extern "C"
