// tower_dev.h — device code of the Winograd form-2 convolution (k_conv3x3_wino2) and of the leaf
// net in one workgroup per board (tower_forward: stem, residual tower, heads), used by conv.hip
// (k_conv3x3_wino2, k_tower_wino). Design notes: conv.hip.
#pragma once
#include "ctx.h"

namespace bk {
namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;

#ifndef BK_WINO_STAMP
#define BK_WINO_STAMP 0  // timing diagnostics only: per-wave s_memtime stamps (bk_wino_stamps)
#endif
#if BK_WINO_STAMP
constexpr int kStampPerWave = 32;
__device__ unsigned long long g_wino_stamps[256 * 8 * kStampPerWave];
#define WSTAMP(i)                                                                                      \
  do {                                                                                                 \
    if (l == 0 && (i) < kStampPerWave)                                                                 \
      g_wino_stamps[(blockIdx.x * 8 + wave) * kStampPerWave + (i)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#define W2STAMP(i, v)                                                                         \
  do {                                                                                        \
    if (l == 0 && (i) < kStampPerWave) g_wino_stamps[(blockIdx.x * 8 + wave) * kStampPerWave + (i)] = (v); \
  } while (0)
#else
#define WSTAMP(i) \
  do {            \
  } while (0)
#define W2STAMP(i, v) \
  do {                \
  } while (0)
#endif

// packed f32 add / subtract (v_pk_add_f32, with the second operand negated for a - b: the same
// IEEE result as a scalar subtraction); the compiler splits a <2 x float> fsub into two VALU ops
__device__ __forceinline__ f32x2 pk_add(f32x2 a, f32x2 b) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f32x2 pk_sub(f32x2 a, f32x2 b) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
constexpr int kW2Threads = 256;
constexpr int kW2UFloats = 4 * 64 * kWave * 4;  // [4 kb][64 q][64 lanes][4]: (s, p) = divmod(4q + e, 16)
constexpr int kW2VBuf = 16 * 16 * 16 * 4;      // floats per V buffer: [16 s][16 p][16 t][4 g]
constexpr unsigned kW2Out = 0x7fff0000u;       // a window offset beyond any buffer: the load returns 0

// Per-lane context of the form-2 kernels: the input buffer, the LDS V buffers, the lane's
// transform role (tile tt of the group, channel quad sq) and MFMA role (wave = output block).
struct W2Lane {
  float* v_lds;
  __amdgpu_buffer_rsrc_t xr;
  int wave, l, tt, sq;
  __device__ f32x4 ld(unsigned o) const {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
  }
  // window offsets of the lane's tile at tile coordinates (ty, tx) of the board whose row 0 is at
  // byte rowbase0, branch-free: a row or column off the board (or an invalid tile) gets a base of
  // kW2Out, so the sum lands beyond the buffer and the load returns 0
  __device__ void window(bool tv, int N, int rowbase0, int ty, int tx, unsigned (&off)[16]) const {
    const int rbase = rowbase0 + (2 * ty - 1) * N * 256 + 16 * sq, cbase = (2 * tx - 1) * 256;
    unsigned rb[4], cb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int yy = 2 * ty - 1 + i, xx = 2 * tx - 1 + i;
      rb[i] = tv && yy >= 0 && yy < N ? (unsigned)(rbase + i * N * 256) : kW2Out;
      cb[i] = xx >= 0 && xx < N ? (unsigned)(cbase + i * 256) : kW2Out;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) off[4 * i + j] = rb[i] + cb[j];
  }
  // B^T d B of the lane's 4 channels as two packed pairs h -> V[buf][sq][p][tt][2h, 2h+1], in 8
  // parts k = (h, i): row i of the 4x4 result, t_i = (B^T d)_i from two window rows, v_i = t_i B
  __device__ void transform_part(const f32x4 (&raw)[16], int buf, int k) const {
    const int h = k >> 2, i = k & 3;
    float* dst = v_lds + buf * kW2VBuf + sq * 1024 + tt * 4 + 2 * h;
    auto d = [&](int q) { return h ? raw[q].zw : raw[q].xy; };
    f32x2 t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (i == 0) t[j] = pk_sub(d(j), d(8 + j));
      else if (i == 1) t[j] = pk_add(d(4 + j), d(8 + j));
      else if (i == 2) t[j] = pk_sub(d(8 + j), d(4 + j));
      else t[j] = pk_sub(d(4 + j), d(12 + j));
    }
    *reinterpret_cast<f32x2*>(dst + (4 * i + 0) * 64) = pk_sub(t[0], t[2]);
    *reinterpret_cast<f32x2*>(dst + (4 * i + 1) * 64) = pk_add(t[1], t[2]);
    *reinterpret_cast<f32x2*>(dst + (4 * i + 2) * 64) = pk_sub(t[2], t[1]);
    *reinterpret_cast<f32x2*>(dst + (4 * i + 3) * 64) = pk_sub(t[1], t[3]);
  }
  // A^T M A + residual + ReLU of the lane's tile (top-left output pixel opix, -1 = none) for
  // channels 16 wave + 4 (l >> 4) + 0..3, on packed channel pairs; y / res: buffer resources whose
  // byte 0 is pixel 0 of their [..][N][N][64] buffers (buffer stores/loads: the destination may be
  // chosen at run time without turning the accesses into flat ones)
  template <bool RELU, bool RES>
  __device__ void epilogue(const f32x4 (&acc)[16], int opix, int N, __amdgpu_buffer_rsrc_t res,
                           __amdgpu_buffer_rsrc_t y) const {
    if (opix < 0) return;
    f32x2 yv[4][2];  // [pixel 2i + j][pair h]
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      auto m = [&](int q) { return h ? acc[q].zw : acc[q].xy; };
      f32x2 u2v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        u2v[j] = pk_add(pk_add(m(j), m(4 + j)), m(8 + j));
        u2v[4 + j] = pk_sub(pk_sub(m(4 + j), m(8 + j)), m(12 + j));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        yv[2 * i][h] = pk_add(pk_add(u2v[4 * i + 0], u2v[4 * i + 1]), u2v[4 * i + 2]);
        yv[2 * i + 1][h] = pk_sub(pk_sub(u2v[4 * i + 1], u2v[4 * i + 2]), u2v[4 * i + 3]);
      }
    }
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const unsigned o = ((unsigned)(opix + (px >> 1) * N + (px & 1)) * 64 + 16 * wave + 4 * (l >> 4)) * 4;
      f32x2 lo = yv[px][0], hi = yv[px][1];
      if (RES) {
        const f32x4 rr = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(res, o, 0, 0));
        lo = pk_add(lo, rr.xy);
        hi = pk_add(hi, rr.zw);
      }
      f32x4 out = f32x4{lo.x, lo.y, hi.x, hi.y};
      if (RELU) {
        out.x = fmaxf(out.x, 0.0f);
        out.y = fmaxf(out.y, 0.0f);
        out.z = fmaxf(out.z, 0.0f);
        out.w = fmaxf(out.w, 0.0f);
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, out), y,
                                             o, 0, 0);
    }
  }
};

// the fused tower's epilogue: ReLU as data (max with floor: 0, or -inf for none), the residual
// (RES, the tower's last conv) from res
// The ResNet heads' 1x1 convs (blokus_nnet.py:146-150), fused into the tower's last layer: per
// output pixel, the dot products of its 64 channels with the 2 policy and 1 value filters. A lane
// holds 4 channels of 4 pixels; the 4 lanes of a tile (l >> 4) meet in two xor-shuffles, and
// each wave's 16-channel partials go to hp[pixel][wave][3] in LDS (summed in a fixed order later).
struct HeadLane {
  f32x4 wp0, wp1, wv;  // the lane's 4 channels of the three 1x1 filters
  float* hp;           // LDS [NN][4][3]
};

template <bool RES, bool HEADS = false>
__device__ __forceinline__ void w2_epilogue_flags(const W2Lane& c, const f32x4 (&acc)[16], int opix, int N,
                                                  float floor, __amdgpu_buffer_rsrc_t res,
                                                  __amdgpu_buffer_rsrc_t y, bool store = true,
                                                  const HeadLane* hl = nullptr) {
  if (opix < 0) return;
  f32x2 yv[4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    auto m = [&](int q) { return h ? acc[q].zw : acc[q].xy; };
    f32x2 u2v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      u2v[j] = pk_add(pk_add(m(j), m(4 + j)), m(8 + j));
      u2v[4 + j] = pk_sub(pk_sub(m(4 + j), m(8 + j)), m(12 + j));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      yv[2 * i][h] = pk_add(pk_add(u2v[4 * i + 0], u2v[4 * i + 1]), u2v[4 * i + 2]);
      yv[2 * i + 1][h] = pk_sub(pk_sub(u2v[4 * i + 1], u2v[4 * i + 2]), u2v[4 * i + 3]);
    }
  }
#pragma unroll
  for (int px = 0; px < 4; ++px) {
    const unsigned o = ((unsigned)(opix + (px >> 1) * N + (px & 1)) * 64 + 16 * c.wave + 4 * (c.l >> 4)) * 4;
    f32x2 lo = yv[px][0], hi = yv[px][1];
    if (RES) {
      const f32x4 rr = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(res, o, 0, 0));
      lo = pk_add(lo, rr.xy);
      hi = pk_add(hi, rr.zw);
    }
    const f32x4 out = f32x4{fmaxf(lo.x, floor), fmaxf(lo.y, floor), fmaxf(hi.x, floor), fmaxf(hi.y, floor)};
    if (store)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, out), y,
                                             o, 0, 0);
    if (HEADS) {
      float d[3];
      const f32x4* w[3] = {&hl->wp0, &hl->wp1, &hl->wv};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float a = out.x * (*w[k]).x + out.y * (*w[k]).y + out.z * (*w[k]).z + out.w * (*w[k]).w;
        a += __shfl_xor(a, 16);
        a += __shfl_xor(a, 32);
        d[k] = a;
      }
      if ((c.l >> 4) == 0) {
        float* dst = hl->hp + ((opix + (px >> 1) * N + (px & 1)) * 4 + c.wave) * 3;
        dst[0] = d[0];
        dst[1] = d[1];
        dst[2] = d[2];
      }
    }
  }
}

// a buffer resource over [p, p + bytes) with its base made provably wave-uniform (readfirstlane),
// so selecting p at run time never makes hipcc wrap the buffer ops in waterfall loops
__device__ __forceinline__ __amdgpu_buffer_rsrc_t w2_rsrc(const float* p, int bytes) {
  const uintptr_t a = (uintptr_t)p;
  const uintptr_t u = ((uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                      (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, bytes, 0x00020000);
}

// The first group's U: this wave's k-steps 0 and 1 (the rest stream in under the first group's
// MFMAs, w2_group<true>), in k-step order, ur[4s + p/4][p%4] = U[16 wave + (l & 15)][4s + (l >> 4)][p]
__device__ __forceinline__ void w2_load_u01(f32x4 (&ur)[64], const f32x4* usrc) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    ur[q] = usrc[q * kWave];
    __builtin_amdgcn_sched_barrier(0);  // keep k-step order: the first group waits step by step
  }
}

// One group of 16 tiles, V already in LDS buffer buf: 16 k-steps of 16 MFMAs (A = U from AGPRs
// via inline asm, B = V from LDS one step ahead, accumulators in VGPRs, the bias as the initial
// accumulator of position (1,1)); meanwhile the next group's window loads go out over steps 0-3
// (offsets from next_window() at step 0, through buffer xr_next) and its transform runs in 8
// parts over steps 8-15 into V[buf ^ 1]. MODE kW2First: this group streams its own U in two
// k-steps ahead (k-steps 0, 1 are loaded before it); in the per-layer kernel the next window is
// already in raw (the prologue loaded it). MODE kW2Last (a layer's last group in the fused
// tower): after the MFMAs, U of the next layer's k-steps 0, 1 (unext). f32 MFMAs run on the SIMD's vector
// ALUs, so a VALU instruction beside them is not hidden and every MFMA <-> VALU switch costs ~10
// cycles (tools/probe/mfma_fill.hip): the MFMA stream carries no VALU, and the VALU work comes
// in batches. Returns with acc ready for the epilogue.
constexpr int kW2Mid = 0, kW2First = 1, kW2Last = 2;
template <int MODE, bool WINDOW_IN_RAW = (MODE == kW2First), class NextWindow>
__device__ __forceinline__ void w2_group(const W2Lane& c, f32x4 (&ur)[64], f32x4 (&raw)[16], const f32x4* usrc,
                                         const f32x4* unext, __amdgpu_buffer_rsrc_t xr_next, f32x4 bias4, int buf,
                                         NextWindow next_window, f32x4 (&acc)[16]) {
  const float* vsrc = c.v_lds + buf * kW2VBuf + (c.l & 15) * 4 + (c.l >> 4);  // V[buf][s][p][t][g]
  float vb[2][16];
  unsigned off[16];
#pragma unroll
  for (int p = 0; p < 16; ++p) vb[0][p] = vsrc[p * 64];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    if (s == 0 && !WINDOW_IN_RAW) next_window(off);
    if (s < 4 && !WINDOW_IN_RAW) {
#pragma unroll
      for (int q = 4 * s; q < 4 * s + 4; ++q)
        raw[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr_next, off[q], 0, 0));
    }
    if (MODE == kW2First && s + 2 < 16) {  // U of k-step s + 2, in order
#pragma unroll
      for (int q = 4 * (s + 2); q < 4 * (s + 2) + 4; ++q) {
        ur[q] = usrc[q * kWave];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (s + 1 < 16) {  // B operands of the next k-step, before any VALU work of this one
#pragma unroll
      for (int p = 0; p < 16; ++p) vb[(s + 1) & 1][p] = vsrc[((s + 1) * 16 + p) * 64];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (s >= 8) c.transform_part(raw, buf ^ 1, s - 8);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const float ua = ur[4 * s + (p >> 2)][p & 3];
      const float vv = vb[s & 1][p];
      if (s == 0 && p == 5)
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %3" : "=&v"(acc[p]) : "a"(ua), "v"(vv), "v"(bias4));
      else if (s == 0)
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=&v"(acc[p]) : "a"(ua), "v"(vv));
      else
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc[p]) : "a"(ua), "v"(vv));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (MODE == kW2Last) w2_load_u01(ur, unext);  // the next layer's first group streams in the rest
  // the accumulators are written by MFMAs the compiler cannot see: wait out the XDL write ->
  // VALU read latency before the epilogue reads them
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}

// One conv layer over B*N*N/4 tiles (any batch): 16-tile groups, the 8 XCDs take contiguous
// eighths of them, each CU a contiguous run (its windows share board rows in L1/L2).
template <bool RELU, bool RES>
__global__ __launch_bounds__(kW2Threads, 1) void k_conv3x3_wino2(const float* __restrict__ x,
                                                                 const float* __restrict__ u2,
                                                                 const float* __restrict__ bias,
                                                                 const float* __restrict__ res,
                                                                 float* __restrict__ y, int N, int tiles) {
  extern __shared__ __attribute__((aligned(16))) float v_lds[];  // [2 buf][16 s][16 p][16 t][4 g]
  const int xcd = blockIdx.x & 7, cu = blockIdx.x >> 3, ncu = gridDim.x >> 3;
  const int groups = (tiles + 15) >> 4;
  const int g_begin = (int)((int64_t)groups * xcd / 8), g_end = (int)((int64_t)groups * (xcd + 1) / 8);
  const int range = g_end - g_begin;
  const int c_lo = g_begin + (int)((int64_t)range * cu / ncu), c_hi = g_begin + (int)((int64_t)range * (cu + 1) / ncu);
  if (c_lo == c_hi) return;
  W2Lane c;
  c.v_lds = v_lds;
  c.wave = threadIdx.x >> 6;
  c.l = threadIdx.x & 63;
  c.tt = c.l & 15;
  c.sq = (c.wave << 2) | (c.l >> 4);
  c.xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, tiles * 1024, 0x00020000);
  const int l = c.l, wave = c.wave;
  W2STAMP(0, __builtin_amdgcn_s_memtime());
  W2STAMP(30, __builtin_amdgcn_s_memrealtime());
  const int T2 = N >> 1, tpb = T2 * T2;
  auto window = [&](int grp, unsigned (&off)[16]) {
    const unsigned tile = (unsigned)(grp * 16 + c.tt);
    const unsigned b = tile / (unsigned)tpb, r = tile - b * (unsigned)tpb;
    const int ty = (int)(r / (unsigned)T2);
    c.window(tile < (unsigned)tiles, N, (int)b * N * N * 256, ty, (int)r - ty * T2, off);
  };
  auto out_pixel = [&](int grp) {  // top-left output pixel of lane l's tile in group grp
    const unsigned tile = (unsigned)(grp * 16 + (l & 15));
    const unsigned b = tile / (unsigned)tpb, r = tile - b * (unsigned)tpb;
    const int ty = (int)(r / (unsigned)T2), tx = (int)r - ty * T2;
    return tile < (unsigned)tiles ? ((int)b * N + 2 * ty) * N + 2 * tx : -1;
  };
  // prologue: the first two groups' windows and the bias, then U of k-steps 0 and 1; the first
  // group's MFMA loop streams in the rest of U
  const f32x4* usrc = reinterpret_cast<const f32x4*>(u2) + (size_t)wave * 64 * kWave + l;
  f32x4 ur[64];
  f32x4 raw[16];
  f32x4 bias4;
  {
    f32x4 raw0[16];
    unsigned off[16];
    window(c_lo, off);
#pragma unroll
    for (int q = 0; q < 16; ++q) raw0[q] = c.ld(off[q]);
    window(c_lo + 1 < c_hi ? c_lo + 1 : c_lo, off);
#pragma unroll
    for (int q = 0; q < 16; ++q) raw[q] = c.ld(off[q]);
    bias4 = *reinterpret_cast<const f32x4*>(bias + 16 * wave + 4 * (l >> 4));
    __builtin_amdgcn_sched_barrier(0);
    w2_load_u01(ur, usrc);
#pragma unroll
    for (int k = 0; k < 8; ++k) c.transform_part(raw0, 0, k);
  }
  __syncthreads();
  W2STAMP(1, __builtin_amdgcn_s_memtime());
  // the last group re-reads its own window into the idle V buffer, so loads and transforms stay
  // unconditional (no load pending across the loop's back edge)
  auto group = [&](int grp, int buf, auto first) {
    W2STAMP(2 + 3 * (grp - c_lo), __builtin_amdgcn_s_memtime());
    const int nxt = grp + 1 < c_hi ? grp + 1 : grp;
    f32x4 acc[16];
    w2_group<decltype(first)::value ? kW2First : kW2Mid>(c, ur, raw, usrc, usrc, c.xr, bias4, buf,
                                                          [&](unsigned (&off)[16]) { window(nxt, off); }, acc);
    W2STAMP(3 + 3 * (grp - c_lo), __builtin_amdgcn_s_memtime());
    c.epilogue<RELU, RES>(acc, out_pixel(grp), N, w2_rsrc(RES ? res : y, tiles * 1024), w2_rsrc(y, tiles * 1024));
    __syncthreads();  // V[buf ^ 1] complete for the next group; V[buf] free to be overwritten
    W2STAMP(4 + 3 * (grp - c_lo), __builtin_amdgcn_s_memtime());
  };
  group(c_lo, 0, std::true_type{});
  int buf = 1;
  for (int grp = c_lo + 1; grp < c_hi; ++grp, buf ^= 1) group(grp, buf, std::false_type{});
  W2STAMP(29, __builtin_amdgcn_s_memtime());
  W2STAMP(31, __builtin_amdgcn_s_memrealtime());
}

// The inference ResNet's whole residual tower (models/blokus_nnet.py:140-141, BN folded) in one
// launch, one workgroup per board: layer l = conv3x3 (Winograd form 2) over the board, ReLU on
// even layers (each block's first conv), the last layer adds the tower input and takes the ReLU;
// intermediate activations ping-pong between hA and hB. A board's tiles depend only on the same
// board, so there is no kernel boundary between layers (no launch gap, no cold L2 after a
// cross-XCD release): the (layer, group) pairs run as one pipeline, each pair loading and
// transforming the NEXT pair's window, across layer boundaries too. That is safe because a window
// only reads rows its layer's predecessor finished at least two pairs earlier (tower_pipeline_ok),
// and a wave's wait for its window loads also waits for all its older stores, so after a group
// barrier every store of two pairs back is complete. A layer's last group refills the U registers
// with the next layer's U step by step (and invalidates L1 before loading next-layer windows).
template <int N>
constexpr bool tower_pipeline_ok() {
  constexpr int T2 = N / 2, TPB = T2 * T2, NG = (TPB + 15) / 16;
  if (NG < 3) return false;
  // the window of group k (tiles 16k..16k+15) reads output rows up to 2*ty_max + 2 of the previous
  // layer, i.e. its tiles up to (ty_max + 1) * T2 + T2 - 1: their group must be <= k + NG - 2
  // (two pairs before the pair that issues the loads, pair (layer, k) - 1)
  for (int k = 0; k < NG; ++k) {
    const int last_tile = 16 * k + 15 < TPB ? 16 * k + 15 : TPB - 1;
    int ty = last_tile / T2 + 1;
    if (ty > T2 - 1) ty = T2 - 1;
    const int need = (ty * T2 + T2 - 1) / 16;  // previous layer's group
    if (need > k + NG - 3) return false;
  }
  return true;
}

// Board-level state of k_tower_wino (plain struct + force-inlined functions: nested lambdas around
// the 256-register U array defeat hipcc's promotion of it to AGPRs)
template <int N>
struct Tower {
  static constexpr int T2 = N / 2, TPB = T2 * T2, NG = (TPB + 15) / 16;
  W2Lane c;
  uintptr_t a_x0, a_a, a_b, a_out;  // the board's base in each activation buffer (integers: a select
                                    // among pointers would make hipcc assume they may alias U)
  const float* u2all;
  const float* biasall;
  int nlayers;
  __device__ static __amdgpu_buffer_rsrc_t rsrc(uintptr_t a, int bytes) { return w2_rsrc((const float*)a, bytes); }
  // selections by bit masks (hipcc turns a select chain into a lookup table in scratch memory)
  __device__ static uintptr_t pick(bool c, uintptr_t a, uintptr_t b) {
    const uintptr_t m = (uintptr_t)0 - (uintptr_t)c;
    return (a & m) | (b & ~m);
  }
  __device__ __amdgpu_buffer_rsrc_t in_of(int layer) const {
    return rsrc(pick(layer == 0, a_x0, pick(layer & 1, a_a, a_b)), N * N * 256);
  }
  __device__ __amdgpu_buffer_rsrc_t out_of(int layer) const {
    return rsrc(pick(layer + 1 == nlayers, a_out, pick(layer & 1, a_b, a_a)), N * N * 256);
  }
  __device__ __amdgpu_buffer_rsrc_t res_of(int layer) const {  // the last layer's residual; 0s otherwise
    return rsrc(a_x0, layer + 1 == nlayers ? N * N * 256 : 0);
  }
  __device__ const f32x4* u_of(int layer) const {
    return reinterpret_cast<const f32x4*>(u2all + (size_t)layer * kW2UFloats) + (size_t)c.wave * 64 * kWave + c.l;
  }
  __device__ f32x4 bias_of(int layer) const {
    return *reinterpret_cast<const f32x4*>(biasall + layer * 64 + 16 * c.wave + 4 * (c.l >> 4));
  }
  __device__ void window(int grp, unsigned (&off)[16]) const {
    const int tile = grp * 16 + c.tt, ty = tile / T2;
    c.window(tile < TPB, N, 0, ty, tile - ty * T2, off);
  }
  __device__ int out_pixel(int grp) const {
    const int tile = grp * 16 + (c.l & 15), ty = tile / T2, tx = tile - ty * T2;
    return tile < TPB ? (2 * ty) * N + 2 * tx : -1;
  }
};

// One (layer, group) pair of the tower pipeline, MODE kW2First / kW2Mid / kW2Last (a layer's last
// group: the next pair is (layer + 1, 0) and U is refilled with the next layer's)
template <int M, bool WINDOW_IN_RAW, bool HEADS, int N>
__device__ __forceinline__ void tower_pair(const Tower<N>& t, f32x4 (&ur)[64], f32x4 (&raw)[16], f32x4& bias4,
                                           int layer, int grp, const HeadLane& hl, bool store_last) {
  const bool last = layer + 1 == t.nlayers, relu = last || !(layer & 1);
  // the next pair: (layer, grp + 1), or (layer + 1, 0) after a layer's last group (the last pair of
  // the tower re-reads its own window into the idle V buffer: unconditional work)
  const bool cross = M == kW2Last && !last;
  const int nl = cross ? layer + 1 : layer, ng = M == kW2Last ? (last ? grp : 0) : grp + 1;
  if (M == kW2Last) asm volatile("buffer_inv sc0" ::: "memory");  // next-layer windows: no stale L1 lines
  f32x4 acc[16];
  w2_group<M, WINDOW_IN_RAW>(t.c, ur, raw, t.u_of(layer), t.u_of(nl), t.in_of(nl), bias4, (layer * Tower<N>::NG + grp) & 1,
              [&](unsigned (&off)[16]) { t.window(ng, off); }, acc);
#if BK_WINO_STAMP
  const int l = t.c.l, wave = t.c.wave;
  if (layer == 2) W2STAMP(10 + grp, __builtin_amdgcn_s_memtime());
#endif
  if (last)  // the tower's last conv: + the tower input (a uniform branch), and the heads' 1x1 convs
    w2_epilogue_flags<true, HEADS>(t.c, acc, t.out_pixel(grp), N, 0.0f, t.res_of(layer), t.out_of(layer), store_last,
                                   &hl);
  else
    w2_epilogue_flags<false>(t.c, acc, t.out_pixel(grp), N, relu ? 0.0f : -__builtin_inff(), t.res_of(layer),
                             t.out_of(layer));
  if (M == kW2Last) {
    bias4 = t.bias_of(nl);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no load pending across the layer loop's back edge
  }
  __syncthreads();  // V[buf ^ 1] complete for the next pair; V[buf] free to be overwritten
#if BK_WINO_STAMP
  if (layer == 2) W2STAMP(3 + grp, __builtin_amdgcn_s_memtime());
#endif
}

// The stem conv (blokus_nnet.py:137, BN folded: conv3x3 8 -> 64 channels + bias + ReLU) of one
// board inside the tower launch: the planar observation staged zero-padded in LDS, then per wave
// (16 output channels) NN/16 pixel tiles x 18 k-steps of v_mfma_f32_16x16x4_f32 with A = im2col
// entries read from LDS at immediate offsets (k-step s = tap s/2, channels 4(s%2)..+3) and B =
// the packed weights in 18 registers (nets.pack_stem_tower); bias + ReLU into x0 (NHWC).
constexpr int kStemCin = 8;
template <int N>
__device__ __forceinline__ void tower_stem(float* lds, const float* __restrict__ obs_b, const float* __restrict__ wst,
                                           const float* __restrict__ bst, __amdgpu_buffer_rsrc_t x0r, int wave, int l) {
  constexpr int NP = N + 2, NN = N * N, TILES = (NN + 15) / 16;
  for (int i = threadIdx.x; i < kStemCin * NP * NP; i += kW2Threads) {
    const int ch = i / (NP * NP), r = i - ch * NP * NP, y = r / NP - 1, x = r - (r / NP) * NP - 1;
    lds[i] = (y >= 0 && y < N && x >= 0 && x < N) ? obs_b[ch * NN + y * N + x] : 0.0f;
  }
  float wb[18];
#pragma unroll
  for (int s = 0; s < 18; ++s) wb[s] = wst[(wave * 18 + s) * kWave + l];
  const int g = l >> 4, m = l & 15;
  const float bm = bst[16 * wave + m];
  __syncthreads();
  for (int tile = 0; tile < TILES; ++tile) {
    const int p = tile * 16 + m, pc = p < NN ? p : NN - 1, py = pc / N, px = pc - (pc / N) * N;
    const float* a = lds + g * NP * NP + py * NP + px;  // channel g, window top-left (padded)
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      const int t = s >> 1;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * (s & 1) * NP * NP + (t / 3) * NP + (t % 3)], wb[s], acc, 0, 0, 0);
    }
    // D: lane (g, m) holds pixels tile*16 + 4g + r, output channel 16 wave + m
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pix = tile * 16 + 4 * g + r;
      if (pix < NN)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, fmaxf(acc[r] + bm, 0.0f)), x0r,
                                              (unsigned)(pix * 64 + 16 * wave + m) * 4, 0, 0);
    }
  }
  // x0 complete and visible to the workgroup before the tower reads its windows
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  asm volatile("buffer_inv sc0" ::: "memory");
}

// The heads after the tower (k_tower_wino<N, true>): the 1x1 convs' weights, the value MLP, the
// outputs (policy features pf [B][2*NN] channel-major, values v [B][P]); out may be skipped.
struct TowerHeads {
  const float *wp, *bp, *wv, *bv, *w1t, *b1, *w2, *b2;
  int P;
  float* pf;
  float* v;
  int store_out;
  const float* obs;  // non-null: the stem runs first (k_tower_wino<N, true, true>) and x0 is its output
  const float* wstem;
  const float* bstem;
};

// The leaf net of board blockIdx.x: k_tower_wino's body. v_lds: [2 buf][16 s][16 p][16 t][4 g] (+ the heads' partials [NN][4][3] with HEADS).
template <int N, bool HEADS, bool STEM = false>
__device__ __forceinline__ void tower_forward(float* v_lds, const float* __restrict__ x0, float* hA, float* hB,
                                              float* __restrict__ out, const float* __restrict__ u2all,
                                              const float* __restrict__ biasall, int nlayers, const TowerHeads& hd) {
  static_assert(tower_pipeline_ok<N>(), "k_tower_wino: board too small for the cross-layer pipeline");
  constexpr int NG = Tower<N>::NG;
  const size_t board = (size_t)blockIdx.x * N * N * 64;
  Tower<N> t;
  t.c.v_lds = v_lds;
  t.c.wave = threadIdx.x >> 6;
  t.c.l = threadIdx.x & 63;
  t.c.tt = t.c.l & 15;
  t.c.sq = (t.c.wave << 2) | (t.c.l >> 4);
  const int l = t.c.l, wave = t.c.wave;
  W2STAMP(0, __builtin_amdgcn_s_memtime());
  W2STAMP(30, __builtin_amdgcn_s_memrealtime());
  // buffer resources of the board in each activation buffer, built once (selecting among
  // resources, never among pointers, keeps every access a buffer op on a uniform descriptor)
  t.a_x0 = (uintptr_t)(x0 + board);
  t.a_a = (uintptr_t)(hA + board);
  t.a_b = (uintptr_t)(hB + board);
  t.a_out = (uintptr_t)(out + board);
  t.u2all = u2all;
  t.biasall = biasall;
  t.nlayers = nlayers;
  t.c.xr = t.in_of(0);
  if (STEM) tower_stem<N>(v_lds, hd.obs + (size_t)blockIdx.x * kStemCin * N * N, hd.wstem, hd.bstem, t.c.xr, wave, l);
  // prologue: windows of pairs (0, 0) and (0, 1), layer 0's bias and U of k-steps 0, 1
  f32x4 ur[64];
  f32x4 raw[16];
  f32x4 bias4;
  {
    f32x4 raw0[16];
    unsigned off[16];
    t.window(0, off);
#pragma unroll
    for (int q = 0; q < 16; ++q) raw0[q] = t.c.ld(off[q]);
    t.window(1, off);
#pragma unroll
    for (int q = 0; q < 16; ++q) raw[q] = t.c.ld(off[q]);
    bias4 = t.bias_of(0);
    __builtin_amdgcn_sched_barrier(0);
    w2_load_u01(ur, t.u_of(0));
#pragma unroll
    for (int k = 0; k < 8; ++k) t.c.transform_part(raw0, 0, k);
  }
  __syncthreads();
  W2STAMP(1, __builtin_amdgcn_s_memtime());
  HeadLane hl;
  constexpr int NN = N * N;
  if (HEADS) {
    const int ch = 16 * wave + 4 * (l >> 4);
    hl.wp0 = *reinterpret_cast<const f32x4*>(hd.wp + ch);
    hl.wp1 = *reinterpret_cast<const f32x4*>(hd.wp + 64 + ch);
    hl.wv = *reinterpret_cast<const f32x4*>(hd.wv + ch);
    hl.hp = v_lds + 2 * kW2VBuf;
  }
  const bool so = !HEADS || hd.store_out;
  tower_pair<kW2First, true, HEADS>(t, ur, raw, bias4, 0, 0, hl, so);
  for (int grp = 1; grp < NG - 1; ++grp) tower_pair<kW2Mid, false, HEADS>(t, ur, raw, bias4, 0, grp, hl, so);
  tower_pair<kW2Last, false, HEADS>(t, ur, raw, bias4, 0, NG - 1, hl, so);
  for (int layer = 1; layer < nlayers; ++layer) {
    tower_pair<kW2First, false, HEADS>(t, ur, raw, bias4, layer, 0, hl, so);
    for (int grp = 1; grp < NG - 1; ++grp) tower_pair<kW2Mid, false, HEADS>(t, ur, raw, bias4, layer, grp, hl, so);
    tower_pair<kW2Last, false, HEADS>(t, ur, raw, bias4, layer, NG - 1, hl, so);
    if (layer == 2) W2STAMP(2, __builtin_amdgcn_s_memtime());
  }
  if (HEADS) {
    // the heads (blokus_nnet.py:146-150, BN folded), as k_resnet_heads but from the partials in hp:
    // pf = relu(1x1 conv + bp) (channel-major), vfeat = relu(value 1x1 conv + bv) in LDS, then
    // v = tanh(W2 relu(W1 vfeat + b1) + b2); the 4 waves sweep quarters of W1's inputs
    const float* hp = hl.hp;
    float* vfeat = v_lds;  // the V buffers are free now
    float* part = v_lds + NN;
    const int bi = blockIdx.x, tid = threadIdx.x;
    for (int i = tid; i < NN; i += kW2Threads) {
      const float* q = hp + i * 12;
      const float p0 = ((q[0] + q[3]) + q[6]) + q[9], p1 = ((q[1] + q[4]) + q[7]) + q[10],
                  pv = ((q[2] + q[5]) + q[8]) + q[11];
      hd.pf[(size_t)bi * 2 * NN + i] = fmaxf(p0 + hd.bp[0], 0.0f);
      hd.pf[(size_t)bi * 2 * NN + NN + i] = fmaxf(p1 + hd.bp[1], 0.0f);
      vfeat[i] = fmaxf(pv + hd.bv[0], 0.0f);
    }
    __syncthreads();
    const int q0 = (NN * wave) / 4, q1 = (NN * (wave + 1)) / 4;
    float acc0 = 0.f, acc1 = 0.f;
    int i = q0;
    for (; i + 10 <= q1; i += 10) {
      float w[10];
#pragma unroll
      for (int u = 0; u < 10; ++u) w[u] = hd.w1t[(size_t)(i + u) * 64 + l];
#pragma unroll
      for (int u = 0; u < 10; u += 2) {
        acc0 += w[u] * vfeat[i + u];
        acc1 += w[u + 1] * vfeat[i + u + 1];
      }
    }
    for (; i < q1; ++i) acc0 += hd.w1t[(size_t)i * 64 + l] * vfeat[i];
    part[wave * 64 + l] = acc0 + acc1;
    __syncthreads();
    if (wave == 0) {
      const float h = fmaxf(((part[l] + part[64 + l]) + (part[128 + l] + part[192 + l])) + hd.b1[l], 0.0f);
      for (int q = 0; q < hd.P; ++q) {
        const float sum = wave_sum_f(hd.w2[q * 64 + l] * h);
        if (l == 0) hd.v[(size_t)bi * hd.P + q] = tanhf(sum + hd.b2[q]);
      }
    }
  }
  W2STAMP(29, __builtin_amdgcn_s_memtime());
  W2STAMP(31, __builtin_amdgcn_s_memrealtime());
  (void)l;
  (void)wave;
}

}  // namespace
}  // namespace bk
