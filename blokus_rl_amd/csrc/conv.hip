// conv.hip — the leaf evaluator's 3x3 convolutions (ResNet of models/blokus_nnet.py:88-151, BN
// folded) as one fused fp32 MFMA kernel per layer: y = act(conv3x3(x, W) + b (+ r)).
//
// Shape: x [B][N][N][64] (CIN = 64, NHWC) or [B][CIN][N][N] (CIN = 4, 8: the observation
// planes), W 64 x CIN x 3 x 3, y [B][N][N][64] (NHWC). As a GEMM: M = B*N*N output pixels, N = 64 channels, K = 9*CIN. At the
// self-play batch (256 boards of 20x20, CIN = 64) that is 7.55 GFLOP per layer: MFMA-bound.
//
// Design (gfx950, f32-in MFMA v_mfma_f32_16x16x4_f32: 64 FLOP/clk/SIMD, exact f32):
//  * One 768-thread workgroup per CU (grid 256), 12 waves = 3 per SIMD. The whole packed weight
//    tensor sits in LDS (9*CIN*64*4 B = 147 KB at CIN=64), loaded once per launch and shared by
//    the 8 waves; every B operand is one conflict-free ds_read_b128 (the 4 output-channel
//    blocks of a k-step, pre-packed in MFMA lane order by the host).
//  * A wave owns a tile of 16 consecutive output pixels x all 64 channels: 4 independent 16x16
//    accumulators (dependent-latency 40 cycles < 4 x 32-cycle issue, so the MFMA pipe never
//    waits on itself). Its A operand comes straight from global memory: per tap, one CIN-wide
//    row per pixel, read as dwordx4 (CIN = 64; planar observation: VEC scalars) in a K order
//    permuted so each vector load feeds VEC consecutive k-steps; out-of-board taps read zeros
//    (padding 1). (A channel-blocked [B][4][NN][16] layout, whose loads are 1 KB contiguous,
//    measured 3-5% slower.)
//  * XCD-aware tiling: the 8 XCDs each take a contiguous eighth of the pixel tiles (whole boards,
//    3.2 MB of input at B=256) so a board's rows are fetched into one XCD's L2 and reused there
//    by all 9 taps; within an XCD each CU takes a contiguous run of tiles (its waves share board
//    rows in L1), and a CU's
//    leftover tiles are split into 16-channel quarters to even out the last round (k_conv3x3).
//  * Epilogue fused: + bias, + residual (the tower's skip connection), ReLU, one store pass.
// Accumulation order differs from MIOpen's (k-ordered fma chain per MFMA), so results agree
// with the MIOpen convolution to f32 rounding, not bitwise.
#include "../../include/blokus_engine.h"
#include "ctx.h"
#include "tower_dev.h"

#include <cstdlib>
#include <type_traits>

namespace bk {
namespace {

constexpr int kCout = 64;
constexpr int kConvThreads = 768;
constexpr int kConvDB = 8;  // B prefetch distance in k-steps
constexpr int kConvWaves = kConvThreads / kWave;

template <int VEC>
struct VecT;
template <>
struct VecT<1> {
  using T = float;
  __device__ static float at(const T& v, int) { return v; }
};
template <>
struct VecT<2> {
  using T = float2;
  __device__ static float at(const T& v, int r) { return r == 0 ? v.x : v.y; }
};
template <>
struct VecT<4> {
  using T = float4;
  __device__ static float at(const T& v, int r) { return r == 0 ? v.x : (r == 1 ? v.y : (r == 2 ? v.z : v.w)); }
};

// A run of output tiles owned by one wave. Tile i = 16 consecutive pixels from 16*tile(i) x NJ
// 16-channel blocks from block jblk(i), the whole K = 9*CIN reduction. k-steps per tap:
// S = CIN / 4 (4 k values per 16x16x4 MFMA); lane group g = lane>>4 holds k index g of each
// step; step s = q*VEC + r reads input channel cin = 4*VEC*q + VEC*g + r (the host packs W in
// the same order). Layouts: CIN = 64 input, the output and the residual are NHWC
// [B][N][N][64] (the leaf batch's channels_last activations); CIN = 4 / 8 input is planar
// [B][CIN][N][N] (the observation the search writes, read with no layout conversion).
//
// Software pipeline over the run's k-steps, carried across tiles (the body is fully unrolled,
// so every ring slot is a fixed register set and the s_waitcnt counts are exact):
//  * A: tap t's Q vector loads go to abuf[t % 3], issued at the start of tap t-2 — for taps 0
//    and 1 of the next tile, during taps 7 and 8 of the current one, before its epilogue
//    stores, so waiting on them never waits on the stores. Loads are unconditional (an in-board
//    address when the tap falls off the board) and the zero padding is a multiply at use, so
//    the compiler never sinks them into branches.
//  * B: one LDS read per k-step (ds_read_b128 = the 4 channel blocks), DB steps ahead; the
//    weights are the same for every tile, so the ring runs on across tile boundaries.
template <int CIN, int VEC, bool RELU, bool RES, int NJ, class TileOf, class JblkOf>
__device__ __forceinline__ void conv_run(const float* __restrict__ x, const f32x4* __restrict__ w_lds,
                                         const float* __restrict__ bias, const float* __restrict__ res,
                                         float* __restrict__ y, int N, int total_pix, int count, TileOf tile,
                                         JblkOf jblk) {
  constexpr int S = CIN / 4;
  constexpr int Q = CIN / (4 * VEC);
  constexpr int KS = 9 * S;
  constexpr int DB = S < kConvDB ? S : kConvDB;  // B prefetch distance in k-steps (divides KS)
  static_assert(KS % DB == 0, "ring must wrap at tile boundaries");
  using V = typename VecT<VEC>::T;
  using WT = typename std::conditional<NJ == 4, f32x4, float>::type;
  if (count <= 0) return;
  const int l = threadIdx.x & 63;
  const int m = l & 15, g = l >> 4;
  const int npix = N * N;
  struct Pix {
    int b, py, px;
    bool in;
  };
  auto pix_of = [&](int t) {
    Pix q;
    const int p = t * 16 + m;
    q.in = p < total_pix;
    q.b = q.in ? p / npix : 0;
    const int rem = p - q.b * npix;
    q.py = rem / N;
    q.px = rem - q.py * N;
    return q;
  };
  V abuf[3][Q];
  float keep[3];
  auto load_tap = [&](const Pix& pp, int tap, V* dst, float& kp) {
    const int yy = pp.py + tap / 3 - 1, xx = pp.px + tap % 3 - 1;
    const bool ok = pp.in && yy >= 0 && yy < N && xx >= 0 && xx < N;
    const int yc = ok ? yy : pp.py, xc = ok ? xx : pp.px;
    const int pix = yc * N + xc;
    kp = ok ? 1.0f : 0.0f;
    if constexpr (CIN % 16 == 0) {
      // NHWC input [B][NN][CIN]: channels 16q + 4g .. +3 of the pixel, one float4 per q
      const float* src = x + ((int64_t)pp.b * npix + pix) * CIN + 4 * g;
#pragma unroll
      for (int q = 0; q < Q; ++q) dst[q] = *reinterpret_cast<const V*>(src + 16 * q);
    } else {
      // planar input [B][CIN][NN] (the observation planes): channels VEC*g .. +VEC-1
      const float* src = x + ((int64_t)pp.b * CIN + VEC * g) * npix + pix;
      V v;
      float* vf = reinterpret_cast<float*>(&v);
#pragma unroll
      for (int r = 0; r < VEC; ++r) vf[r] = src[(int64_t)r * npix];
      dst[0] = v;
    }
  };
  int j0 = jblk(0);
  auto read_w = [&](int ks) -> WT {
    if constexpr (NJ == 4) {
      return w_lds[ks * kWave + l];
    } else {
      return reinterpret_cast<const float*>(w_lds + ks * kWave + l)[j0];
    }
  };
  float bias_r[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) bias_r[j] = bias[16 * (j0 + j) + m];
  Pix cur = pix_of(tile(0));
  WT wring[DB];
  load_tap(cur, 0, abuf[0], keep[0]);
  load_tap(cur, 1, abuf[1], keep[1]);
#pragma unroll
  for (int s = 0; s < DB; ++s) wring[s] = read_w(s);
  for (int i = 0; i < count; ++i) {
    const int t = tile(i);
    const bool more = i + 1 < count;
    const Pix nxt = pix_of(more ? tile(i + 1) : t);
    f32x4 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
      for (int sl = 0; sl < S; ++sl) {
        const int ks = tap * S + sl;
        if (sl == 0) {
          if (tap + 2 < 9) load_tap(cur, tap + 2, abuf[(tap + 2) % 3], keep[(tap + 2) % 3]);
          else if (more) load_tap(nxt, tap + 2 - 9, abuf[(tap + 2) % 3], keep[(tap + 2) % 3]);
        }
        const WT w = wring[ks % DB];
        wring[ks % DB] = read_w((ks + DB) % KS);
        const float av = VecT<VEC>::at(abuf[tap % 3][sl / VEC], sl % VEC) * keep[tap % 3];
        if constexpr (NJ == 4) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, w[0], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, w[1], acc[1], 0, 0, 0);
          acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, w[2], acc[2], 0, 0, 0);
          acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, w[3], acc[3], 0, 0, 0);
        } else {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, w, acc[0], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // D layout: lane l holds rows (pixels) 4g + v, column (channel) m of each 16x16 block
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int po = t * 16 + 4 * g + v;
      if (po < total_pix) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const size_t o = (size_t)po * kCout + 16 * (j0 + j) + m;
          float val = acc[j][v] + bias_r[j];
          if (RES) val = val + res[o];
          if (RELU) val = fmaxf(val, 0.0f);
          y[o] = val;
        }
      }
    }
    cur = nxt;
    if constexpr (NJ == 1) {  // quarter tiles may change channel block: refresh B ring + bias
      if (more && jblk(i + 1) != j0) {
        j0 = jblk(i + 1);
        bias_r[0] = bias[16 * j0 + m];
#pragma unroll
        for (int s = 0; s < DB; ++s) wring[s] = read_w(s);
      }
    }
  }
}

// Work split: the 8 XCDs take contiguous eighths of the 16-pixel tiles; inside an XCD, each CU
// takes a contiguous run of them. A CU's waves take whole tiles round-robin for
// R = floor(T_cu / waves) rounds; the L < waves leftover tiles are cut into 4L quarter tiles
// (16 channels each) dealt over the waves, so no SIMD carries a whole extra tile at the end.
template <int CIN, int VEC, bool RELU, bool RES>
__global__ __launch_bounds__(kConvThreads) void k_conv3x3(const float* __restrict__ x, const f32x4* __restrict__ wp,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ res, float* __restrict__ y,
                                                          int N, int total_pix) {
  constexpr int S = CIN / 4;
  extern __shared__ __attribute__((aligned(16))) f32x4 w_lds[];  // [9][S][64 lanes] x (4 channel blocks)
  const int tiles = (total_pix + 15) >> 4;
  const int nxcd = 8;
  const int xcd = blockIdx.x % nxcd, cu = blockIdx.x / nxcd, ncu = gridDim.x / nxcd;
  const int t_begin = (int)((int64_t)tiles * xcd / nxcd), t_end = (int)((int64_t)tiles * (xcd + 1) / nxcd);
  if ((int64_t)(t_end - t_begin) * (cu + 1) / ncu == (int64_t)(t_end - t_begin) * cu / ncu) return;  // no tiles here
  for (int i = threadIdx.x; i < 9 * S * kWave; i += kConvThreads) w_lds[i] = wp[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  // contiguous tiles per CU: its waves work on neighbouring 16-pixel strips at the same time,
  // so the board rows their 9 taps read are shared in the CU's L1
  const int range = t_end - t_begin;
  const int c_lo = (int)((int64_t)range * cu / ncu), c_hi = (int)((int64_t)range * (cu + 1) / ncu);
  const int t_cu = c_hi - c_lo;
  const int rounds = t_cu / kConvWaves;
  const int left = t_cu - rounds * kConvWaves;
  const int base = t_begin + c_lo;
  conv_run<CIN, VEC, RELU, RES, 4>(
      x, w_lds, bias, res, y, N, total_pix, rounds, [&](int r) { return base + r * kConvWaves + wave; },
      [](int) { return 0; });
  const int nq = wave < 4 * left ? (4 * left - wave + kConvWaves - 1) / kConvWaves : 0;
  conv_run<CIN, VEC, RELU, RES, 1>(
      x, w_lds, bias, res, y, N, total_pix, nq,
      [&](int i) { return base + rounds * kConvWaves + (wave + i * kConvWaves) / 4; },
      [&](int i) { return (wave + i * kConvWaves) % 4; });
}

template <int CIN, int VEC>
int launch_conv(const float* x, const f32x4* wp, const float* b, const float* r, float* y, int N, int total,
                int relu, hipStream_t s, int blocks) {
  const size_t lds = sizeof(f32x4) * 9 * (CIN / 4) * kWave;
  if (relu && r)
    hipLaunchKernelGGL((k_conv3x3<CIN, VEC, true, true>), dim3(blocks), dim3(kConvThreads), lds, s, x, wp, b, r, y, N,
                       total);
  else if (relu)
    hipLaunchKernelGGL((k_conv3x3<CIN, VEC, true, false>), dim3(blocks), dim3(kConvThreads), lds, s, x, wp, b, r, y,
                       N, total);
  else if (r)
    hipLaunchKernelGGL((k_conv3x3<CIN, VEC, false, true>), dim3(blocks), dim3(kConvThreads), lds, s, x, wp, b, r, y,
                       N, total);
  else
    hipLaunchKernelGGL((k_conv3x3<CIN, VEC, false, false>), dim3(blocks), dim3(kConvThreads), lds, s, x, wp, b, r, y,
                       N, total);
  return launch_check("k_conv3x3");
}

// ---------------------------------------------------------------------------------------------
// Winograd F(2x2, 3x3) form for CIN = 64 and even N (the 20x20 self-play net): all arithmetic
// f32 (the f32 MFMA is an exact fmaf chain), 2.25x fewer multiplies than the direct form.
// Each output 2x2 tile t (B * (N/2)^2 of them) reads its 4x4 input window d (zero padded), and
//   y_t = A^T [ sum_cin U[cin] (.) (B^T d_cin B) ] A,   U = G g G^T (host, fp64 -> f32),
// i.e. 16 independent GEMMs (one per transform position p = 4i + j) of [tiles x 64] x [64 x 64].
// Mapping: a wave owns 16 tiles (MFMA columns) x KB blocks of 16 output channels (MFMA rows) x
// all 16 positions = 16 KB accumulators. At k-step s lane (g = l>>4, m = l&15) takes channel
// 16g + s of tile m's 16 window pixels (float4 loads: 4 steps each), transforms them in
// registers (32 adds: the B operands of all 16 positions at once); the A operands (U) come from
// LDS (conflict-free ds_read_b32, 256 B per (block, p, s)). Step s's MFMAs are interleaved with
// step s+1's LDS reads and transform. After the last step each lane holds all 16 positions of
// channels 4g..4g+3 (of each block) of its own tile: the output transform, bias, residual and
// ReLU run in registers, one float4 store per output pixel and block. The workgroup (one per
// CU) holds U for its 32-channel half (131 KB of LDS); blocks b and b + 8 sit on the same XCD
// with opposite halves, and each XCD takes a contiguous eighth of the tile groups, so both
// halves of a window are fetched into one L2.
//   KB = 1: 8 waves (2 per SIMD, 256 registers), waves w and w^1 the two blocks of a group.
//   KB = 2: 4 waves (1 per SIMD, 512 registers), a wave both blocks.
constexpr int kWinoKB = 1;
constexpr int kWinoThreads = kWinoKB == 1 ? 512 : 256;
constexpr int kWinoHalf = 2 * 16 * 16 * kWave;  // floats of U per 32-channel half: [2 blk][16 p][16 s][64]

template <int KB, bool RELU, bool RES>
__global__ __launch_bounds__(KB == 1 ? 512 : 256, 1) void k_conv3x3_wino(const float* __restrict__ x,
                                                                         const float* __restrict__ uw,
                                                                         const float* __restrict__ bias,
                                                                         const float* __restrict__ res,
                                                                         float* __restrict__ y, int N, int tiles) {
  constexpr int kThreads = KB == 1 ? 512 : 256;
  constexpr int kSlots = 4;            // groups in flight per workgroup
  constexpr int NBUF = KB == 1 ? 1 : 2;  // float4 window buffers (A prefetch depth)
  extern __shared__ __attribute__((aligned(16))) float u_lds[];  // [2 blk][16 p][16 s][64 lanes]
  const int half = (blockIdx.x >> 3) & 1, xcd = blockIdx.x & 7;
  const int cu = blockIdx.x >> 4, ncu = gridDim.x >> 4;
  const int groups = (tiles + 15) >> 4;
  const int g_begin = (int)((int64_t)groups * xcd / 8), g_end = (int)((int64_t)groups * (xcd + 1) / 8);
  const int range = g_end - g_begin;
  const int c_lo = g_begin + (int)((int64_t)range * cu / ncu), c_hi = g_begin + (int)((int64_t)range * (cu + 1) / ncu);
  if (c_lo == c_hi) return;
  {
    const float4* src = reinterpret_cast<const float4*>(uw + (size_t)half * kWinoHalf);
    float4* dst = reinterpret_cast<float4*>(u_lds);
    for (int i = threadIdx.x; i < kWinoHalf / 4; i += kThreads) dst[i] = src[i];
  }
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  WSTAMP(0);
  __syncthreads();
  WSTAMP(1);
  const int m = l & 15, g = l >> 4;
  const int kb0 = KB == 1 ? (wave & 1) : 0, slot = KB == 1 ? (wave >> 1) : wave;
  const int T2 = N >> 1, tpb = T2 * T2;
  const float* ub = u_lds + kb0 * (16 * 16 * kWave) + l;
  float bias_k[KB][4];
#pragma unroll
  for (int k = 0; k < KB; ++k)
#pragma unroll
    for (int vv = 0; vv < 4; ++vv) bias_k[k][vv] = bias[32 * half + 16 * (kb0 + k) + 4 * g + vv];
  // the input through a buffer descriptor: 32-bit offsets, and out-of-range reads return 0 —
  // a window pixel off the board (zero padding) or past the last tile gets an offset beyond the
  // buffer, so padding costs nothing in the inner loop
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, tiles * 1024, 0x00020000);
  constexpr unsigned kOut = 0x7fff0000u;
  // byte offsets of this lane's tile (MFMA column m) window: 16 pixels, channel 16g
  auto window = [&](int grp, unsigned (&off)[16]) {
    const int tile = grp * 16 + m;
    const bool tv = tile < tiles;
    const int b = tv ? tile / tpb : 0, r = tv ? tile - b * tpb : 0;
    const int ty = r / T2, tx = r - ty * T2;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int yy = 2 * ty - 1 + i, xx = 2 * tx - 1 + j;
        const bool v = tv && yy >= 0 && yy < N && xx >= 0 && xx < N;
        off[4 * i + j] = v ? (unsigned)(((b * N + yy) * N + xx) * 256 + 64 * g) : kOut;
      }
  };
  auto ld = [&](unsigned o) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
  };
  unsigned off[16];
  f32x4 raw[NBUF][16];
  int grp = c_lo + slot;
  if (grp < c_hi) {
    window(grp, off);
#pragma unroll
    for (int q = 0; q < 16; ++q) raw[0][q] = ld(off[q]);
  }
  int task = 0;
  for (; grp < c_hi; grp += kSlots, ++task) {
    WSTAMP(2 + 3 * task);
    f32x4 acc[KB][16];
#pragma unroll
    for (int k = 0; k < KB; ++k)
#pragma unroll
      for (int p = 0; p < 16; ++p) acc[k][p] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bw[2][16 * KB];
#pragma unroll
    for (int kp = 0; kp < 16 * KB; ++kp) bw[0][kp] = ub[(kp * 16) * kWave];
    const int nxt = grp + kSlots;
    // A loads of quad qd (channels 16g + 4qd .. +3) into buf, or the next group's first quad
    auto load_quad = [&](int qd, int buf) {
      if (qd < 4) {
#pragma unroll
        for (int q = 0; q < 16; ++q) raw[buf][q] = ld(off[q] + 16 * qd);
      } else if (nxt < c_hi) {
        unsigned offn[16];
        window(nxt, offn);
#pragma unroll
        for (int q = 0; q < 16; ++q) raw[buf][q] = ld(offn[q]);
      }
    };
    // B^T d B of k-step s: the B operands of its 16 positions
    auto transform = [&](int s, float (&v)[16]) {
      float d[16], t[16];
      const int r = s & 3;
#pragma unroll
      for (int q = 0; q < 16; ++q) d[q] = raw[NBUF == 2 ? (s >> 2) & 1 : 0][q][r];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[0 + j] = d[0 + j] - d[8 + j];
        t[4 + j] = d[4 + j] + d[8 + j];
        t[8 + j] = d[8 + j] - d[4 + j];
        t[12 + j] = d[4 + j] - d[12 + j];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[4 * i + 0] = t[4 * i + 0] - t[4 * i + 2];
        v[4 * i + 1] = t[4 * i + 1] + t[4 * i + 2];
        v[4 * i + 2] = t[4 * i + 2] - t[4 * i + 1];
        v[4 * i + 3] = t[4 * i + 1] - t[4 * i + 3];
      }
    };
    float vc[16];
    transform(0, vc);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (NBUF == 2 && (s & 3) == 0) load_quad((s >> 2) + 1, ((s >> 2) + 1) & 1);
      float vn[16];
      if (s + 1 < 16) {
#pragma unroll
        for (int kp = 0; kp < 16 * KB; ++kp) bw[(s + 1) & 1][kp] = ub[(kp * 16 + s + 1) * kWave];
        transform(s + 1, vn);
        // single buffer: the quad's last transform done -> refill it with the next quad
        if (NBUF == 1 && ((s + 1) & 3) == 3) load_quad(((s + 1) >> 2) + 1, 0);
      }
      // U as the A operand (rows = output channels), the window as B (columns = tiles):
      // D[channel 4g + vv][tile m]
#pragma unroll
      for (int k = 0; k < KB; ++k)
#pragma unroll
        for (int p = 0; p < 16; ++p)
          acc[k][p] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[s & 1][k * 16 + p], vc[p], acc[k][p], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");  // keep each step's loads in its step (no hoisting across steps)
      if (s + 1 < 16) {
#pragma unroll
        for (int p = 0; p < 16; ++p) vc[p] = vn[p];
      }
    }
    WSTAMP(3 + 3 * task);
    // A^T M A for (tile m; channels 32h + 16(kb0 + k) + 4g + vv) + bias (+ residual), ReLU
    const int tile = grp * 16 + m;
    if (tile < tiles) {
      const int ob = tile / tpb, orr = tile - ob * tpb;
      const int oy = 2 * (orr / T2), ox = 2 * (orr - (orr / T2) * T2);
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        float yv[4][4];  // [pixel 2i + j][vv]
#pragma unroll
        for (int vv = 0; vv < 4; ++vv) {
          float u2[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            u2[j] = acc[k][j][vv] + acc[k][4 + j][vv] + acc[k][8 + j][vv];
            u2[4 + j] = acc[k][4 + j][vv] - acc[k][8 + j][vv] - acc[k][12 + j][vv];
          }
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            yv[2 * i][vv] = u2[4 * i + 0] + u2[4 * i + 1] + u2[4 * i + 2] + bias_k[k][vv];
            yv[2 * i + 1][vv] = u2[4 * i + 1] - u2[4 * i + 2] - u2[4 * i + 3] + bias_k[k][vv];
          }
        }
#pragma unroll
        for (int px = 0; px < 4; ++px) {
          const size_t o =
              ((size_t)(ob * N + oy + (px >> 1)) * N + ox + (px & 1)) * 64 + 32 * half + 16 * (kb0 + k) + 4 * g;
          float4 out = make_float4(yv[px][0], yv[px][1], yv[px][2], yv[px][3]);
          if (RES) {
            const float4 rr = *reinterpret_cast<const float4*>(res + o);
            out.x += rr.x;
            out.y += rr.y;
            out.z += rr.z;
            out.w += rr.w;
          }
          if (RELU) {
            out.x = fmaxf(out.x, 0.0f);
            out.y = fmaxf(out.y, 0.0f);
            out.z = fmaxf(out.z, 0.0f);
            out.w = fmaxf(out.w, 0.0f);
          }
          *reinterpret_cast<float4*>(y + o) = out;
        }
      }
    }
    if (nxt < c_hi) window(nxt, off);
    WSTAMP(4 + 3 * task);
  }
}

// ---------------------------------------------------------------------------------------------
// Winograd F(2x2, 3x3), form 2 (the default): the same arithmetic as k_conv3x3_wino, but the
// transformed weights U stay in REGISTERS and the transformed input windows V go through LDS,
// so every input window is loaded and transformed once per launch (form 1 does it 4x: two
// channel halves on two CUs x two waves) and one CU covers all 64 output channels.
//  * One 256-thread workgroup per CU (4 waves, 1 per SIMD). Wave kb holds U for output channels
//    16kb..16kb+15 in AGPRs: per lane the A operands of all 16 positions x 16 k-steps (256
//    registers), loaded once per launch (64 KB per wave, L2-resident).
//  * Work unit = a group of 16 output tiles (one MFMA column each); the 8 XCDs take contiguous
//    eighths of the groups, each CU a contiguous run of them (its windows share board rows in
//    L1/L2). Per group the CU's 256 threads each transform one (tile, 4-channel quad): 16
//    float4 window loads (buffer loads; off-board and past-the-end pixels read 0), B^T d B in
//    registers on channel pairs (v_pk_add_f32), 16 ds_write_b128 into V[s][p][t][4 channels].
//  * MFMA loop (per group, per wave): 16 k-steps x 16 positions of v_mfma_f32_16x16x4_f32,
//    A = U straight from AGPRs (inline asm), B = V (16 conflict-free ds_read_b32 per step, one
//    step ahead), accumulators in VGPRs; the bias is the initial accumulator of position (1,1),
//    which the output transform adds to all four pixels of a tile.
//  * f32 MFMAs run on the SIMD's vector ALUs: a VALU instruction beside them is not hidden, and
//    each switch between MFMA and VALU costs ~10 cycles (measured, tools/probe/mfma_fill.hip).
//    So the loop body is MFMAs and LDS reads only; the VALU work comes in three batches per
//    group, all on packed pairs: the window offsets (step 0), the next group's input transform
//    (after step 7; its loads were issued at step 0) and the output transform epilogue.
//  * V is double-buffered in LDS (2 x 64 KB): one barrier per group.
// (form 2 and the tower's device code: tower_dev.h)

template <int N, bool HEADS, bool STEM = false>
__global__ __launch_bounds__(kW2Threads, 1) void k_tower_wino(const float* __restrict__ x0, float* hA, float* hB,
                                                              float* __restrict__ out,
                                                              const float* __restrict__ u2all,
                                                              const float* __restrict__ biasall, int nlayers,
                                                              TowerHeads hd) {
  extern __shared__ __attribute__((aligned(16))) float v_lds[];
  tower_forward<N, HEADS, STEM>(v_lds, x0, hA, hB, out, u2all, biasall, nlayers, hd);
}

// BK_CONV_DIRECT=1 forces the direct form for every shape (tests compare the two);
// BK_CONV_WINO=1 selects Winograd form 1 (k_conv3x3_wino) instead of form 2
bool direct_only() {
  const char* e = getenv("BK_CONV_DIRECT");
  return e && *e && *e != '0';
}
bool wino_form1() {
  const char* e = getenv("BK_CONV_WINO");
  return e && *e == '1';
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

#if BK_WINO_STAMP
// diagnostics build only: copy the per-wave stamps [256 blocks][8 waves][32] to host memory
int bk_wino_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wino_stamps), sizeof(g_wino_stamps)) == hipSuccess ? 0 : -1;
}
int bk_wino_stamps_clear() {
  static unsigned long long zeros[256 * 8 * kStampPerWave];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_wino_stamps), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif

int bk_conv3x3_packed_floats(int cin) {
  // cin 64: the direct form's 9*64*64 operands, then the Winograd form's U (2 halves)
  return (cin == 4 || cin == 8) ? 9 * cin * kCout : cin == 64 ? 9 * 64 * kCout + 2 * kWinoHalf + kW2UFloats : -1;
}

int bk_tower_u_floats(void) { return kW2UFloats; }
int bk_tower_supported(int N) { return N == 14 || N == 20; }

namespace {
int tower_launch(const float* x0, int B, int N, int nlayers, const float* u2all, const float* biasall, float* hA,
                 float* hB, float* out, const TowerHeads* hd, void* stream) {
  BK_REQUIRE(x0 && u2all && biasall && hA && hB && B >= 0 && nlayers >= 1, "bad argument");
  BK_REQUIRE(out || (hd && !hd->store_out), "bad argument");
  BK_REQUIRE(bk_tower_supported(N), "bk_resnet_tower: N must be 14 or 20");
  BK_REQUIRE(((uintptr_t)x0 & 15u) == 0 && ((uintptr_t)hA & 15u) == 0 && ((uintptr_t)hB & 15u) == 0 &&
                 ((uintptr_t)out & 15u) == 0 && ((uintptr_t)u2all & 15u) == 0 && ((uintptr_t)biasall & 15u) == 0,
             "bk_resnet_tower: 16-byte aligned buffers");
  BK_REQUIRE((int64_t)N * N * 256 < (1ll << 31), "bk_resnet_tower: board too large");
  if (B == 0) return BK_OK;
  // V buffers (128 KB), then the heads' per-pixel partials [NN][4 waves][3]
  const int lds = (int)(sizeof(float) * (2 * kW2VBuf + (hd ? N * N * 12 : 0)));
  {
    const void* fns[6] = {(const void*)k_tower_wino<14, false>, (const void*)k_tower_wino<20, false>,
                          (const void*)k_tower_wino<14, true>,  (const void*)k_tower_wino<20, true>,
                          (const void*)k_tower_wino<14, true, true>, (const void*)k_tower_wino<20, true, true>};
    if (set_max_dynamic_lds(fns, 6, (int)(sizeof(float) * (2 * kW2VBuf + 20 * 20 * 12))) != BK_OK) return BK_EHIP;
  }
  hipStream_t s = (hipStream_t)stream;
  const TowerHeads h = hd ? *hd : TowerHeads{};
  if (N == 20 && hd && hd->obs)
    hipLaunchKernelGGL((k_tower_wino<20, true, true>), dim3(B), dim3(kW2Threads), lds, s, x0, hA, hB, out, u2all,
                       biasall, nlayers, h);
  else if (N == 14 && hd && hd->obs)
    hipLaunchKernelGGL((k_tower_wino<14, true, true>), dim3(B), dim3(kW2Threads), lds, s, x0, hA, hB, out, u2all,
                       biasall, nlayers, h);
  else if (N == 20 && hd)
    hipLaunchKernelGGL((k_tower_wino<20, true>), dim3(B), dim3(kW2Threads), lds, s, x0, hA, hB, out, u2all, biasall,
                       nlayers, h);
  else if (N == 20)
    hipLaunchKernelGGL((k_tower_wino<20, false>), dim3(B), dim3(kW2Threads), lds, s, x0, hA, hB, out, u2all, biasall,
                       nlayers, h);
  else if (hd)
    hipLaunchKernelGGL((k_tower_wino<14, true>), dim3(B), dim3(kW2Threads), lds, s, x0, hA, hB, out, u2all, biasall,
                       nlayers, h);
  else
    hipLaunchKernelGGL((k_tower_wino<14, false>), dim3(B), dim3(kW2Threads), lds, s, x0, hA, hB, out, u2all, biasall,
                       nlayers, h);
  return launch_check("k_tower_wino");
}
}  // namespace

int bk_resnet_tower(const float* x0, int B, int N, int nlayers, const float* u2all, const float* biasall, float* hA,
                    float* hB, float* out, void* stream) {
  BK_REQUIRE(out, "bad argument");
  return tower_launch(x0, B, N, nlayers, u2all, biasall, hA, hB, out, nullptr, stream);
}

int bk_resnet_tower_heads(const float* x0, int B, int N, int nlayers, const float* u2all, const float* biasall,
                          float* hA, float* hB, float* out, const float* wp, const float* bp, const float* wv,
                          const float* bv, const float* w1t, const float* b1, const float* w2, const float* b2, int P,
                          float* pf, float* vout, void* stream) {
  BK_REQUIRE(wp && bp && wv && bv && w1t && b1 && w2 && b2 && pf && vout && P > 0, "bad argument");
  BK_REQUIRE(((uintptr_t)wp & 15u) == 0 && ((uintptr_t)wv & 15u) == 0, "bk_resnet_tower_heads: 16-byte aligned wp, wv");
  TowerHeads h{wp, bp, wv, bv, w1t, b1, w2, b2, P, pf, vout, out ? 1 : 0, nullptr, nullptr, nullptr};
  return tower_launch(x0, B, N, nlayers, u2all, biasall, hA, hB, out, &h, stream);
}

int bk_stem_tower_u_floats(void) { return 4 * 18 * kWave; }

int bk_resnet_stem_tower_heads(const float* obs, int B, int N, int cin, const float* wstem, const float* bstem,
                               int nlayers, const float* u2all, const float* biasall, float* x0, float* hA, float* hB,
                               float* out, const float* wp, const float* bp, const float* wv, const float* bv,
                               const float* w1t, const float* b1, const float* w2, const float* b2, int P, float* pf,
                               float* vout, void* stream) {
  BK_REQUIRE(obs && wstem && bstem && x0, "bad argument");
  BK_REQUIRE(cin == kStemCin, "bk_resnet_stem_tower_heads: the stem takes 8 observation planes");
  BK_REQUIRE(wp && bp && wv && bv && w1t && b1 && w2 && b2 && pf && vout && P > 0, "bad argument");
  BK_REQUIRE(((uintptr_t)wp & 15u) == 0 && ((uintptr_t)wv & 15u) == 0, "bk_resnet_stem_tower_heads: 16-byte aligned wp, wv");
  TowerHeads h{wp, bp, wv, bv, w1t, b1, w2, b2, P, pf, vout, out ? 1 : 0, obs, wstem, bstem};
  return tower_launch(x0, B, N, nlayers, u2all, biasall, hA, hB, out, &h, stream);
}

int bk_conv3x3_form(int N, int cin) { return cin == 64 && N % 2 == 0 && !direct_only() ? 1 : 0; }

int bk_conv3x3(const float* x, int B, int N, int cin, const float* wpacked, const float* bias, const float* residual,
               int relu, float* y, void* stream) {
  BK_REQUIRE(x && wpacked && bias && y && B >= 0 && N > 0 && N <= 32, "bad argument");
  BK_REQUIRE(cin == 4 || cin == 8 || cin == 64, "bk_conv3x3: cin must be 4, 8 or 64");
  BK_REQUIRE(((uintptr_t)x & 15u) == 0 && ((uintptr_t)wpacked & 15u) == 0, "bk_conv3x3: 16-byte aligned x, weights");
  if (B == 0) return BK_OK;
  const int64_t total = (int64_t)B * N * N;
  BK_REQUIRE(total < (1ll << 30), "bk_conv3x3: batch too large");
  static int blocks = 0;
  if (!blocks) {
    int dev = 0, cus = 256;
    if (hip_check(hipGetDevice(&dev), "hipGetDevice") != BK_OK) return BK_EHIP;
    if (hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute") !=
        BK_OK)
      return BK_EHIP;
    blocks = (cus / 8) * 8 > 0 ? (cus / 8) * 8 : 8;
  }
  const f32x4* wp = reinterpret_cast<const f32x4*>(wpacked);
  hipStream_t s = (hipStream_t)stream;
  if (cin == 64) {
    {  // 147 KB of dynamic LDS (above the 64 KB default)
      const int bytes = (int)(sizeof(f32x4) * 9 * 16 * kWave);
      const void* fns[4] = {(const void*)k_conv3x3<64, 4, true, true>, (const void*)k_conv3x3<64, 4, true, false>,
                            (const void*)k_conv3x3<64, 4, false, true>, (const void*)k_conv3x3<64, 4, false, false>};
      if (set_max_dynamic_lds(fns, 4, bytes) != BK_OK) return BK_EHIP;
    }
    if (bk_conv3x3_form(N, cin) == 1 && !wino_form1()) {
      const int lds = (int)(sizeof(float) * 2 * kW2VBuf);
      {
        const void* fns[4] = {(const void*)k_conv3x3_wino2<true, true>, (const void*)k_conv3x3_wino2<true, false>,
                              (const void*)k_conv3x3_wino2<false, true>, (const void*)k_conv3x3_wino2<false, false>};
        if (set_max_dynamic_lds(fns, 4, lds) != BK_OK) return BK_EHIP;
      }
      BK_REQUIRE(total * 64 < (1ll << 31), "bk_conv3x3: batch too large");
      const float* u2 = wpacked + 9 * 64 * kCout + 2 * kWinoHalf;
      const int tiles = (int)(total / 4);
      const int g = blocks >= 8 ? blocks / 8 * 8 : 8;
      if (relu && residual)
        hipLaunchKernelGGL((k_conv3x3_wino2<true, true>), dim3(g), dim3(kW2Threads), lds, s, x, u2, bias, residual, y, N,
                           tiles);
      else if (relu)
        hipLaunchKernelGGL((k_conv3x3_wino2<true, false>), dim3(g), dim3(kW2Threads), lds, s, x, u2, bias, residual, y, N,
                           tiles);
      else if (residual)
        hipLaunchKernelGGL((k_conv3x3_wino2<false, true>), dim3(g), dim3(kW2Threads), lds, s, x, u2, bias, residual, y,
                           N, tiles);
      else
        hipLaunchKernelGGL((k_conv3x3_wino2<false, false>), dim3(g), dim3(kW2Threads), lds, s, x, u2, bias, residual, y,
                           N, tiles);
      return launch_check("k_conv3x3_wino2");
    }
    if (bk_conv3x3_form(N, cin) == 1) {
      const int lds = (int)(sizeof(float) * kWinoHalf);
      {
        const void* fns[4] = {(const void*)k_conv3x3_wino<kWinoKB, true, true>, (const void*)k_conv3x3_wino<kWinoKB, true, false>,
                              (const void*)k_conv3x3_wino<kWinoKB, false, true>, (const void*)k_conv3x3_wino<kWinoKB, false, false>};
        if (set_max_dynamic_lds(fns, 4, lds) != BK_OK) return BK_EHIP;
      }
      BK_REQUIRE(total * 64 < (1ll << 31), "bk_conv3x3: batch too large");
      const float* uw = wpacked + 9 * 64 * kCout;
      const int tiles = (int)(total / 4);
      const int g = blocks >= 16 ? blocks / 16 * 16 : 16;
      if (relu && residual)
        hipLaunchKernelGGL((k_conv3x3_wino<kWinoKB, true, true>), dim3(g), dim3(kWinoThreads), lds, s, x, uw, bias, residual, y, N,
                           tiles);
      else if (relu)
        hipLaunchKernelGGL((k_conv3x3_wino<kWinoKB, true, false>), dim3(g), dim3(kWinoThreads), lds, s, x, uw, bias, residual, y,
                           N, tiles);
      else if (residual)
        hipLaunchKernelGGL((k_conv3x3_wino<kWinoKB, false, true>), dim3(g), dim3(kWinoThreads), lds, s, x, uw, bias, residual, y,
                           N, tiles);
      else
        hipLaunchKernelGGL((k_conv3x3_wino<kWinoKB, false, false>), dim3(g), dim3(kWinoThreads), lds, s, x, uw, bias, residual,
                           y, N, tiles);
      return launch_check("k_conv3x3_wino");
    }
    return launch_conv<64, 4>(x, wp, bias, residual, y, N, (int)total, relu, s, blocks);
  }
  if (cin == 8) return launch_conv<8, 2>(x, wp, bias, residual, y, N, (int)total, relu, s, blocks);
  return launch_conv<4, 1>(x, wp, bias, residual, y, N, (int)total, relu, s, blocks);
}

}  // extern "C"
