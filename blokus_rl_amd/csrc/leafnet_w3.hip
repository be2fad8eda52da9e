// leafnet_w3.hip — the leaf ResNet (models/blokus_nnet.py:88-151, eval-mode BN folded) of one
// 20x20 board per workgroup, with its residual tower as Winograd F(2x2,3x3) convolutions on the
// split-f16 MFMA products of k_leafnet_x3 (leafnet.hip): every fp32 operand x = hi + lo (two f16
// halves, 22 significant bits), each product hi*hi + lo*hi + hi*lo on v_mfma_f32_16x16x32_f16
// with f32 accumulation. The transform domain needs 16 products per 2x2 output tile where the
// direct form needs 36: 672 MFMAs per wave and conv instead of 1350.
//
// Work split (the channel split): wave w owns output channels 16w..16w+15 for all 16 transform
// positions, its share of U = G g G^T (hi and lo, 16 positions x 2 K-chunks of 32 input
// channels: 256 registers) in AGPRs for the whole conv. A lane's accumulators then hold all 16
// positions of one (tile, 4 output channels), so the output transform A^T M A, bias, ReLU and the
// next layer's scaling stay in registers: no cross-wave reduction.
//
// LDS (160 KiB): [0, 32 KiB) the V ring — two units of 16 KiB, a unit = one transform row xi
// (4 positions) of one group of 16 tiles, all 64 input channels, split halves; [32 KiB, ...) the
// layer input as an fp32 grid of 22 x 22 zero-haloed pixels x 64 channels (256 B a pixel, channel
// quad j of column C at position j ^ (((C - 1) >> 1) & 7)). The 100 tiles of a 20x20 board form 7
// groups of 16 (the last holds 4; its spare columns repeat tile 99 and are never written out).
// Per unit: one barrier; the MFMAs of the unit's 4 positions read their B fragments from the
// ring, while all 256 threads build the NEXT unit's V (thread = one tile x 4 input channels:
// B^T d B for one xi from two window rows, split, written to the other ring slot). Outputs of a
// group are held in registers until no later V of the same layer reads their pixels
// (tools/w3/lds_plan.py: the write schedule and the bank-conflict check of every access), then
// written into the grid in place. Operand scaling as x3: U per output channel on the host, the
// activations per board and layer from the bound |y| <= A max|x| + B (nets.pack_x3), here into
// [2^12, 2^13) so that |V| <= 4 max|x| stays below 2^15.
//
// The stem (8 -> 64, direct, k_leafnet_x3's form) and the heads are x3's; the stem output x0 (the
// tower's final residual) waits in a global workspace ([B][N*N][64] f32) for the last conv.
#include "../../include/blokus_engine.h"
#include "ctx.h"

#define BK_LN_VACC 1  // the stem's accumulators in VGPRs: the AGPRs are the tower's U
#include "leafnet_common.h"

namespace bk {
namespace {

constexpr int kW3N = 20, kW3T = 10, kW3Tiles = 100, kW3Groups = 7, kW3GW = kW3N + 2;
constexpr int kW3UnitB = 16384;                            // one V unit: 4 eta x 2 chunks x 2 parts x 4 octets x 16 tiles x 16 B
constexpr int kW3Grid = 2 * kW3UnitB;                      // the grid after the ring
constexpr int kW3Pix = 256;                                // 64 fp32 channels
constexpr int kW3RowB = kW3GW * kW3Pix;                    // 5632 B per grid row
constexpr int kW3Red = kW3Grid + kW3GW * kW3GW * kW3Pix;   // wave maxima
constexpr int kW3Lds = kW3Red + 64;
static_assert(kW3Lds <= 160 * 1024, "k_leafnet_w3: LDS");
constexpr int kW3UConv = 16 * 2 * 4 * 2 * 64 * 16;          // bytes of one conv's split U (256 KiB)

// the unit from which a group's outputs may overwrite the grid: the last unit whose V reads
// one of the group's output rows has passed its barrier (tools/w3/lds_plan.py)
__host__ __device__ constexpr int w3_write_unit(int g) {
  return g == 0 ? 7 : g == 1 ? 12 : g == 2 ? 15 : g == 3 ? 19 : g == 4 ? 20 : g == 5 ? 27 : 28;
}

__device__ __forceinline__ int w3_swz(int C) { return ((C - 1) >> 1) & 7; }

#ifndef BK_W3_ABL
#define BK_W3_ABL 0  // timing ablations only (wrong outputs): 1 no V pieces, 2 no output transform, 4 no unit barriers
#endif

#if BK_LN_STAMP
// timing diagnostics only (make w3stamps): per-wave s_memtime stamps of one launch, tools/w3/stamps_w3.py
__device__ unsigned long long g_w3_stamps[256 * 4 * 128];
#define W3STAMP(i)                                                                                         \
  do {                                                                                                     \
    if (l == 0 && blockIdx.x < 256) g_w3_stamps[(blockIdx.x * 4 + wave) * 128 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define W3STAMP(i) \
  do {             \
  } while (0)
#endif

// f32 adds / subtracts and the f16 split as volatile asm: the unit's VALU work stays spread
// between its MFMA triples in the order written. Scalar ops, not v_pk_add_f32: beside MFMAs a
// packed f32 op costs several times the issue slots of the two scalar ops it replaces
// (MI355X_MICROARCH.md, per-instruction constants: "packed f32 VALU ... an anti-lever beside MFMAs").
__device__ __forceinline__ float vadd(float a, float b) {
  float r;
  asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vsub(float a, float b) {
  float r;
  asm volatile("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f32x4 vadd4(f32x4 a, f32x4 b) {
  return f32x4{vadd(a.x, b.x), vadd(a.y, b.y), vadd(a.z, b.z), vadd(a.w, b.w)};
}
__device__ __forceinline__ f32x4 vsub4(f32x4 a, f32x4 b) {
  return f32x4{vsub(a.x, b.x), vsub(a.y, b.y), vsub(a.z, b.z), vsub(a.w, b.w)};
}
__device__ __forceinline__ void vsplit2(float x0, float x1, unsigned& hi, unsigned& lo) {
  asm volatile(
      "v_cvt_pk_f16_f32 %0, %2, %3\n\t"
      "v_fma_mixlo_f16 %1, -%0, 1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, -%0, 1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(x0), "v"(x1));
}

template <int NACC>
__device__ __forceinline__ void w3_drain(f32x4 (&acc)[NACC]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < NACC; ++i) asm volatile("" : "+v"(acc[i]));
}

// U of one (position, chunk, part) straight into AGPRs (no VGPR hop): the compiler does not track
// these loads, so every layer waits for them explicitly (vmcnt(0)) before its first MFMA
__device__ __forceinline__ h16x8 w3_uload(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  h16x8 r;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=a"(r) : "v"(voff), "s"(rs), "s"(soff));
  return r;
}

__global__ __launch_bounds__(kLnThreads, 1) void k_leafnet_w3(const float* __restrict__ obs,
                                                              const h16x8* __restrict__ wstem,
                                                              const float* __restrict__ sstem,
                                                              const float* __restrict__ bstem,
                                                              const h16x8* __restrict__ ut,
                                                              const float* __restrict__ st,
                                                              const float* __restrict__ bt,
                                                              const float* __restrict__ bounds, int nlayers,
                                                              LnHeads hd, float* __restrict__ x0g,
                                                              float* __restrict__ xout) {
  constexpr int N = kW3N, NN = N * N, RS = ln_row(N), NG = ln_groups(N), PIX_IT = (NN + kLnThreads - 1) / kLnThreads;
  constexpr int PL = ln_plane(N);
  static_assert(2 * PL <= kW3Grid, "k_leafnet_w3: the stem input planes live in the V ring");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* sin = lds;  // the stem's input planes (hi, lo): inside the ring, used before it
  float* red = reinterpret_cast<float*>(lds + kW3Red);
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oc = 16 * wave + 4 * ks;
  const size_t b = blockIdx.x;
  W3STAMP(0);

  const __amdgpu_buffer_rsrc_t urs = ln_rsrc(ut, (unsigned)nlayers * kW3UConv);
  const int uvo = l * 16;
  auto usoff = [&](int layer, int p, int c, int h) { return (((layer * 16 + p) * 2 + c) * 4 + wave) * 2048 + h * 1024; };
  h16x8 U[16][2][2];

  // the observation loads
  const float* ob = obs + b * kStemCinX3 * NN;
  float xin[PIX_IT][kStemCinX3];
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
#pragma unroll
    for (int c = 0; c < kStemCinX3; ++c) xin[it][c] = p < NN ? ob[c * NN + p] : 0.0f;
  }
  // zero the halos: the stem planes' (as k_leafnet_x3) and the grid's (rows 0, 21; columns 0, 21)
  {
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
      *reinterpret_cast<u32x4*>(lds + plane * PL + (row * RS + col) * 16) = u32x4{0u, 0u, 0u, 0u};
    }
    constexpr int kGHalo = 2 * kW3GW + 2 * N;  // haloed pixels of the grid
    for (int i = tid; i < kGHalo * 16; i += kLnThreads) {
      const int k = i >> 4, qd = i & 15;
      int row, col;
      if (k < 2 * kW3GW) {
        row = k < kW3GW ? 0 : kW3GW - 1;
        col = k < kW3GW ? k : k - kW3GW;
      } else {
        row = 1 + ((k - 2 * kW3GW) >> 1);
        col = ((k - 2 * kW3GW) & 1) ? kW3GW - 1 : 0;
      }
      *reinterpret_cast<u32x4*>(lds + kW3Grid + (row * kW3GW + col) * kW3Pix + qd * 16) = u32x4{0u, 0u, 0u, 0u};
    }
  }
  // the stem's pixel slots (k_leafnet_x3's map), its weights, scale and bias
  constexpr int kBias = (RS + 1) * 16;
  int sb[NG];
  unsigned valid = 0;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int sl = kLnPixMap<N>.slot[16 * g + n];
    sb[g] = (sl >= 0 ? sl : RS + 1) * 16 - kBias;
    valid |= (sl >= 0 ? 1u : 0u) << g;
  }
  auto is_valid = [&](int g) { return NN % 16 == 0 || ((valid >> g) & 1u); };
  h16x8 wsa[3][2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    wsa[j][0] = wstem[((j * 4 + wave) * 2) * 64 + l];
    wsa[j][1] = wstem[((j * 4 + wave) * 2 + 1) * 64 + l];
  }
  const f32x4 s_stem = *reinterpret_cast<const f32x4*>(sstem + oc), b_stem = *reinterpret_cast<const f32x4*>(bstem + oc);

  // ---- stem input: scaled by the board maximum, split (k_leafnet_x3)
  float m = 0.0f;
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it)
#pragma unroll
    for (int c = 0; c < kStemCinX3; ++c) m = fmaxf(m, fabsf(xin[it][c]));
  const float max_obs = block_max(m, red + 8, wave, l);
  int ex = scale_exp(max_obs);
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
    if (p < NN) {
      unsigned h[4], o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split2(ldexpf(xin[it][2 * q], ex), ldexpf(xin[it][2 * q + 1], ex), h[q], o[q]);
      unsigned char* dst = sin + ((p / N + 1) * RS + p % N + 1) * 16;
      *reinterpret_cast<u32x4*>(dst) = u32x4{h[0], h[1], h[2], h[3]};
      *reinterpret_cast<u32x4*>(dst + PL) = u32x4{o[0], o[1], o[2], o[3]};
    }
  }
  __syncthreads();

  // ---- stem conv (direct, 3 chunks)
  float max_in;
  {
    f32x4 acc[NG];
    h16x8 rb[kLnSlots][2];
    auto toff = [&](int j) {
      const int t = 4 * j + ks < 9 ? 4 * j + ks : 8;
      return ((t / 3 - 1) * RS + (t % 3 - 1)) * 16 + kBias;
    };
    ln_prime<NG, PL>(rb, sin, sb, toff(0));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j == 0)
        ln_chunk<NG, true, PL>(acc, wsa[0][0], wsa[0][1], sin, sb, toff(0), toff(1), rb);
      else
        ln_chunk<NG, false, PL>(acc, wsa[j][0], wsa[j][1], sin, sb, toff(j), toff(j < 2 ? j + 1 : j), rb);
    }
    ln_mfma_drain(acc);
    // U of the first tower conv (straight into the AGPRs, free from here on): in flight under the
    // stem's epilogue and the first V
#pragma unroll
    for (int p = 0; p < 16; ++p)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int h = 0; h < 2; ++h) U[p][c][h] = w3_uload(urs, uvo, usoff(0, p, c, h));
    // x0 = relu(acc s + b) (unscaled) -> the workspace; x0 2^ex0 -> the grid (the first conv's input)
    const int ex0 = scale_exp(bounds[0] * max_obs + bounds[1]) - 2;
    const f32x2 s01{ldexpf(s_stem.x, -ex), ldexpf(s_stem.y, -ex)}, s23{ldexpf(s_stem.z, -ex), ldexpf(s_stem.w, -ex)};
    const f32x2 b01{b_stem.x, b_stem.y}, b23{b_stem.z, b_stem.w};
    const float up = ldexpf(1.0f, ex0);
    float mx = 0.0f;
    float* x0b = x0g + b * NN * 64;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      f32x2 y01 = pk_fma(f32x2{acc[g][0], acc[g][1]}, s01, b01);
      f32x2 y23 = pk_fma(f32x2{acc[g][2], acc[g][3]}, s23, b23);
      y01 = f32x2{max_bits(y01.x, 0), max_bits(y01.y, 0)};
      y23 = f32x2{max_bits(y23.x, 0), max_bits(y23.y, 0)};
      if (is_valid(g)) {
        mx = max3_abs(max3_abs(mx, y01.x, y01.y), y23.x, y23.y);
        const int px = ln_pixel<N>((sb[g] + kBias) / 16);
        const int r = px / N, c = px - r * N;
        *reinterpret_cast<f32x4*>(x0b + px * 64 + oc) = f32x4{y01.x, y01.y, y23.x, y23.y};
        *reinterpret_cast<f32x4*>(lds + kW3Grid + ((r + 1) * kW3GW + c + 1) * kW3Pix + 16 * ((4 * wave + ks) ^ ((c >> 1) & 7))) =
            f32x4{y01.x * up, y01.y * up, y23.x * up, y23.y * up};
      }
    }
    mx = wave_max_f(mx);
    if (l == 0) red[wave] = mx;
    __syncthreads();
    max_in = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    ex = ex0;
    W3STAMP(1);
  }

  // ---- the V producer: thread = (tile slot pn, channel quad q) of a group (lane groups of the
  // ds_read_b128 banking: the 16 lanes of one group read the 16 quads of one pixel)
  const int l5 = l & 31;
  const bool g1 = (l5 >= 4 && l5 < 12) || (l5 >= 16 && l5 < 20) || l5 >= 28;
  const int pq = g1 ? (l5 < 12 ? l5 - 4 : (l5 < 20 ? l5 - 8 : l5 - 16)) : (l5 < 4 ? l5 : (l5 < 16 ? l5 - 8 : l5 - 12));
  const int pn = 4 * wave + 2 * (l >> 5) + (g1 ? 1 : 0);
  const int pc = pq >> 3, po = (pq >> 1) & 3;
  // its V-ring write offset (eta, part, unit slot as immediates) and the MFMA lane's B read offset
  const int vw = pc * 2048 + po * 256 + ((pn ^ (2 * po)) * 16) + 8 * (pq & 1);
  const int vr = (ks * 16 + (n ^ (2 * ks))) * 16;
  // window column addresses of the producer's tile in group g (row k: + k * kW3RowB)
  // (lane-derived values come in as arguments made opaque per group, so that the compiler does not
  // hoist the addresses of all 7 groups out of the layer loop and keep them live)
  auto win_cols = [&](int g, int pnx, int (&va)[4]) {
    const int t = min(16 * g + pnx, kW3Tiles - 1), ti = t / kW3T, tj = t - ti * kW3T;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int C = 2 * tj + k;
      va[k] = kW3Grid + (2 * ti * kW3GW + C) * kW3Pix + 16 * (pq ^ w3_swz(C));
    }
  };
  auto rd = [&](int va, int k) { return *reinterpret_cast<const f32x4*>(lds + va + k * kW3RowB); };
  // grid reads of V(g, xi): window rows r0, r1 of the 4 columns (B^T row xi = d0 - d2, d1 + d2,
  // d2 - d1, d1 - d3), issued one unit ahead of the unit that builds V
  auto fetch = [&](int xi, const int (&va)[4], f32x4 (&dq)[8]) {
    const int r0 = xi == 0 ? 0 : 1, r1 = xi == 0 ? 2 : (xi == 3 ? 3 : 2);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      dq[2 * k] = rd(va[k], r0);
      dq[2 * k + 1] = rd(va[k], r1);
    }
  };
  // building V(u) from its reads, in 8 pieces that ride between the 8 MFMA triples of a unit:
  // 0, 1: the row combinations t of columns 0-1, 2-3; 2, 3: the column combinations v[0..1],
  // v[2..3]; 4..7: split v[e] and store it to ring slot `slot`. Volatile asm keeps each piece
  // where it is placed (the compiler would otherwise gather them into one VALU block).
  struct Prod {
    f32x4 t[4], v[4];
  };
  auto piece = [&](int i, int xi, const f32x4 (&dq)[8], Prod& pr, int slot) {
    if (i < 2) {
#pragma unroll
      for (int k = 2 * i; k < 2 * i + 2; ++k) {
        const f32x4 a = dq[2 * k], c = dq[2 * k + 1];
        pr.t[k] = xi == 1 ? vadd4(a, c) : (xi == 2 ? vsub4(c, a) : vsub4(a, c));
      }
    } else if (i == 2) {
      pr.v[0] = vsub4(pr.t[0], pr.t[2]);
      pr.v[1] = vadd4(pr.t[1], pr.t[2]);
    } else if (i == 3) {
      pr.v[2] = vsub4(pr.t[2], pr.t[1]);
      pr.v[3] = vsub4(pr.t[1], pr.t[3]);
    } else {
      const int e = i - 4;
      unsigned h0, h1, l0, l1;
      vsplit2(pr.v[e].x, pr.v[e].y, h0, l0);
      vsplit2(pr.v[e].z, pr.v[e].w, h1, l1);
      unsigned char* d = lds + slot * kW3UnitB + vw + e * 4096;
      *reinterpret_cast<u32x2*>(d) = u32x2{h0, h1};
      *reinterpret_cast<u32x2*>(d + 1024) = u32x2{l0, l1};
    }
  };

  // ---- the output side: lane (wave, l) holds output channels oc..oc+3 of tile slot n
  auto out_addr = [&](int g, int nx) {  // grid byte offset of the tile's top-left output pixel, quad oc/4
    const int t = min(16 * g + nx, kW3Tiles - 1), ti = t / kW3T, tj = t - ti * kW3T;
    return kW3Grid + ((2 * ti + 1) * kW3GW + 2 * tj + 1) * kW3Pix + 16 * ((4 * wave + ks) ^ (tj & 7));
  };
  auto out_pixel = [&](int g, int nx) {  // board pixel of that output
    const int t = min(16 * g + nx, kW3Tiles - 1), ti = t / kW3T, tj = t - ti * kW3T;
    return 2 * ti * N + 2 * tj;
  };
  auto tile_ok = [&](int g) { return g < kW3Groups - 1 || 16 * g + n < kW3Tiles; };

  // ---- residual tower
  f32x4 acc[16];
  for (int layer = 0; layer < nlayers; ++layer) {
    const bool last = layer + 1 == nlayers;
    const f32x4 sv = *reinterpret_cast<const f32x4*>(st + layer * 64 + oc);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bt + layer * 64 + oc);
    const int ex_out = last ? 0 : scale_exp(bounds[2 * (layer + 1)] * max_in + bounds[2 * (layer + 1) + 1]) - 2;
    const int k = last ? 0 : ex_out;
    const f32x2 s01{ldexpf(sv.x, k - ex), ldexpf(sv.y, k - ex)}, s23{ldexpf(sv.z, k - ex), ldexpf(sv.w, k - ex)};
    const f32x2 b01{ldexpf(bv.x, k), ldexpf(bv.y, k)}, b23{ldexpf(bv.z, k), ldexpf(bv.w, k)};
    const int floor = (last || !(layer & 1)) ? 0 : (int)0x80000000u;  // ReLU after each block's first conv
    float mx = 0.0f;
    f32x4 y[kW3Groups][4];  // a group's outputs (subpixel a b), held until their write unit
    const float* x0b = x0g + b * NN * 64;
    // a group's outputs into its (now dead) grid pixels (the last conv's too: the heads read them)
    auto write_out = [&](int gw, const f32x4 (&yy)[4], int nx) {
      if (!tile_ok(gw)) return;
      unsigned char* d = lds + out_addr(gw, nx);
      *reinterpret_cast<f32x4*>(d) = yy[0];
      *reinterpret_cast<f32x4*>(d + kW3Pix) = yy[1];
      *reinterpret_cast<f32x4*>(d + kW3RowB) = yy[2];
      *reinterpret_cast<f32x4*>(d + kW3RowB + kW3Pix) = yy[3];
    };
    if (layer == 1) W3STAMP(2);
    // V(0, 0) up front (its piece order without MFMAs), and the reads of V(0, 1)
    f32x4 dq[8];
    int vacur[4], vanext[4];  // window columns of this group's tiles and (from xi = 2 on) the next's
    win_cols(0, pn, vacur);
    {
      Prod pr;
      fetch(0, vacur, dq);
#pragma unroll
      for (int i = 0; i < 8; ++i) piece(i, 0, dq, pr, 0);
      fetch(1, vacur, dq);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this conv's U (direct-to-AGPR loads)
    if (layer == 1) W3STAMP(3);
    f32x4 Yp[4];  // the previous group's output transform (its epilogue runs in the next unit)
    f32x4 xr[4];  // last conv: x0 of the previous group's outputs
    // the epilogue of group gp from its transform Y, subpixels a0..a1-1: y = Y s + b (+ x0),
    // ReLU, the board maximum
    auto finish = [&](int gp, const f32x4 (&Y)[4], int a0, int a1) {
      const bool ok = tile_ok(gp);
#pragma unroll
      for (int a = a0; a < a1; ++a) {
        f32x2 y01 = pk_fma(f32x2{Y[a].x, Y[a].y}, s01, b01);
        f32x2 y23 = pk_fma(f32x2{Y[a].z, Y[a].w}, s23, b23);
        if (last) {
          y01 = pk_add(y01, f32x2{xr[a].x, xr[a].y});
          y23 = pk_add(y23, f32x2{xr[a].z, xr[a].w});
        }
        y01 = f32x2{max_bits(y01.x, floor), max_bits(y01.y, floor)};
        y23 = f32x2{max_bits(y23.x, floor), max_bits(y23.y, floor)};
        if (ok) mx = max3_abs(max3_abs(mx, y01.x, y01.y), y23.x, y23.y);
        y[gp][a] = f32x4{y01.x, y01.y, y23.x, y23.y};
      }
    };
    // the output transform of transform row xi in three parts: Z = M A (z0 = M0 + M1 + M2,
    // z1 = M1 - M2 - M3), then Y += A^T[.][xi] Z
    f32x4 z0, z1;
    auto zpart = [&](int part, int xi, f32x4 (&Y)[4]) {
      if (part == 0) {
        z0 = vadd4(vadd4(acc[4 * xi], acc[4 * xi + 1]), acc[4 * xi + 2]);
      } else if (part == 1) {
        z1 = vsub4(vsub4(acc[4 * xi + 1], acc[4 * xi + 2]), acc[4 * xi + 3]);
      } else if (xi == 0) {
        Y[0] = z0;
        Y[1] = z1;
      } else if (xi == 1) {
        Y[0] = vadd4(Y[0], z0);
        Y[1] = vadd4(Y[1], z1);
        Y[2] = z0;
        Y[3] = z1;
      } else if (xi == 2) {
        Y[0] = vadd4(Y[0], z0);
        Y[1] = vadd4(Y[1], z1);
        Y[2] = vsub4(Y[2], z0);
        Y[3] = vsub4(Y[3], z1);
      } else {
        Y[2] = vsub4(Y[2], z0);
        Y[3] = vsub4(Y[3], z1);
      }
    };
    f32x4 Yc[4];  // this group's transform
#pragma unroll
    for (int g = 0; g < kW3Groups; ++g) {
      int pnx = pn, nx = n;
      asm volatile("" : "+v"(pnx), "+v"(nx));
#pragma unroll
      for (int xi = 0; xi < 4; ++xi) {
        const int u = 4 * g + xi, slot = u & 1;
        const bool more = u + 1 < 4 * kW3Groups;  // a next unit to build V for
        if (layer == 1) W3STAMP(4 + u);
        // the barrier: the V stores of this unit's slot done (all but the 8 grid reads of the
        // V after next, issued last, which may stay in flight across it)
        if (BK_W3_ABL & 4)
          asm volatile("" ::: "memory");
        else if (u == 0 || u + 1 >= 4 * kW3Groups)
          __syncthreads();
        else
          asm volatile("s_waitcnt lgkmcnt(8)\n\ts_barrier" ::: "memory");
        if (layer == 1) W3STAMP(32 + u);
        if (xi == 0 && g > 0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) vacur[k] = vanext[k];
        }
        if (xi == 2 && g + 1 < kW3Groups) win_cols(g + 1, pnx, vanext);
        // the groups whose outputs may now overwrite the grid (epilogue done in an earlier unit)
#pragma unroll
        for (int gw = 0; gw < kW3Groups - 1; ++gw)
          if (w3_write_unit(gw) == u && 4 * gw + 4 < u) write_out(gw, y[gw], nx);
        // B fragments of the unit's 4 positions (2 chunks, hi/lo), one position ahead
        const unsigned char* rbase = lds + slot * kW3UnitB + vr;
        h16x8 bf[2][2][2];
        auto bload = [&](int e) {
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int h = 0; h < 2; ++h)
              bf[e & 1][c][h] = *reinterpret_cast<const h16x8*>(rbase + e * 4096 + c * 2048 + h * 1024);
        };
        bload(0);
        // the unit's schedule: V pieces 0-1 under the B fragments' LDS latency, then after
        // triple i piece i + 2, the output transform of the previous row in three parts (after
        // triples 2-4), and at xi = 0 the previous group's epilogue (after triples 5-6)
        Prod pr;
        constexpr int kSt = -1;
        const int su = (u == 9 ? 64 : (u == 12 ? 80 : (u == 10 ? 96 : kSt)));
        if (layer == 1 && su >= 0) W3STAMP(su);
        if (more && !(BK_W3_ABL & 1)) {
          piece(0, (u + 1) & 3, dq, pr, slot ^ 1);
          piece(1, (u + 1) & 3, dq, pr, slot ^ 1);
        }
        if (layer == 1 && su >= 0) W3STAMP(su + 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int e = i >> 1, c = i & 1, p = 4 * xi + e;
          if (c == 0 && e < 3) bload(e + 1);
          const h16x8(&B)[2] = bf[e & 1][c];
          if (c == 0)
            asm volatile(
                "v_mfma_f32_16x16x32_f16 %0, %1, %2, 0\n\t"
                "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
                "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
                : "=&v"(acc[p])
                : "a"(U[p][0][0]), "v"(B[0]), "a"(U[p][0][1]), "v"(B[1]));
          else
            asm volatile(
                "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
                "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
                "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
                : "+v"(acc[p])
                : "a"(U[p][1][0]), "v"(B[0]), "a"(U[p][1][1]), "v"(B[1]));
          if (layer == 1 && su >= 0) W3STAMP(su + 2 + i);  // after triple i
          if (more && i + 2 < 8 && !(BK_W3_ABL & 1)) piece(i + 2, (u + 1) & 3, dq, pr, slot ^ 1);
          if (i >= 2 && i <= 4 && !(BK_W3_ABL & 2)) {
            if (xi > 0) zpart(i - 2, xi - 1, Yc);
            else if (g > 0) zpart(i - 2, 3, Yp);
          }
          if ((i == 5 || i == 6) && xi == 0 && g > 0) finish(g - 1, Yp, i == 5 ? 0 : 2, i == 5 ? 2 : 4);
          if (i == 6 && xi == 0 && g > 0) {
            // a group whose pixels are already dead (write unit = this one) goes out right away
            if (w3_write_unit(g - 1) == u) write_out(g - 1, y[g - 1], nx);
            if (last && xout && tile_ok(g - 1)) {
              const int px = out_pixel(g - 1, nx);
#pragma unroll
              for (int a = 0; a < 4; ++a)
                *reinterpret_cast<f32x4*>(xout + (b * NN + px + (a >> 1) * N + (a & 1)) * 64 + oc) = y[g - 1][a];
            }
          }
          // the last group: position e is done with U after its second chunk -> the next conv's
          if (g == kW3Groups - 1 && !last && c == 1) {
#pragma unroll
            for (int cc = 0; cc < 2; ++cc)
#pragma unroll
              for (int h = 0; h < 2; ++h) U[p][cc][h] = w3_uload(urs, uvo, usoff(layer + 1, p, cc, h));
          }
        }
        if (layer == 1 && su >= 0) W3STAMP(su + 10);
        // the reads of the V after next (built during the next unit)
        if (u + 2 < 4 * kW3Groups) fetch((u + 2) & 3, xi < 2 ? vacur : vanext, dq);
        if (layer == 1 && su >= 0) W3STAMP(su + 11);
        if (xi == 3) {  // this group's transform is complete but for row 3: finished in the next unit
#pragma unroll
          for (int a = 0; a < 4; ++a) Yp[a] = Yc[a];
          if (last) {  // x0 of this group's outputs, for its epilogue in the next unit
            const int px = out_pixel(g, nx);
#pragma unroll
            for (int a = 0; a < 4; ++a) xr[a] = *reinterpret_cast<const f32x4*>(x0b + (px + (a >> 1) * N + (a & 1)) * 64 + oc);
          }
        }
      }
    }
    // the last group's row 3 and epilogue, then its outputs (after the layer's last read: no wait)
    w3_drain(acc);
#pragma unroll
    for (int part = 0; part < 3; ++part) zpart(part, 3, Yp);
    finish(kW3Groups - 1, Yp, 0, 4);
    if (last && xout && tile_ok(kW3Groups - 1)) {
      const int px = out_pixel(kW3Groups - 1, n);
#pragma unroll
      for (int a = 0; a < 4; ++a)
        *reinterpret_cast<f32x4*>(xout + (b * NN + px + (a >> 1) * N + (a & 1)) * 64 + oc) = y[kW3Groups - 1][a];
    }
    write_out(kW3Groups - 1, y[kW3Groups - 1], n);
    // the board maximum of this conv's output (the next conv's bound), then the next conv
    if (layer == 1) W3STAMP(60);
    mx = wave_max_f(mx);
    if (l == 0) red[4 + 4 * (layer & 1) + wave] = mx;
    __syncthreads();
    if (layer == 1) W3STAMP(61);
    max_in = fmaxf(fmaxf(red[4 + 4 * (layer & 1)], red[5 + 4 * (layer & 1)]),
                   fmaxf(red[6 + 4 * (layer & 1)], red[7 + 4 * (layer & 1)]));
    ex = ex_out;
  }

  W3STAMP(62);
  // ---- heads (blokus_nnet.py:146-150, BN folded) from the tower output in the grid: wave w takes
  // channels 16w..16w+15 of pixel p (lane), the 4 waves' partials meet in LDS (the dead V ring)
  float* hp = reinterpret_cast<float*>(lds);  // [NN][4 waves][3]
  {
    f32x4 wq[3][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wq[0][i] = *reinterpret_cast<const f32x4*>(hd.wp + 16 * wave + 4 * i);
      wq[1][i] = *reinterpret_cast<const f32x4*>(hd.wp + 64 + 16 * wave + 4 * i);
      wq[2][i] = *reinterpret_cast<const f32x4*>(hd.wv + 16 * wave + 4 * i);
    }
    for (int p = l; p < NN; p += 64) {
      const int r = p / N, c = p - r * N;
      const unsigned char* px = lds + kW3Grid + ((r + 1) * kW3GW + c + 1) * kW3Pix;
      const int sw = (c >> 1) & 7;
      float d[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 yv = *reinterpret_cast<const f32x4*>(px + 16 * ((4 * wave + i) ^ sw));
#pragma unroll
        for (int k = 0; k < 3; ++k) d[k] += yv.x * wq[k][i].x + yv.y * wq[k][i].y + yv.z * wq[k][i].z + yv.w * wq[k][i].w;
      }
      float* dst = hp + (p * 4 + wave) * 3;
      dst[0] = d[0];
      dst[1] = d[1];
      dst[2] = d[2];
    }
  }
  __syncthreads();
  float* vfeat = hp + NN * 12;
  float* part = vfeat + NN;
  const float bp0 = hd.bp[0], bp1 = hd.bp[1], bv0 = hd.bv[0];
  for (int i = tid; i < NN; i += kLnThreads) {
    const float* q = hp + i * 12;
    const float p0 = ((q[0] + q[3]) + q[6]) + q[9], p1 = ((q[1] + q[4]) + q[7]) + q[10],
                pv = ((q[2] + q[5]) + q[8]) + q[11];
    hd.pf[b * 2 * NN + i] = fmaxf(p0 + bp0, 0.0f);
    hd.pf[b * 2 * NN + NN + i] = fmaxf(p1 + bp1, 0.0f);
    vfeat[i] = fmaxf(pv + bv0, 0.0f);
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
    float w2[kMaxP], b2[kMaxP];
#pragma unroll
    for (int q = 0; q < kMaxP; ++q) {
      w2[q] = q < hd.P ? hd.w2[q * 64 + l] : 0.0f;
      b2[q] = q < hd.P ? hd.b2[q] : 0.0f;
    }
    const float h = fmaxf(((part[l] + part[64 + l]) + (part[128 + l] + part[192 + l])) + hd.b1[l], 0.0f);
#pragma unroll
    for (int q = 0; q < kMaxP; ++q) {
      if (q < hd.P) {
        const float sum = wave_sum_f(w2[q] * h);
        if (l == 0) hd.v[b * hd.P + q] = tanhf(sum + b2[q]);
      }
    }
  }
  W3STAMP(63);
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_leafnet_w3_supported(int N) { return N == kW3N; }

#if BK_LN_STAMP
int bk_w3_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_w3_stamps), sizeof(g_w3_stamps)) == hipSuccess ? 0 : -1;
}
#endif

int bk_leafnet_w3_weight_bytes(void) { return kW3UConv; }

int bk_leafnet_w3(const float* obs, int B, int N, int cin, const void* wstem, const float* sstem, const float* bstem,
                  int nlayers, const void* utower, const float* stower, const float* btower, const float* bounds,
                  const float* wp, const float* bp, const float* wv, const float* bv, const float* w1t,
                  const float* b1, const float* w2, const float* b2, int P, float* pf, float* vout, float* x0ws,
                  float* out, void* stream) {
  BK_REQUIRE(obs && wstem && sstem && bstem && utower && stower && btower && bounds && x0ws && B >= 0, "bad argument");
  BK_REQUIRE(wp && bp && wv && bv && w1t && b1 && w2 && b2 && pf && vout && P > 0 && P <= kMaxP, "bad argument");
  BK_REQUIRE(cin == kStemCinX3, "bk_leafnet_w3: the stem takes 8 observation planes");
  BK_REQUIRE(nlayers >= 1, "bk_leafnet_w3: at least one tower conv");
  BK_REQUIRE(bk_leafnet_w3_supported(N), "bk_leafnet_w3: N must be 20");
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  BK_REQUIRE(a16(wstem) && a16(utower) && a16(sstem) && a16(bstem) && a16(stower) && a16(btower) && a16(wp) &&
                 a16(wv) && a16(out) && a16(x0ws),
             "bk_leafnet_w3: 16-byte aligned buffers");
  if (B == 0) return BK_OK;
  {
    const void* fns[1] = {(const void*)k_leafnet_w3};
    if (set_max_dynamic_lds(fns, 1, kW3Lds) != BK_OK) return BK_EHIP;
  }
  const LnHeads h{wp, bp, wv, bv, w1t, b1, w2, b2, P, pf, vout};
  hipLaunchKernelGGL(k_leafnet_w3, dim3(B), dim3(kLnThreads), kW3Lds, (hipStream_t)stream, obs,
                     reinterpret_cast<const h16x8*>(wstem), sstem, bstem, reinterpret_cast<const h16x8*>(utower),
                     stower, btower, bounds, nlayers, h, x0ws, out);
  return launch_check("k_leafnet_w3");
}

}  // extern "C"
