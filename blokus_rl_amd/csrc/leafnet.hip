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
// board's layer input lives in LDS as zero-haloed pixel grids of split halves, one plane per
// 8 channels (ln_plane): the B fragment of lane l is one ds_read_b128 per half at the slot of
// column l%16 of group g (LnPixMap) shifted by the tap, in the plane of channels 8(l/16).. of
// the chunk. The A fragments
// (weights) stream from global memory (L2-resident across the 32 boards of an XCD), one chunk
// ahead. The accumulators of all NG groups stay in registers for the layer; the epilogue applies
// scale, bias, (residual), ReLU, finds the board maximum, splits and writes the next layer input
// in place. The stem output x0 stays in registers for the tower's final residual, and the last
// layer's epilogue feeds the heads' 1x1 convs straight from the registers.
#include "../../include/blokus_engine.h"
#include "ctx.h"

// the MFMA accumulators in VGPRs: the epilogue's VALU reads them without 100 v_accvgpr_read per
// layer (AGPRs: 159.7 vs 157.9 us a launch, self-play +0.9%, three interleaved rounds on one box;
// x0 still waits in AGPRs)
#define BK_LN_VACC 1
#include "leafnet_common.h"

#ifndef BK_LN_EPIW
#define BK_LN_EPIW 1  // a tower conv's outputs stored group by group inside its epilogue (0: all after it)
#endif

namespace bk {
namespace {

constexpr bool kLnEpiWrite = BK_LN_EPIW != 0;
#ifndef BK_LN_IL
#define BK_LN_IL 1  // the tower's B-fragment reads between the MFMAs of each triple (ln_chunk_il)
#endif
constexpr bool kLnInterleave = BK_LN_IL != 0;

template <int N>
__global__ __launch_bounds__(kLnThreads, 1) void k_leafnet_x3(const float* __restrict__ obs,
                                                              const h16x8* __restrict__ wstem,
                                                              const float* __restrict__ sstem,
                                                              const float* __restrict__ bstem,
                                                              const h16x8* __restrict__ wt,
                                                              const float* __restrict__ st,
                                                              const float* __restrict__ bt,
                                                              const float* __restrict__ bounds, int nlayers,
                                                              LnHeads hd, float* __restrict__ xout) {
  constexpr int NN = N * N, RS = ln_row(N), NG = ln_groups(N), PIX_IT = (NN + kLnThreads - 1) / kLnThreads;
  constexpr int PL = ln_plane(N);
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* act = lds;                  // 16 planes [hi q | lo q][(N+2) x RS slots][16 B]
  unsigned char* sin = lds + 16 * PL;        // 2 planes: the stem input hi, lo
  float* red = reinterpret_cast<float*>(lds + ln_lds_body(N));
  constexpr int X0L = ln_x0_lds_groups(N);   // x0 groups 0..X0L-1 stashed in LDS
  f32x4* x0s = reinterpret_cast<f32x4*>(lds + 16 * PL);
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int oc = 16 * wave + 4 * ks;  // the lane's 4 output channels oc..oc+3 in the D fragments
  const size_t b = blockIdx.x;
  LNSTAMP(0, __builtin_amdgcn_s_memtime());
  LNSTAMP(30, __builtin_amdgcn_s_memrealtime());

  // the observation loads first (their latency under the halo zeroing below)
  const float* ob = obs + b * kStemCinX3 * NN;
  float xin[PIX_IT][kStemCinX3];
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
#pragma unroll
    for (int c = 0; c < kStemCinX3; ++c) xin[it][c] = p < NN ? ob[c * NN + p] : 0.0f;
  }
  // zero the halo of all 18 planes (rows 0 and N+1, columns 0 and N+1..RS-1; the only slots read
  // that no layer writes: interiors are written before they are read)
  {
    constexpr int kHaloCols = RS - N, kHalo = 2 * RS + N * kHaloCols;
    for (int i = tid; i < 18 * kHalo; i += kLnThreads) {
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

  // the lane's grid slot in each group, in bytes (a spare column reads slot 0 of the halo: zeros),
  // and the mask of groups where the lane's column is a board pixel
  // ab[g] = the lane's B-read base: its slot + its k-group's plane block, less kBias so that
  // every chunk's plane/tap offset is a non-negative immediate (no address VALU in the MFMA loop);
  // a spare column reads at pixel (0, 0) (its MFMA column is never written out)
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
  auto slot_b = [&](int g) { return ab[g] - ks * 4 * PL + kBias; };  // the lane's slot in group g, bytes

  // the weights stream through a ring of kLnWpf + 1 chunks, kLnWpf chunks ahead of the MFMAs and
  // on into the next layer (18 chunks per layer: the ring slot of chunk c is c % (kLnWpf + 1) in
  // every layer), so no layer starts on an exposed L2 load
  static_assert(18 % (kLnWpf + 1) == 0, "kLnWpf: the ring must divide the 18 chunks of a layer");
  constexpr int kLayerBlocks = 18 * 4 * 2;  // (chunk, wave, part) blocks of 64 x 16 B per layer
  const __amdgpu_buffer_rsrc_t wrs = ln_rsrc(wt, (unsigned)nlayers * kLayerBlocks * 1024u);
  // part p (0 hi, 1 lo) of the lane's A fragment of chunk c of tower layer `layer`
  auto wload = [&](int layer, int c, int p) {
    return __builtin_bit_cast(h16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                         wrs, l * 16, ((layer * kLayerBlocks + c * 8 + wave * 2 + p) * 64) * 16, 0));
  };
  h16x8 wq[kLnWpf + 1][2];  // issued here: in flight under the stem
#pragma unroll
  for (int c = 0; c < kLnWpf; ++c) {
    wq[c][0] = wload(0, c, 0);
    wq[c][1] = wload(0, c, 1);
  }
  // the stem's weights (3 chunks), scale and bias, in flight under the observation loads
  h16x8 wsa[3][2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    wsa[j][0] = wstem[((j * 4 + wave) * 2) * 64 + l];
    wsa[j][1] = wstem[((j * 4 + wave) * 2 + 1) * 64 + l];
  }
  const f32x4 s_stem = *reinterpret_cast<const f32x4*>(sstem + oc), b_stem = *reinterpret_cast<const f32x4*>(bstem + oc);

  // ---- stem input: the planar observation [8][N][N] of the board, scaled by its maximum, split
  float m = 0.0f;
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it)
#pragma unroll
    for (int c = 0; c < kStemCinX3; ++c) m = fmaxf(m, fabsf(xin[it][c]));
  const float max_obs = block_max(m, red + 8, wave, l);  // the barrier also orders the zeroing before the writes
  int ex = scale_exp(max_obs);
#pragma unroll
  for (int it = 0; it < PIX_IT; ++it) {
    const int p = tid + it * kLnThreads;
    if (p < NN) {
      unsigned h[4], o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split2(ldexpf(xin[it][2 * q], ex), ldexpf(xin[it][2 * q + 1], ex), h[q], o[q]);
      const u32x4 hi{h[0], h[1], h[2], h[3]}, lo{o[0], o[1], o[2], o[3]};
      unsigned char* dst = sin + ((p / N + 1) * RS + p % N + 1) * 16;
      *reinterpret_cast<u32x4*>(dst) = hi;
      *reinterpret_cast<u32x4*>(dst + PL) = lo;
    }
  }
  __syncthreads();
  LNSTAMP(1, __builtin_amdgcn_s_memtime());

  // ---- stem conv: 3 chunks; lane k-group ks of chunk j is tap 4j + ks (taps > 8 carry zero weights)
  f32x4 acc[NG];
  h16x8 rb[kLnSlots][2];
  {
    auto toff = [&](int j) {
      const int t = 4 * j + ks < 9 ? 4 * j + ks : 8;
      return ((t / 3 - 1) * RS + (t % 3 - 1)) * 16 + kBias - ks * 4 * PL;  // from ab: the stem grid has 2 planes
    };
    ln_prime<NG, PL>(rb, sin, ab, toff(0));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j == 0)
        ln_chunk<NG, true, PL>(acc, wsa[0][0], wsa[0][1], sin, ab, toff(0), toff(1), rb);
      else
        ln_chunk<NG, false, PL>(acc, wsa[j][0], wsa[j][1], sin, ab, toff(j), toff(j < 2 ? j + 1 : j), rb);
    }
  }
  ln_mfma_drain(acc);
  LNSTAMP(2, __builtin_amdgcn_s_memtime());

  // Epilogue of a conv: y = acc * s + bias (+ x0) (ReLU), s = the inverse weight scale x 2^-ex_in.
  // OUT: y is the next layer's input: scaled by 2^ex_out (ex_out from a bound on |y|, so no board
  // reduction is needed before the split), split, and the packed halves kept in acc's registers
  // until every wave has finished reading the grid (bar 1), then written; the lane's max |y|
  // (unscaled) is returned for the next layer's bound. !OUT (the last conv): y stays in acc.
  // WRITE (with OUT, after a barrier that every wave has finished reading the grid): each group's
  // halves are stored into the grid as soon as they are split, so the LDS stores drain under the
  // next groups' VALU instead of after all of it.
  auto epilogue = [&](f32x4 sv, f32x4 bv, bool relu, bool residual, const f32x4 (&x0)[NG], bool out, int ex_out,
                      bool write = false) {
    const int o = 2 * wave + (ks >> 1);
    unsigned char* wbase = act + ((o & 3) * 4 + (o >> 2) * 2) * PL + (ks & 1) * 8;  // as write_act
    // OUT folds the output scale 2^ex_out into s and bias (exact: powers of two), so y comes out
    // scaled and goes straight to the split; the lane maximum is unscaled once at the end
    const int k = out ? ex_out : 0;
    const f32x2 s01{ldexpf(sv.x, k - ex), ldexpf(sv.y, k - ex)}, s23{ldexpf(sv.z, k - ex), ldexpf(sv.w, k - ex)};
    const f32x2 b01{ldexpf(bv.x, k), ldexpf(bv.y, k)}, b23{ldexpf(bv.z, k), ldexpf(bv.w, k)};
    const int floor = relu ? 0 : (int)0x80000000u;
    float mx = 0.0f;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      f32x2 y01 = pk_fma(f32x2{acc[g][0], acc[g][1]}, s01, b01);
      f32x2 y23 = pk_fma(f32x2{acc[g][2], acc[g][3]}, s23, b23);
      if (residual) {  // only without OUT (the last conv): x0 is unscaled
        y01 = pk_add(y01, f32x2{x0[g][0], x0[g][1]});
        y23 = pk_add(y23, f32x2{x0[g][2], x0[g][3]});
      }
      y01 = f32x2{max_bits(y01.x, floor), max_bits(y01.y, floor)};
      y23 = f32x2{max_bits(y23.x, floor), max_bits(y23.y, floor)};
      if (is_valid(g)) mx = max3_abs(max3_abs(mx, y01.x, y01.y), y23.x, y23.y);
      if (out) {
        unsigned h0, h1, l0, l1;
        split2(y01.x, y01.y, h0, l0);
        split2(y23.x, y23.y, h1, l1);
        if (write) {
          if (is_valid(g)) {
            *reinterpret_cast<u32x2*>(wbase + slot_b(g)) = u32x2{h0, h1};
            *reinterpret_cast<u32x2*>(wbase + slot_b(g) + PL) = u32x2{l0, l1};
          }
        } else {
          acc[g] = f32x4{__builtin_bit_cast(float, h0), __builtin_bit_cast(float, h1), __builtin_bit_cast(float, l0),
                         __builtin_bit_cast(float, l1)};
        }
      } else {
        acc[g] = f32x4{y01.x, y01.y, y23.x, y23.y};
      }
    }
    return ldexpf(mx, -k);
  };
  // the packed halves in acc -> the activation grid. The lane holds channels oc..oc+3 (hi, lo) of
  // octet o = 2 wave + ks/2; the k-groups ks and ks^1 (rows of 16 lanes) hold the two halves of the
  // octet's 16-B slot. v_permlane16_swap gives the even row both rows' hi halves and the odd row
  // both lo halves, so each lane stores one 16-B slot (hi plane, or the lo plane next to it).
  auto write_act = [&]() {
    const int o = 2 * wave + (ks >> 1);
    // each lane stores its 4 channels' hi and lo halves (8 B each) into its half of the octet's
    // 16-B slot in the hi plane and in the lo plane (no lane swaps)
    unsigned char* base = act + ((o & 3) * 4 + (o >> 2) * 2) * PL + (ks & 1) * 8;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const u32x4 w = __builtin_bit_cast(u32x4, acc[g]);  // {hi 01, hi 23, lo 01, lo 23}
      if (is_valid(g)) {
        *reinterpret_cast<u32x2*>(base + slot_b(g)) = u32x2{w.x, w.y};
        *reinterpret_cast<u32x2*>(base + slot_b(g) + PL) = u32x2{w.z, w.w};
      }
    }
  };
  // the scale of a conv's output from the bound |y| <= A max_in + B (A = the largest row L1 norm
  // of the weights, B = the largest |bias|: nets.pack_x3)
  auto out_exp = [&](int conv, float max_in) { return scale_exp(bounds[2 * conv] * max_in + bounds[2 * conv + 1]); };
  // wave maxima -> red[par][wave] before the barrier, the board maximum after it
  auto post_max = [&](float mx, int par) {
    mx = wave_max_f(mx);
    if (l == 0) red[4 * par + wave] = mx;
  };
  auto board_max = [&](int par) {
    return fmaxf(fmaxf(red[4 * par], red[4 * par + 1]), fmaxf(red[4 * par + 2], red[4 * par + 3]));
  };

  f32x4 x0[NG];
  float max_in;
  {
    const int ex_out = out_exp(0, max_obs);
#pragma unroll
    for (int g = 0; g < NG; ++g) x0[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the stem output itself is kept (unscaled) for the tower's final residual
    const float mx = epilogue(s_stem, b_stem, true, false, x0, false, 0);
#pragma unroll
    for (int g = 0; g < NG; ++g) x0[g] = acc[g];
    const float up = ldexpf(1.0f, ex_out);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      unsigned h0, h1, l0, l1;
      split2(x0[g][0] * up, x0[g][1] * up, h0, l0);
      split2(x0[g][2] * up, x0[g][3] * up, h1, l1);
      acc[g] = f32x4{__builtin_bit_cast(float, h0), __builtin_bit_cast(float, h1), __builtin_bit_cast(float, l0),
                     __builtin_bit_cast(float, l1)};
    }
    // x0 waits out the tower in AGPRs (read once, by the last conv): its VGPRs go to the loop
#pragma unroll
    for (int g = X0L; g < NG; ++g) asm volatile("" : "+a"(x0[g]));
    post_max(mx, 0);
    __syncthreads();  // every wave is done with the stem's input planes (the x0 stash reuses them)
    write_act();
#pragma unroll
    for (int g = 0; g < X0L; ++g) {
      x0s[g * kLnThreads + tid] = x0[g];
      x0[g] = f32x4{0.f, 0.f, 0.f, 0.f};  // not kept in registers
    }
    __syncthreads();
    max_in = board_max(0);
    ex = ex_out;
  }
  LNSTAMP(3, __builtin_amdgcn_s_memtime());

  // ---- residual tower: nlayers convs 64 -> 64; ReLU after each block's first conv; the last
  // adds x0 and takes the ReLU (x = relu(x + res_blocks(x)), blokus_nnet.py:140-141)
  for (int layer = 0; layer < nlayers; ++layer) {
    const bool more = layer + 1 < nlayers;
    // the layer's output scale and bias (folded BN) are loaded here, under the MFMA loop
    const f32x4 sv = *reinterpret_cast<const f32x4*>(st + layer * 64 + oc);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bt + layer * 64 + oc);
    // the next conv's output bound (bounds holds the stem and every tower conv: always in range)
    const float bnd_a = bounds[2 * (layer + 1)], bnd_b = bounds[2 * (layer + 1) + 1];
    // chunk c = (tap c/2, channel half c%2): the lane's octet 4 (c%2) + ks has its hi plane at
    // ks*4 + 2 (c%2) (lo next to it), so from ab the offset is a compile-time immediate < 2^16
    auto coff_of = [&](int c) {
      const int t = c >> 1;
      return 2 * (c & 1) * PL + ((t / 3 - 1) * RS + (t % 3 - 1)) * 16 + kBias;
    };
    ln_prime<NG, PL>(rb, act, ab, coff_of(0));
    if (layer == 1) LNSTAMP(26, __builtin_amdgcn_s_memtime());
#pragma unroll
    for (int c = 0; c < 18; ++c) {
      if (layer == 1 && c == 1) LNSTAMP(27, __builtin_amdgcn_s_memtime());
      if (layer == 1 && c == 9) LNSTAMP(28, __builtin_amdgcn_s_memtime());
      const int cn = c + kLnWpf, sn = cn % (kLnWpf + 1);
      if (cn < 18) {
        wq[sn][0] = wload(layer, cn, 0);
        wq[sn][1] = wload(layer, cn, 1);
      } else {  // the next layer's first chunks; the last layer reloads its own (never used): an
                // unconditional load keeps the wait count static (a branch made it vmcnt(0), an
                // exposed L2 round trip per layer)
        const int nl = more ? layer + 1 : layer;
        wq[sn][0] = wload(nl, cn - 18, 0);
        wq[sn][1] = wload(nl, cn - 18, 1);
      }
      const h16x8* w = wq[c % (kLnWpf + 1)];
      if constexpr (kLnInterleave) {
        if (c == 0)
          ln_chunk_il<NG, true, PL>(acc, w[0], w[1], act, ab, coff_of(0), coff_of(1), rb);
        else
          ln_chunk_il<NG, false, PL>(acc, w[0], w[1], act, ab, coff_of(c), coff_of(c + 1 < 18 ? c + 1 : c), rb);
      } else {
        if (c == 0)
          ln_chunk<NG, true, PL>(acc, w[0], w[1], act, ab, coff_of(0), coff_of(1), rb);
        else
          ln_chunk<NG, false, PL>(acc, w[0], w[1], act, ab, coff_of(c), coff_of(c + 1 < 18 ? c + 1 : c), rb);
      }
    }
    // the last chunk's read-ahead (ln_chunk_il: untracked) lands before its registers are reused
    if constexpr (kLnInterleave) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ln_mfma_drain(acc);
    if (layer < 8) LNSTAMP(4 + 2 * layer, __builtin_amdgcn_s_memtime());
    const bool last = layer + 1 == nlayers;
#ifndef BK_LN_ABL
#define BK_LN_ABL 0  // timing diagnostics only (wrong outputs): 1 no grid writes or barriers between tower
                     // convs, 2 = 1 without the epilogue arithmetic as well
#endif
    if (!last && BK_LN_ABL != 0) {
      if constexpr ((BK_LN_ABL & 2) == 0) {
        const int ex_out = scale_exp(bnd_a * max_in + bnd_b);
        const float mx = epilogue(sv, bv, !(layer & 1), false, x0, true, ex_out);
        max_in = fmaxf(max_in, mx);  // keep the arithmetic live
        ex = ex_out;
      }
    } else if (!last && kLnEpiWrite) {
      const int ex_out = scale_exp(bnd_a * max_in + bnd_b);  // = out_exp(layer + 1, max_in)
      if (layer == 1) LNSTAMP(21, __builtin_amdgcn_s_memtime());
      __syncthreads();  // every wave has finished reading the grid: the outputs go in place as made
      if (layer == 1) LNSTAMP(22, __builtin_amdgcn_s_memtime());
      const float mx = epilogue(sv, bv, !(layer & 1), false, x0, true, ex_out, true);
      if (layer == 1) LNSTAMP(23, __builtin_amdgcn_s_memtime());
      post_max(mx, (layer + 1) & 1);
      if (layer == 1) LNSTAMP(24, __builtin_amdgcn_s_memtime());
      __syncthreads();
      if (layer == 1) LNSTAMP(25, __builtin_amdgcn_s_memtime());
      max_in = board_max((layer + 1) & 1);
      ex = ex_out;
    } else if (!last) {
      const int ex_out = scale_exp(bnd_a * max_in + bnd_b);  // = out_exp(layer + 1, max_in)
      const float mx = epilogue(sv, bv, !(layer & 1), false, x0, true, ex_out);
      if (layer == 1) LNSTAMP(21, __builtin_amdgcn_s_memtime());
      post_max(mx, (layer + 1) & 1);
      if (layer == 1) LNSTAMP(22, __builtin_amdgcn_s_memtime());
      __syncthreads();  // every wave has finished reading the grid
      if (layer == 1) LNSTAMP(23, __builtin_amdgcn_s_memtime());
      write_act();
      if (layer == 1) LNSTAMP(24, __builtin_amdgcn_s_memtime());
      __syncthreads();
      if (layer == 1) LNSTAMP(25, __builtin_amdgcn_s_memtime());
      max_in = board_max((layer + 1) & 1);
      ex = ex_out;
    } else {
#pragma unroll
      for (int g = 0; g < X0L; ++g) x0[g] = x0s[g * kLnThreads + tid];
      epilogue(sv, bv, true, true, x0, false, 0);
    }
    if (layer < 8) LNSTAMP(5 + 2 * layer, __builtin_amdgcn_s_memtime());
  }

  // ---- outputs: the tower output (optional) and the heads (blokus_nnet.py:146-150, BN folded)
  if (xout) {
#pragma unroll
    for (int g = 0; g < NG; ++g)
      if (is_valid(g))
        *reinterpret_cast<f32x4*>(xout + (b * NN + ln_pixel<N>(slot_b(g) / 16)) * 64 + oc) = acc[g];
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
        // the sum over the 4 k-groups: a + a(lane ^ 16), then + (lane ^ 32), as two VALU swaps
        // (v_permlane16/32_swap) instead of LDS permutes; x + y is the same sum in either order
        const float a = y.x * (*w[k]).x + y.y * (*w[k]).y + y.z * (*w[k]).z + y.w * (*w[k]).w;
        const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
        const float a16 = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
        const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a16), __float_as_uint(a16), false, false);
        d[k] = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
      }
      if (ks == 0 && is_valid(g)) {
        float* dst = hp + (ln_pixel<N>(slot_b(g) / 16) * 4 + wave) * 3;
        dst[0] = d[0];
        dst[1] = d[1];
        dst[2] = d[2];
      }
    }
  }
  __syncthreads();
  LNSTAMP(20, __builtin_amdgcn_s_memtime());
  // pf = relu(policy 1x1 conv + bp) (channel-major), vfeat = relu(value 1x1 conv + bv), then
  // v = tanh(W2 relu(W1 vfeat + b1) + b2); the 4 waves sweep quarters of W1's inputs
  float* vfeat = hp + NN * 12;
  float* part = vfeat + NN;
  // the head biases in registers first: read inside the loop, each was re-loaded after every pf
  // store (the compiler cannot rule out aliasing), one dependent round trip per store
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
    // wave w: inputs [Q w, Q (w + 1)) of W1 (L2-resident), every load issued before the first FMA
    constexpr int Q = NN / 4;
    static_assert(NN % 4 == 0, "k_leafnet_x3: quarters of the value-MLP inputs");
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
    // W2 rows and b2 loaded together before the value stores (same aliasing as above)
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
  LNSTAMP(29, __builtin_amdgcn_s_memtime());
  LNSTAMP(31, __builtin_amdgcn_s_memrealtime());
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

#if BK_LN_STAMP
int bk_ln_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ln_stamps), sizeof(g_ln_stamps)) == hipSuccess ? 0 : -1;
}
int bk_ln_stamps_clear() {
  static unsigned long long zeros[256 * 4 * kLnStamps];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ln_stamps), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif

int bk_leafnet_x3(const float* obs, int B, int N, int cin, const void* wstem, const float* sstem, const float* bstem,
                  int nlayers, const void* wtower, const float* stower, const float* btower, const float* bounds,
                  const float* wp,
                  const float* bp, const float* wv, const float* bv, const float* w1t, const float* b1,
                  const float* w2, const float* b2, int P, float* pf, float* vout, float* out, void* stream) {
  BK_REQUIRE(obs && wstem && sstem && bstem && wtower && stower && btower && bounds && B >= 0, "bad argument");
  BK_REQUIRE(wp && bp && wv && bv && w1t && b1 && w2 && b2 && pf && vout && P > 0, "bad argument");
  BK_REQUIRE(cin == kStemCinX3, "bk_leafnet_x3: the stem takes 8 observation planes");
  BK_REQUIRE(nlayers >= 1, "bk_leafnet_x3: at least one tower conv");
  BK_REQUIRE(bk_leafnet_x3_supported(N), "bk_leafnet_x3: N must be 14 or 20");
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  BK_REQUIRE(a16(wstem) && a16(wtower) && a16(sstem) && a16(bstem) && a16(stower) && a16(btower) && a16(wp) &&
                 a16(wv) && a16(out),
             "bk_leafnet_x3: 16-byte aligned buffers");
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
                       stower, btower, bounds, nlayers, h, out);
  else
    hipLaunchKernelGGL(k_leafnet_x3<14>, dim3(B), dim3(kLnThreads), ln_lds_bytes(14), s, obs, ws, sstem, bstem, wt,
                       stower, btower, bounds, nlayers, h, out);
  return launch_check("k_leafnet_x3");
}

}  // extern "C"
