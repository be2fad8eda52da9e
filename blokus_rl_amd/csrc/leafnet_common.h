// leafnet_common.h — pieces shared by the leaf-net kernels on split-f16 MFMA products
// (leafnet.hip: k_leafnet_x3, direct convolutions): the operand split, power-of-two scaling, the
// stem's pixel map and direct K-chunk loop, the MFMA drain.
#pragma once
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

#ifndef BK_LN_DUMMY
#define BK_LN_DUMMY 0  // timing diagnostic only: dummy VALU ops after each MFMA triple (ln_chunk;
                       // profiles/r06_leafnet_valu_shadow.json: ~5.5 cycles each, not hidden)
#endif
#ifndef BK_LN_STAMP
#define BK_LN_STAMP 0  // timing diagnostics only: per-wave s_memtime stamps (bk_ln_stamps)
#endif
#if BK_LN_STAMP
constexpr int kLnStamps = 32;
__device__ unsigned long long g_ln_stamps[256 * 4 * kLnStamps];
#define LNSTAMP(i, v)                                                                                          \
  do {                                                                                                         \
    if (l == 0 && blockIdx.x < 256) g_ln_stamps[(blockIdx.x * 4 + wave) * kLnStamps + (i)] = (v);              \
  } while (0)
#else
#define LNSTAMP(i, v) \
  do {                \
  } while (0)
#endif

constexpr int kLnThreads = 256;
constexpr int kStemCinX3 = 8;
constexpr int kBlock = 64 * 8;     // f16 per (chunk, wave, part) block of packed weights: 64 lanes x 8

__host__ __device__ constexpr int ln_chunks(int cin) { return cin == 64 ? 18 : 3; }

// B-fragment pipeline: the grid reads of a group are issued kLnPf groups ahead of its MFMAs, in a
// ring of kLnSlots register slots that runs on across chunk boundaries (the last kLnPf groups of
// a chunk load the first kLnPf of the next), so the LDS latency is never exposed at a chunk start.
// The slot of group g is g % kLnSlots in every chunk, which needs NG % kLnSlots == 0: the board's
// groups are padded with spare ones (all columns spare: halo reads, no writes) up to a multiple.
#ifndef BK_LN_VACC
#define BK_LN_VACC 0  // the MFMA accumulators in VGPRs (1: leafnet.hip, and leafnet_w3.hip, whose AGPRs hold U) or AGPRs (0)
#endif
#if BK_LN_VACC
#define BK_ACC_W "=&v"
#define BK_ACC_RW "+v"
#else
#define BK_ACC_W "=&a"
#define BK_ACC_RW "+a"
#endif
// read-ahead: 2 groups of B fragments (3, 4: no gain, also with ln_chunk_il), 1 chunk of weights (2: no gain)
constexpr int kLnPf = 2, kLnSlots = 5, kLnWpf = 1;
static_assert(kLnPf >= 1 && kLnPf < kLnSlots, "kLnPf");
__host__ __device__ constexpr int ln_groups(int N) { return ((N * N + 15) / 16 + kLnSlots - 1) / kLnSlots * kLnSlots; }

// The layer input in LDS: 16 planes, each a zero-haloed grid of (N+2) rows x ln_row(N) slots of
// 16 B (8 f16). Channel octet o (channels 8o..8o+7) has its hi halves in plane 4 (o % 4) + 2 (o / 4)
// and its lo halves in the next plane: the octets a lane's k-group ks reads (ks and 4 + ks) sit
// in its own block of 4 planes, so one base register per group reaches every chunk's tap and
// half with an immediate offset (< 3 planes + 2 rows). A plane
// is a multiple of 256 B (the LDS bank period), so the 16-B chunk of every plane of a slot sits in
// the same 4 banks, and the lanes of one ds_read_b128 lane group (16 distinct pixels of a group,
// k-groups ks and ks^1) are conflict-free when their slots differ mod 16 (LnPixMap). The stem's
// input (8 channels) takes two more planes (hi, lo).
__host__ __device__ constexpr int ln_row(int N) { return N == 14 ? 18 : N + 2; }  // slot classes mod 16 balanced
__host__ __device__ constexpr int ln_plane(int N) { return ((N + 2) * ln_row(N) * 16 + 255) / 256 * 256; }
// The stem output's groups that wait out the tower in LDS instead of registers (k_leafnet_x3<20>:
// the register file holds the other 18 groups; all 25 would spill 26 registers to scratch), in the
// stem planes' region (dead after the stem) and above it: [group][256 threads] x 16 B
__host__ __device__ constexpr int ln_x0_lds_groups(int N) { return N == 20 ? 7 : 0; }
// LDS bytes of k_leafnet_x3<N>: 16 activation planes, then the 2 stem planes or the x0 stash
// (whichever is larger), then the wave maxima (2 x 4 + 4 floats)
__host__ __device__ constexpr int ln_lds_body(int N) {
  return 16 * ln_plane(N) + (2 * ln_plane(N) > ln_x0_lds_groups(N) * 256 * 16 ? 2 * ln_plane(N)
                                                                                 : ln_x0_lds_groups(N) * 256 * 16);
}
__host__ __device__ constexpr int ln_lds_bytes(int N) { return ln_lds_body(N) + 64; }

// The board's pixels in MFMA columns: slot (g, n) of pixel group g, column n. Any bijection works
// (reads and writes use the same map); this one gives each group 16 pixels whose grid slots are
// distinct mod 16 where the slot classes allow (one pixel per class, leftovers fill the gaps),
// so the B-fragment reads are bank-conflict-free. Entries: grid slot (row + 1) * ln_row + col + 1,
// or -1 for a spare column (N*N not a multiple of 16).
template <int N>
struct LnPixMap {
  static constexpr int NN = N * N, NG = ln_groups(N), RS = ln_row(N);
  int slot[NG * 16];
  constexpr LnPixMap() : slot() {
    bool used[NN] = {};
    for (int i = 0; i < NG * 16; ++i) slot[i] = -1;
    for (int g = 0; g < NG; ++g)
      for (int r = 0; r < 16; ++r)
        for (int p = 0; p < NN; ++p) {
          const int sl = (p / N + 1) * RS + p % N + 1;
          if (!used[p] && sl % 16 == r) {
            used[p] = true;
            slot[g * 16 + r] = sl;
            break;
          }
        }
    int p = 0;
    for (int i = 0; i < NG * 16; ++i) {
      if (slot[i] >= 0) continue;
      while (p < NN && used[p]) ++p;
      if (p == NN) break;
      used[p] = true;
      slot[i] = (p / N + 1) * RS + p % N + 1;
    }
  }
};
template <int N>
__device__ constexpr LnPixMap<N> kLnPixMap{};
template <int N>
__device__ __forceinline__ int ln_pixel(int slot) {  // grid slot -> board pixel index
  return (slot / ln_row(N) - 1) * N + slot % ln_row(N) - 1;
}

__device__ __forceinline__ f32x4 mfma16(h16x8 a, h16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// x (already scaled) -> packed f16 halves: hi = f16(x) (round to nearest), lo = f16(x - hi)
// (3 VALU ops per pair: x - hi is exact in f32 (|x - hi| <= half an f16 ulp of x), so the mix op's
// one rounding of fma(-hi, 1, x) to f16 is f16(x - hi) as a convert-back-and-subtract form
// computes it (5 ops): bitwise the same)
__device__ __forceinline__ void split2(float x0, float x1, unsigned& hi, unsigned& lo) {
  asm("v_cvt_pk_f16_f32 %0, %2, %3\n\t"
      "v_fma_mixlo_f16 %1, -%0, 1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, -%0, 1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(x0), "v"(x1));
}

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
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
// 4-wide adds / subtracts as two packed f32 ops (the compiler emits four v_sub_f32 for f32x4)
__device__ __forceinline__ f32x4 add4(f32x4 a, f32x4 b) {
  const f32x2 lo = pk_add(f32x2{a.x, a.y}, f32x2{b.x, b.y}), hi = pk_add(f32x2{a.z, a.w}, f32x2{b.z, b.w});
  return f32x4{lo.x, lo.y, hi.x, hi.y};
}
__device__ __forceinline__ f32x4 sub4(f32x4 a, f32x4 b) {
  const f32x2 lo = pk_sub(f32x2{a.x, a.y}, f32x2{b.x, b.y}), hi = pk_sub(f32x2{a.z, a.w}, f32x2{b.z, b.w});
  return f32x4{lo.x, lo.y, hi.x, hi.y};
}
__device__ __forceinline__ f32x4 fma4(f32x4 a, f32x4 b, f32x4 c) {
  const f32x2 lo = pk_fma(f32x2{a.x, a.y}, f32x2{b.x, b.y}, f32x2{c.x, c.y});
  const f32x2 hi = pk_fma(f32x2{a.z, a.w}, f32x2{b.z, b.w}, f32x2{c.z, c.w});
  return f32x4{lo.x, lo.y, hi.x, hi.y};
}

// max(m, |a|, |b|) in one VALU op (fmaxf would canonicalize every input first)
__device__ __forceinline__ float max3_abs(float m, float a, float b) {
  float r;
  asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
// max(y, floor) as signed integers: y for floor = INT_MIN, relu(y) for floor = 0 (-0 -> +0),
// one v_max_i32 (the float max would add a canonicalize per input)
__device__ __forceinline__ float max_bits(float y, int floor) {
  return __builtin_bit_cast(float, max(__builtin_bit_cast(int, y), floor));
}

// a buffer resource over [p, p + bytes), its base made provably wave-uniform (readfirstlane): the
// tower's weight loads as buffer ops (a per-lane VGPR offset + a wave-uniform SGPR offset per
// chunk) instead of one 64-bit VGPR address per load
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ln_rsrc(const void* p, unsigned bytes) {
  const uintptr_t a = (uintptr_t)p;
  const uintptr_t u = ((uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                      (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, (int)bytes, 0x00020000);
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

// The lane's B fragments (hi, lo) of one group: grid + pb (the lane's slot in bytes) + coff (the
// chunk's plane and tap offset); HALF = byte offset of the lo halves from the hi halves.
template <int HALF>
__device__ __forceinline__ void ln_load(h16x8 (&r)[2], const unsigned char* grid, int pb, int coff) {
  const unsigned char* q = grid + pb + coff;
  r[0] = *reinterpret_cast<const h16x8*>(q);
  r[1] = *reinterpret_cast<const h16x8*>(q + HALF);
}

// Fill the ring with the first kLnPf groups of a chunk (at a layer start, after the barrier).
template <int NG, int HALF>
__device__ __forceinline__ void ln_prime(h16x8 (&rb)[kLnSlots][2], const unsigned char* grid, const int (&pb)[NG],
                                         int coff) {
#pragma unroll
  for (int g = 0; g < kLnPf; ++g) ln_load<HALF>(rb[g], grid, pb[g], coff);
}

// One K chunk over the board's NG pixel groups: acc[g] += ah*bh + al*bh + ah*bl with the group's
// B fragments from the ring, whose reads run kLnPf groups ahead and on into the next chunk
// (coff_next; on the last chunk of a layer any in-grid offset: those reads are never consumed).
// The MFMAs are inline asm with the accumulator in place (srcC = vdst: back-to-back accumulation,
// no copies; VGPRs or AGPRs per BK_LN_VACC); INIT starts the accumulators from 0.
template <int NG, bool INIT, int HALF>
__device__ __forceinline__ void ln_chunk(f32x4 (&acc)[NG], h16x8 ah, h16x8 al, const unsigned char* grid,
                                         const int (&pb)[NG], int coff, int coff_next, h16x8 (&rb)[kLnSlots][2]) {
  static_assert(NG % kLnSlots == 0, "ln_chunk: the ring slot of a group must not depend on the chunk");
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int gp = g + kLnPf;
    if (gp < NG)
      ln_load<HALF>(rb[gp % kLnSlots], grid, pb[gp], coff);
    else
      ln_load<HALF>(rb[gp % kLnSlots], grid, pb[gp - NG], coff_next);
    const h16x8 bh = rb[g % kLnSlots][0], bl = rb[g % kLnSlots][1];
    if (INIT)
      asm volatile(
          "v_mfma_f32_16x16x32_f16 %0, %1, %2, 0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
          : BK_ACC_W(acc[g])
          : "v"(ah), "v"(bh), "v"(al), "v"(bl));
    else
      asm volatile(
          "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
          : BK_ACC_RW(acc[g])
          : "v"(ah), "v"(bh), "v"(al), "v"(bl));
#if BK_LN_DUMMY
    {  // timing diagnostic only: BK_LN_DUMMY independent VALU ops after each triple (the MFMA shadow)
      float d0 = __builtin_bit_cast(float, (unsigned)g), d1 = d0;
#pragma unroll
      for (int k = 0; k < BK_LN_DUMMY; ++k) {
        if (k & 1)
          asm volatile("v_add_f32 %0, %0, %0" : "+v"(d1));
        else
          asm volatile("v_add_f32 %0, %0, %0" : "+v"(d0));
      }
      asm volatile("" ::"v"(d0), "v"(d1));
    }
#endif
  }
}

// ln_chunk with each group's two B-fragment reads (kLnPf groups ahead) issued between its three
// MFMAs in one asm block: wait (lgkmcnt(2 (kLnPf - 1)): the reads of the kLnPf - 1 blocks before
// are the only ones still allowed in flight), MFMA, read hi, MFMA, read lo, MFMA — one instruction in each MFMA's
// issue gap instead of two reads and a wait in one (a 16x16x32 MFMA holds the SIMD's issue for 8
// of its 16 cycles: MI355X_MICROARCH.md). The reads are invisible to the compiler: the grid offsets
// must be compile-time constants (immediates), the ring registers are only read by later blocks
// (after their wait), and the caller waits lgkmcnt(0) after its last chunk, before the ring
// registers can be reused. Same MFMAs on the same operands as ln_chunk: the sums are bitwise equal.
template <int NG, bool INIT, int HALF>
__device__ __forceinline__ void ln_chunk_il(f32x4 (&acc)[NG], h16x8 ah, h16x8 al, const unsigned char* grid,
                                            const int (&pb)[NG], int coff, int coff_next, h16x8 (&rb)[kLnSlots][2]) {
  static_assert(NG % kLnSlots == 0, "ln_chunk_il: the ring slot of a group must not depend on the chunk");
  const unsigned gbase = (unsigned)(uintptr_t)grid;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int gp = g + kLnPf;
    const unsigned addr = gbase + (unsigned)(gp < NG ? pb[gp] : pb[gp - NG]);
    h16x8& n0 = rb[gp % kLnSlots][0];
    h16x8& n1 = rb[gp % kLnSlots][1];
    if (gp < NG) {
      if (INIT)
        asm volatile(
            "s_waitcnt lgkmcnt(%10)\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %5, 0\n\t"
            "ds_read_b128 %1, %7 offset:%8\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %4, %5, %0\n\t"
            "ds_read_b128 %2, %7 offset:%9\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %6, %0"
            : BK_ACC_W(acc[g]), "=&v"(n0), "=&v"(n1)
            : "v"(ah), "v"(al), "v"(rb[g % kLnSlots][0]), "v"(rb[g % kLnSlots][1]), "v"(addr), "i"(coff), "i"(coff + HALF), "i"(2 * (kLnPf - 1)));
      else
        asm volatile(
            "s_waitcnt lgkmcnt(%10)\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %5, %0\n\t"
            "ds_read_b128 %1, %7 offset:%8\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %4, %5, %0\n\t"
            "ds_read_b128 %2, %7 offset:%9\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %6, %0"
            : BK_ACC_RW(acc[g]), "=&v"(n0), "=&v"(n1)
            : "v"(ah), "v"(al), "v"(rb[g % kLnSlots][0]), "v"(rb[g % kLnSlots][1]), "v"(addr), "i"(coff), "i"(coff + HALF), "i"(2 * (kLnPf - 1)));
    } else {
      if (INIT)
        asm volatile(
            "s_waitcnt lgkmcnt(%10)\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %5, 0\n\t"
            "ds_read_b128 %1, %7 offset:%8\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %4, %5, %0\n\t"
            "ds_read_b128 %2, %7 offset:%9\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %6, %0"
            : BK_ACC_W(acc[g]), "=&v"(n0), "=&v"(n1)
            : "v"(ah), "v"(al), "v"(rb[g % kLnSlots][0]), "v"(rb[g % kLnSlots][1]), "v"(addr), "i"(coff_next),
              "i"(coff_next + HALF), "i"(2 * (kLnPf - 1)));
      else
        asm volatile(
            "s_waitcnt lgkmcnt(%10)\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %5, %0\n\t"
            "ds_read_b128 %1, %7 offset:%8\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %4, %5, %0\n\t"
            "ds_read_b128 %2, %7 offset:%9\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %6, %0"
            : BK_ACC_RW(acc[g]), "=&v"(n0), "=&v"(n1)
            : "v"(ah), "v"(al), "v"(rb[g % kLnSlots][0]), "v"(rb[g % kLnSlots][1]), "v"(addr), "i"(coff_next),
              "i"(coff_next + HALF), "i"(2 * (kLnPf - 1)));
    }
  }
}

// the accumulators are written by MFMAs the compiler cannot see: wait out the MFMA write ->
// VALU read latency before the epilogue reads them. Each accumulator then passes through an empty
// asm that follows the wait (volatile asm keeps its order), so no read of it can be scheduled
// above the wait (an 8-wave variant of this kernel read one too early without this).
template <int NG>
__device__ __forceinline__ void ln_mfma_drain(f32x4 (&acc)[NG]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int g = 0; g < NG; ++g) asm volatile("" : BK_ACC_RW(acc[g]));
}

struct LnHeads {
  const float *wp, *bp, *wv, *bv, *w1t, *b1, *w2, *b2;
  int P;
  float* pf;
  float* v;
};

}  // namespace
}  // namespace bk
