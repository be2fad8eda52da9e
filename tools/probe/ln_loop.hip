// Probe: the k_leafnet_x3 MFMA loop in isolation (timing experiment, not product). One workgroup
// per CU, WAVES waves; per wave NG pixel groups x MB output-channel blocks, 18 K chunks per layer,
// 3 v_mfma_f32_16x16x32_f16 per (group, block, chunk) on split operands. B fragments are read from
// an LDS grid (two ds_read_b128 per group, PF groups ahead, bank-conflict-free lane slots) or, in
// MODE 0, taken from registers (the MFMA floor). Prints cycles per layer (s_memtime, median wave).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

using h16x8 = _Float16 __attribute__((ext_vector_type(8)));
using f32x4 = float __attribute__((ext_vector_type(4)));

constexpr int kHalf = 32768;  // lo halves: byte offset from the hi halves (MODE 1)
constexpr int kPL = 7936;     // MODE 2: the leaf kernel's plane size (20x20 board, 22-slot rows)

// MODE 2: the leaf kernel's bank-aware pixel map (leafnet.hip LnPixMap<20>)
struct PixMap {
  int slot[25 * 16];
  constexpr PixMap() : slot() {
    bool used[400] = {};
    for (int i = 0; i < 400; ++i) slot[i] = -1;
    for (int g = 0; g < 25; ++g)
      for (int r = 0; r < 16; ++r)
        for (int p = 0; p < 400; ++p) {
          const int sl = (p / 20 + 1) * 22 + p % 20 + 1;
          if (!used[p] && sl % 16 == r) {
            used[p] = true;
            slot[g * 16 + r] = sl;
            break;
          }
        }
    int p = 0;
    for (int i = 0; i < 400; ++i) {
      if (slot[i] >= 0) continue;
      while (p < 400 && used[p]) ++p;
      used[p] = true;
      slot[i] = (p / 20 + 1) * 22 + p % 20 + 1;
    }
  }
};
__device__ constexpr PixMap kPix{};

template <int NG, int MB, int MODE, int PF, int HOFF>
__device__ __forceinline__ void chunk(f32x4 (&acc)[MB][NG], const h16x8 (&a)[MB][2], const unsigned char* grid,
                                      const int (&pb)[NG], int coff, int coffn, h16x8 (&rb)[8][2], int c) {
  constexpr int S = PF + 1;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int i = c * NG + g;  // flattened group index (c is a compile-time constant after unrolling)
    if (MODE >= 1) {
      const int gp = g + PF;  // MODE 3/4: kHalf offset
      const unsigned char* q = grid + (gp < NG ? pb[gp] + coff : pb[gp - NG] + coffn);
      rb[(i + PF) % S][0] = *reinterpret_cast<const h16x8*>(q);
      rb[(i + PF) % S][1] = *reinterpret_cast<const h16x8*>(q + HOFF);
    }
    const h16x8 bh = rb[i % S][0], bl = rb[i % S][1];
#pragma unroll
    for (int m = 0; m < MB; ++m)
      asm volatile(
          "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %3, %2, %0\n\t"
          "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
          : "+a"(acc[m][g])
          : "v"(a[m][0]), "v"(bh), "v"(a[m][1]), "v"(bl));
  }
}

template <int NG, int MB, int MODE, int PF, int WAVES, int PLS, int HOFF>
__global__ __launch_bounds__(64 * WAVES, 1) void k(const h16x8* __restrict__ w, float* out,
                                                   unsigned long long* clk, int layers) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, l = tid & 63, n = l & 15, ks = l >> 4, wave = tid >> 6;
  for (int i = tid; i < 16 * kPL / 16; i += 64 * WAVES) {
    h16x8 v;
    for (int e = 0; e < 8; ++e) v[e] = (_Float16)(((i * 8 + e) * 37 % 97) * 0.01f);
    reinterpret_cast<h16x8*>(lds)[i] = v;
  }
  __syncthreads();
  int pb[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g)
    pb[g] = MODE == 2   ? kPix.slot[16 * g + n] * 16
            : MODE == 5 ? (g < 24 ? kPix.slot[16 * g + n] * 16 : (400 + n) * 16)      // leaf map, group 24 fixed
            : MODE == 3 ? ((g * 16 + (n * 5 + g) % 16) * 16) % 16384 + 1024          // permuted within 256 B
            : MODE == 4 || MODE == 6 ? (64 + n + 16 * ((g * 7 + n * 3) % 25)) * 16    // scattered, n distinct
            : MODE == 7 ? kPix.slot[16 * g + n] * 16
                        : ((g * 16 + n) * 16) % 16384 + 1024;
  f32x4 acc[MB][NG];
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[m][g] = f32x4{0.f, 0.f, 0.f, 0.f};
  h16x8 rb[8][2];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    rb[s][0] = w[(s * 2) * 64 + l];
    rb[s][1] = w[(s * 2 + 1) * 64 + l];
  }
  h16x8 a[2][MB][2];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int layer = 0; layer < layers; ++layer) {
    if (MODE >= 1) {
#pragma unroll
      for (int g = 0; g < PF; ++g) {
        rb[g][0] = *reinterpret_cast<const h16x8*>(lds + pb[g] + ks * PLS);
        rb[g][1] = *reinterpret_cast<const h16x8*>(lds + pb[g] + ks * PLS + HOFF);
      }
    }
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      a[0][m][0] = w[((wave * MB + m) * 2) * 64 + l];
      a[0][m][1] = w[((wave * MB + m) * 2 + 1) * 64 + l];
    }
#pragma unroll
    for (int c = 0; c < 18; ++c) {
      if (c + 1 < 18) {
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          a[(c + 1) & 1][m][0] = w[(((c + 1) * 8 + wave * MB + m) * 2) * 64 + l];
          a[(c + 1) & 1][m][1] = w[(((c + 1) * 8 + wave * MB + m) * 2 + 1) * 64 + l];
        }
      }
      auto co = [&](int cc) {
        if (MODE != 2 && MODE != 5 && MODE != 6) return ks * PLS + (cc % 9) * 16;
        const int t = cc >> 1;
        return (4 * (cc & 1) + ks) * kPL + ((t / 3 - 1) * 22 + (t % 3 - 1)) * 16;
      };
      const int coff = co(c), coffn = co(c + 1 < 18 ? c + 1 : c);
      chunk<NG, MB, MODE, PF, HOFF>(acc, a[c & 1], lds, pb, coff, coffn, rb, c);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int g = 0; g < NG; ++g) s += acc[m][g][0] + acc[m][g][1] + acc[m][g][2] + acc[m][g][3];
  out[blockIdx.x * 64 * WAVES + tid] = s;
  if (l == 0) clk[blockIdx.x * WAVES + wave] = t1 - t0;
}

template <int NG, int MB, int MODE, int PF, int WAVES, int PLS = 4096, int HOFF = (MODE == 2 || MODE == 5) ? 8 * kPL : kHalf>
void run(const char* name, const h16x8* w, float* out, unsigned long long* clk, int blocks) {
  const int layers = 10;
  hipFuncSetAttribute((const void*)k<NG, MB, MODE, PF, WAVES, PLS, HOFF>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((k<NG, MB, MODE, PF, WAVES, PLS, HOFF>), dim3(blocks), dim3(64 * WAVES), 16 * kPL, 0, w, out, clk, layers);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * WAVES);
  hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double med = (double)h[h.size() / 2] / layers;
  const double floor = 18.0 * NG * MB * 3 * 16;
  printf("%-34s cycles/layer %8.0f  floor %6.0f  ratio %.3f  (%.1f extra cycles per group-step)\n", name, med, floor,
         med / floor, (med - floor) / (18.0 * NG));
}

int main() {
  h16x8* w;
  float* out;
  unsigned long long* clk;
  hipMalloc(&w, 1 << 22);
  hipMemset(w, 0, 1 << 22);
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&clk, 256 * 8 * 8);
  const int B = 256;
  run<25, 1, 0, 2, 4>("4w NG25 MB1 regs (floor)", w, out, clk, B);
  run<25, 1, 1, 2, 4>("4w NG25 MB1 lds pf2", w, out, clk, B);
  run<25, 1, 1, 4, 4>("4w NG25 MB1 lds pf4", w, out, clk, B);
  run<25, 1, 2, 2, 4>("4w NG25 MB1 leaf map pf2", w, out, clk, B);
  run<25, 1, 2, 4, 4>("4w NG25 MB1 leaf map pf4", w, out, clk, B);
  run<25, 1, 5, 2, 4>("4w NG25 MB1 leaf map g24 fixed pf2", w, out, clk, B);
  run<25, 1, 3, 2, 4>("4w NG25 MB1 permuted-256B pf2", w, out, clk, B);
  run<25, 1, 4, 2, 4, kPL, 8 * kPL>("4w scattered, leaf planes", w, out, clk, B);
  run<25, 1, 6, 2, 4, kPL, 8 * kPL>("4w scattered, leaf chunk offsets", w, out, clk, B);
  run<25, 1, 7, 2, 4, kPL, 8 * kPL>("4w leaf map, simple chunk offsets", w, out, clk, B);
  run<25, 1, 4, 2, 4, 4096, 8 * kPL>("4w scattered, leaf lo offset", w, out, clk, B);
  run<25, 1, 4, 2, 4, kPL, kHalf>("4w scattered, leaf plane stride", w, out, clk, B);
  run<25, 1, 4, 2, 4>("4w NG25 MB1 scattered pf2", w, out, clk, B);
  run<13, 2, 0, 2, 4>("4w NG13 MB2 regs (floor)", w, out, clk, B);
  run<13, 2, 1, 2, 4>("4w NG13 MB2 lds pf2", w, out, clk, B);
  run<13, 2, 1, 4, 4>("4w NG13 MB2 lds pf4", w, out, clk, B);
  run<13, 1, 0, 2, 8>("8w NG13 MB1 regs (floor)", w, out, clk, B);
  run<13, 1, 1, 2, 8>("8w NG13 MB1 lds pf2", w, out, clk, B);
  run<13, 1, 1, 4, 8>("8w NG13 MB1 lds pf4", w, out, clk, B);
  return 0;
}
