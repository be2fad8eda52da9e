// tables.cpp — host-side construction of the action space of one preset.
//
// Canonical action order (the reference's colosseumrl order is unpinned):
//   id = enumeration over (piece 0..20, orientation, origin row, origin col), where a piece's
//   orientation o is the o-th distinct shape met while applying the square's symmetries in the
//   order  (r,c) (c,-r) (-r,-c) (-c,r) (r,-c) (-c,-r) (-r,c) (c,r),  each shape normalised to
//   min row/col 0. 20x20 gives 91 orientations and 30433 ids (docs/README.md:128).
#include "tables.h"

#include <cstring>

namespace bk {
namespace {

// The 21 standard pieces drawn on a 5x5 grid ('#' = cell), in the engine's piece order.
const char* kPieceArt[kNumPieces] = {
    "#",                              // monomino
    "##",                             // domino
    "###",                            // I3
    "#.|##",                          // V3
    "####",                           // I4
    "#.|#.|##",                       // L4
    "###|.#.",                        // T4
    ".##|##.",                        // S4
    "##|##",                          // O4
    ".##|##.|.#.",                    // F5
    "#####",                          // I5
    "#.|#.|#.|##",                    // L5
    ".#|.#|##|#.",                    // N5
    "##|##|#.",                       // P5
    "###|.#.|.#.",                    // T5
    "#.#|###",                        // U5
    "#..|#..|###",                    // V5
    "#..|##.|.##",                    // W5
    ".#.|###|.#.",                    // X5
    ".#|##|.#|.#",                    // Y5
    "##.|.#.|.##",                    // Z5
};

// A shape is a 25-bit mask over a 5x5 box, bit (r*5 + c).
uint32_t art_mask(const char* s, int* ncell) {
  uint32_t m = 0;
  int r = 0, c = 0;
  *ncell = 0;
  for (; *s; ++s) {
    if (*s == '|') { ++r; c = 0; continue; }
    if (*s == '#') { m |= 1u << (r * 5 + c); ++*ncell; }
    ++c;
  }
  return m;
}

uint32_t apply_sym(uint32_t m, int k) {
  int rr[25], cc[25], n = 0;
  for (int b = 0; b < 25; ++b) {
    if (!((m >> b) & 1u)) continue;
    int r = b / 5, c = b % 5, tr, tc;
    switch (k) {
      case 0: tr = r; tc = c; break;
      case 1: tr = c; tc = -r; break;
      case 2: tr = -r; tc = -c; break;
      case 3: tr = -c; tc = r; break;
      case 4: tr = r; tc = -c; break;
      case 5: tr = -c; tc = -r; break;
      case 6: tr = -r; tc = c; break;
      default: tr = c; tc = r; break;
    }
    rr[n] = tr; cc[n] = tc; ++n;
  }
  int minr = 99, minc = 99;
  for (int i = 0; i < n; ++i) { if (rr[i] < minr) minr = rr[i]; if (cc[i] < minc) minc = cc[i]; }
  uint32_t out = 0;
  for (int i = 0; i < n; ++i) out |= 1u << ((rr[i] - minr) * 5 + (cc[i] - minc));
  return out;
}

}  // namespace

bool build_preset(int N, int P, int max_cells, Preset* pr) {
  if (N < 5 || N > kMaxN || (P != 2 && P != 4) || max_cells < 1 || max_cells > 5) return false;
  Preset& p = *pr;
  p = Preset();
  p.N = N; p.P = P; p.max_cells = max_cells;
  int ncells[kNumPieces];
  uint32_t base_mask[kNumPieces];
  p.num_pieces = 0;
  for (int i = 0; i < kNumPieces; ++i) {
    base_mask[i] = art_mask(kPieceArt[i], &ncells[i]);
    if (ncells[i] <= max_cells) p.num_pieces = i + 1;
  }
  p.full_pieces = p.num_pieces >= 32 ? 0xFFFFFFFFu : ((1u << p.num_pieces) - 1u);
  if (P == 4) {
    const int r[4] = {0, 0, N - 1, N - 1}, c[4] = {0, N - 1, 0, N - 1};
    for (int k = 0; k < 4; ++k) { p.corner_r[k] = r[k]; p.corner_c[k] = c[k]; }
  } else {
    p.corner_r[0] = 0; p.corner_c[0] = 0; p.corner_r[1] = N - 1; p.corner_c[1] = N - 1;
  }

  int id = 0;
  for (int pc = 0; pc < p.num_pieces; ++pc) {
    p.piece_item_off[pc] = p.num_items;
    uint32_t seen[8];
    int nseen = 0;
    for (int k = 0; k < 8; ++k) {
      uint32_t m = apply_sym(base_mask[pc], k);
      bool dup = false;
      for (int j = 0; j < nseen; ++j) dup |= seen[j] == m;
      if (dup) continue;
      const int o = nseen;
      seen[nseen++] = m;
      int dr[5], dc[5], n = 0, h = 0, w = 0;
      for (int b = 0; b < 25; ++b)
        if ((m >> b) & 1u) {
          dr[n] = b / 5; dc[n] = b % 5;
          if (dr[n] + 1 > h) h = dr[n] + 1;
          if (dc[n] + 1 > w) w = dc[n] + 1;
          ++n;
        }
      {
        std::vector<int> od = {pc, h, w, n};
        for (int q = 0; q < 5; ++q) od.push_back(q < n ? dr[q] : dr[0]);
        for (int q = 0; q < 5; ++q) od.push_back(q < n ? dc[q] : dc[0]);
        p.orients.push_back(od);
      }
      const int R = N - h + 1, W = N - w + 1;
      for (int r = 0; r < R; ++r) {
        const int item = p.num_items++;
        p.items.push_back(Item::pack(id, r, W, pc, n, dr, dc));
        for (int c = 0; c < W; ++c) {
          p.act.push_back((uint32_t)item | ((uint32_t)c << 16) | ((uint32_t)pc << 24));
          p.act_table.insert(p.act_table.end(), {pc, o, r, c});
          for (int q = 0; q < 5; ++q)
            p.act_cells.push_back(q < n ? (int16_t)((r + dr[q]) * N + c + dc[q]) : (int16_t)-1);
          ++id;
        }
      }
    }
  }
  for (int pc = p.num_pieces; pc <= kNumPieces; ++pc) p.piece_item_off[pc] = p.num_items;
  p.A = id;
  p.mask_words = (id + 63) / 64;
  p.mask_words32 = (id + 31) / 32;
  return id < 65536 && p.num_items < 65536;
}

}  // namespace bk
