// tables.h — piece / orientation / action tables of one board preset, built on the host at
// context creation and uploaded once. Replaces the action-string tables the reference builds
// from colosseumrl (`_set_all_possible_moves`, blokus_rl/colossumrl/blokus_wrapper.py:281-324).
#pragma once
#include <cstdint>
#include <vector>

namespace bk {

constexpr int kMaxN = 20;
constexpr int kMaxP = 4;
constexpr int kNumPieces = 21;
constexpr int kStateBytes = 384;
constexpr int kStateWords = kStateBytes / 4;  // 96 u32

// Byte offsets inside the 384-byte state (include/blokus_engine.h).
constexpr int kOffPieces = 320;
constexpr int kOffHash = 336;
constexpr int kOffToMove = 344;
constexpr int kOffPly = 348;
constexpr int kOffFlags = 352;
// u32-word offsets
constexpr int kWPieces = kOffPieces / 4;  // 80
constexpr int kWHash = kOffHash / 4;      // 84 (lo), 85 (hi)
constexpr int kWToMove = kOffToMove / 4;  // 86
constexpr int kWPly = kOffPly / 4;        // 87
constexpr int kWFlags = kOffFlags / 4;    // 88

constexpr uint32_t kFlagOver = 1u;
constexpr int kFlagDeadShift = 4;

// One "item" = one (orientation, origin row): the W origin columns of that row form W
// consecutive action ids starting at `base`. Packed in 64 bits:
//   [0,16)  base id   [16,21) origin row r   [21,26) W   [26,31) piece   [31,34) ncell
//   [34,64) 5 cells x 6 bits (dr:3 | dc:3 << 3); cells past ncell repeat cell 0, so a
//           kernel can always OR five shifted rows (idempotent) without a branch.
struct Item {
  static uint64_t pack(int base, int r, int W, int piece, int ncell, const int* dr, const int* dc) {
    uint64_t v = (uint64_t)base | ((uint64_t)r << 16) | ((uint64_t)W << 21) | ((uint64_t)piece << 26) |
                 ((uint64_t)ncell << 31);
    for (int k = 0; k < 5; ++k) {
      const int q = k < ncell ? k : 0;
      uint64_t cell = (uint64_t)(dr[q] | (dc[q] << 3));
      v |= cell << (34 + 6 * k);
    }
    return v;
  }
};

struct Preset {
  int N = 20, P = 4, max_cells = 5;
  int num_pieces = 21;
  int A = 0;            // action count
  int mask_words = 0;   // ceil(A/64)
  int mask_words32 = 0; // ceil(A/32)
  int num_items = 0;
  int corner_r[kMaxP] = {0}, corner_c[kMaxP] = {0};
  int piece_item_off[kNumPieces + 1] = {0};  // items of piece i: [off[i], off[i+1])
  std::vector<uint64_t> items;     // [num_items]
  // per fixed orientation (canonical order): piece, h, w, n, dr[5], dc[5] (unused cells = cell 0)
  std::vector<std::vector<int>> orients;
  std::vector<uint32_t> act;       // [A]: item index (low 16) | origin col << 16 | piece << 24
  std::vector<int32_t> act_table;  // [A*4]: piece, orientation, row, col
  std::vector<int16_t> act_cells;  // [A*5]: r*N + c, -1 pad
  uint32_t full_pieces = 0;
};

// Builds the preset; returns false on an unsupported (N, P, max_cells).
bool build_preset(int N, int P, int max_cells, Preset* out);

}  // namespace bk
