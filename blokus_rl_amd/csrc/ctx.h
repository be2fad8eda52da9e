// ctx.h — host-side context of the engine library (one board preset on one device).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "common.h"
#include "tables.h"

struct bk_ctx {
  bk::Preset pre;
  bk::DevPreset dp;
  int device = 0;
  uint64_t* d_items = nullptr;
  uint4* d_act_it = nullptr;  // [A] item + act word per action (place_action)
  uint32_t* d_pack = nullptr;       // [W64] x 4: k_legal_mask_staged's word assembly table
  bool legal_items_kernel = false;  // BK_LEGAL_KERNEL=items selects the item-loop kernel (A/B)
  int legal_wpb = 1;                // BK_LEGAL_WPB: variant of k_legal_mask_rows (A/B knob)
};

namespace bk {
void set_error(const std::string& msg);
int hip_check(hipError_t e, const char* what);
// Launch-error check after a kernel launch.
int launch_check(const char* what);
// Raise the dynamic-LDS limit of kernels fns[0..n) to `bytes` on the current device, once per
// (device, kernel); thread-safe.
int set_max_dynamic_lds(const void* const* fns, int n, int bytes);
}  // namespace bk

#define BK_REQUIRE(cond, msg)            \
  do {                                   \
    if (!(cond)) {                       \
      bk::set_error(msg);                \
      return BK_EINVAL;                  \
    }                                    \
  } while (0)
