// Radix sort of the MSM digit keys (bucket index) with their point-index
// payloads -- the one non-templated piece of the MSM pipeline, kept in its own
// translation unit (rocPRIM's sort is heavy to compile).
//
// (Measured on MI355X at 2^20 BN254 / 16.7M pairs with 20-bit keys: the
// library default 0.43 ms; forced 8-bit warp-match places 0.59 ms; 11-bit
// places, two passes, 1.88 ms -- the default stays.)
#include <hipcub/hipcub.hpp>

#include "msm.hpp"
#include "runtime.hpp"

namespace gm {

int msm_sort_pairs(gm_ctx* ctx, Arena& arena, const uint32_t* keys_in, uint32_t* keys_out,
                   const uint32_t* vals_in, uint32_t* vals_out, size_t M, int end_bit) {
  size_t tmp_bytes = 0;
  GM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys_in, keys_out, vals_in, vals_out, (int)M, 0,
                                            end_bit, ctx->stream));
  DevBuf tmp;
  if (int rc = tmp.alloc(arena, tmp_bytes)) return rc;
  GM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tmp_bytes, keys_in, keys_out, vals_in, vals_out, (int)M, 0,
                                            end_bit, ctx->stream));
  return GM_OK;
}

// Shared-bucket cost model: n*W accumulation adds + ~3 reduction adds per
// bucket, paid once (not per window).  Picks c = 20 / W = 13 for 2^20 BN254
// points and c = 22 / W = 12 for 2^24.
MsmPrecomp msm_choose_precomp(size_t n, int bits) {
  MsmPrecomp best;
  double best_cost = 1e300;
  for (uint32_t c = 8; c <= 24; c++) {
    const uint32_t W = (uint32_t)((bits + 1 + c - 1) / c);
    const double cost = (double)n * W + 3.0 * (double)(1u << (c - 1));
    if (cost < best_cost) {
      best_cost = cost;
      best.c = c;
      best.W = W;
    }
  }
  best.stride = n;
  return best;
}

}  // namespace gm
