// Bucket sort of the MSM digits.  The digits themselves (and the coarse
// histogram) come from k_msm_digits in msm_impl.hpp, which decodes scalars.
//
// The sort only has to GROUP entries by bucket: the accumulation adds every
// point of a bucket exactly, so the order inside a bucket does not matter and no
// pass needs to be stable.  That makes each level a plain counting sort with
// LDS-atomic cursors:
//   k_msm_s1_scan     one block: exclusive scan of the NC coarse counts, and the
//                     part table -- a coarse bin above S2_BIG entries (skewed
//                     scalars, e.g. boolean witness wires) is split into parts.
//   k_msm_s1_scatter  digits -> coarse bins (8-B entries bucket | value << 32).
//   k_msm_s2_local    one block per part.  A single-part bin is finished here:
//                     LDS histogram of its 2^F buckets, LDS scan, offsets[];
//                     a bin of <= S2_STAGE entries (the usual case: ~4K) is held
//                     in registers, sorted into LDS and copied out coalesced,
//                     a larger one is read twice and scattered.  A part of a
//                     split bin only adds its LDS histogram into fcount
//                     (global atomics, <= 2^F each).
//   k_msm_s2_scan     split bins: scan of fcount -> offsets and cursors.
//   k_msm_s2_scatter  split bins: per part, one global range reservation per
//                     bucket, then the scatter.
// Traffic per entry: 8 B written in pass 1; 8 B read + 8 B written here (staged bins).
#include "msm.hpp"
#include "runtime.hpp"
#include "sort_util.hpp"

namespace gm {

static __global__ void __launch_bounds__(1024) k_msm_s1_scan(const uint32_t* __restrict__ ccount, uint32_t NC,
                                                             uint32_t T, uint32_t* __restrict__ cbase,
                                                             uint32_t* __restrict__ ccursor,
                                                             uint32_t* __restrict__ pbase,
                                                             uint32_t* __restrict__ offsets) {
  __shared__ uint32_t a[8192];
  __shared__ uint32_t wsum[17];
  const uint32_t t = threadIdx.x;
  for (uint32_t q = t; q < NC; q += S_THREADS) a[q] = ccount[q];
  const uint32_t total = block_excl_scan(a, NC, wsum);
  for (uint32_t q = t; q < NC; q += S_THREADS) {
    cbase[q] = a[q];
    ccursor[q] = a[q];
    const uint32_t cnt = ccount[q];
    a[q] = cnt > S2_BIG ? (cnt + S2_BIG - 1) / S2_BIG : 1u;
  }
  if (t == 0) {
    cbase[NC] = total;
    offsets[T] = total;
  }
  const uint32_t parts = block_excl_scan(a, NC, wsum);
  for (uint32_t q = t; q < NC; q += S_THREADS) pbase[q] = a[q];
  if (t == 0) pbase[NC] = parts;
}

// Pass-1 partition: block (chunk, w) moves the non-zero digits of window w of
// S1_PTS points into the coarse bins: LDS histogram with ranks, one global range
// reservation per touched bin, then the 8-B entries (bucket | value << 32).  In
// the plain layout with 2^F <= nb the block touches only window w's bins
// [h0, h0 + nh), so its LDS is small and its write runs long (S1_PTS / nh
// entries per bin on average).
constexpr uint32_t S1_PPT = 8, S1_PTS = S_THREADS * S1_PPT;
static __global__ void __launch_bounds__(1024) k_msm_s1_scatter(const uint32_t* __restrict__ dig, uint32_t n,
                                                                uint32_t nb, uint32_t shared_stride, uint32_t F,
                                                                uint32_t NC, uint32_t nh,
                                                                uint32_t* __restrict__ ccursor,
                                                                uint64_t* __restrict__ tmp) {
  extern __shared__ uint32_t s1_lds[];
  uint32_t* hist = s1_lds;
  uint32_t* cur = s1_lds + nh;
  const uint32_t t = threadIdx.x, w = blockIdx.y, base = blockIdx.x * S1_PTS;
  const uint32_t wb = shared_stride ? 0u : w * nb;     // window's first bucket
  const uint32_t h0 = nh == NC ? 0u : wb >> F;          // first coarse bin in LDS
  for (uint32_t q = t; q < nh; q += S_THREADS) hist[q] = 0;
  __syncthreads();
  uint32_t dv[S1_PPT], rk[S1_PPT];
#pragma unroll
  for (uint32_t r = 0; r < S1_PPT; r++) {
    const uint32_t i = base + r * S_THREADS + t;
    dv[r] = i < n ? dig[(size_t)w * n + i] : 0xffffffffu;
    if (dv[r] != 0xffffffffu) rk[r] = lds_rank_add(hist, (((dv[r] & 0x7fffffffu) + wb) >> F) - h0);
  }
  __syncthreads();
  for (uint32_t q = t; q < nh; q += S_THREADS)
    if (hist[q]) cur[q] = atomicAdd(&ccursor[h0 + q], hist[q]);
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < S1_PPT; r++) {
    if (dv[r] == 0xffffffffu) continue;
    const uint32_t i = base + r * S_THREADS + t;
    const uint32_t b = (dv[r] & 0x7fffffffu) + wb;
    const uint32_t v = (shared_stride ? w * shared_stride + i : i) | (dv[r] & 0x80000000u);
    tmp[cur[(b >> F) - h0] + rk[r]] = ((uint64_t)v << 32) | b;
  }
}

// block j -> (coarse bin, part): largest H with pbase[H] <= j
// (no split bins, the usual case: part j is bin j)
__device__ __forceinline__ void s2_locate(const uint32_t* __restrict__ pbase, uint32_t NC, uint32_t j, uint32_t* sh) {
  if (threadIdx.x == 0) {
    uint32_t lo = 0, hi = NC;  // pbase[lo] <= j < pbase[hi]
    if (pbase[NC] == NC) lo = j, hi = j + 1;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pbase[mid] <= j) lo = mid;
      else hi = mid;
    }
    sh[0] = lo;
    sh[1] = j - pbase[lo];
  }
  __syncthreads();
}

// LDS layout: hist[2^F] | staged keys[S2_STAGE] | staged values[S2_STAGE].
static __global__ void __launch_bounds__(1024) k_msm_s2_local(const uint64_t* __restrict__ tmp,
                                                              const uint32_t* __restrict__ cbase,
                                                              const uint32_t* __restrict__ pbase, uint32_t NC,
                                                              uint32_t F, uint32_t T, uint32_t* __restrict__ fcount,
                                                              uint32_t* __restrict__ keys_out,
                                                              uint32_t* __restrict__ vals_out,
                                                              uint32_t* __restrict__ offsets) {
  extern __shared__ uint32_t s2_lds[];
  __shared__ uint32_t sh[2], wsum[17];
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  // no split bins (the usual case): part j is bin j -- the three loads issue together
  const uint32_t parts = pbase[NC];
  const uint32_t cj0 = j < NC ? cbase[j] : 0u, cj1 = j < NC ? cbase[j + 1] : 0u;
  if (j >= parts) return;
  uint32_t H, p, start, cnt;
  if (parts == NC) {
    H = j;
    p = 0;
    start = cj0;
    cnt = cj1 - cj0;
  } else {
    s2_locate(pbase, NC, j, sh);
    H = sh[0];
    p = sh[1];
    start = cbase[H];
    cnt = cbase[H + 1] - start;
  }
  const uint32_t b0 = H << F, nf = min(1u << F, T - b0), fmask = (1u << F) - 1;
  uint32_t* hist = s2_lds;
  for (uint32_t q = t; q < nf; q += S_THREADS) hist[q] = 0;
  __syncthreads();
  if (cnt <= S2_STAGE) {
    // whole bin in registers: local counting sort staged in LDS, then one
    // coalesced copy of the bin's sorted keys / values
    constexpr uint32_t IPT = S2_STAGE / S_THREADS;
    uint64_t x[IPT];
    uint32_t rk[IPT];
#pragma unroll
    for (uint32_t it = 0; it < IPT; it++) {
      const uint32_t e = it * S_THREADS + t;
      if (e < cnt) {
        x[it] = tmp[start + e];
        rk[it] = lds_rank_add(hist, (uint32_t)x[it] & fmask);
      }
    }
    block_excl_scan(hist, nf, wsum);
    for (uint32_t f = t; f < nf; f += S_THREADS) offsets[b0 + f] = start + hist[f];
    uint32_t* sk = s2_lds + nf;
    uint32_t* sv = sk + S2_STAGE;
#pragma unroll
    for (uint32_t it = 0; it < IPT; it++) {
      const uint32_t e = it * S_THREADS + t;
      if (e < cnt) {
        const uint32_t b = (uint32_t)x[it];
        const uint32_t pos = hist[b & fmask] + rk[it];
        sk[pos] = b;
        sv[pos] = (uint32_t)(x[it] >> 32);
      }
    }
    __syncthreads();
    for (uint32_t q = t; q < cnt; q += S_THREADS) {
      keys_out[start + q] = sk[q];
      vals_out[start + q] = sv[q];
    }
  } else if (cnt <= S2_BIG) {
    // too large to stage: two reads, scattered writes
    for (uint32_t e = t; e < cnt; e += S_THREADS) lds_rank_add(hist, (uint32_t)tmp[start + e] & fmask);
    block_excl_scan(hist, nf, wsum);
    for (uint32_t f = t; f < nf; f += S_THREADS) offsets[b0 + f] = start + hist[f];
    __syncthreads();
    for (uint32_t e = t; e < cnt; e += S_THREADS) {
      const uint64_t x = tmp[start + e];
      const uint32_t b = (uint32_t)x;
      const uint32_t pos = start + lds_rank_add(hist, b & fmask);
      keys_out[pos] = b;
      vals_out[pos] = (uint32_t)(x >> 32);
    }
  } else {
    const uint32_t lo = p * S2_BIG, hi = min(lo + S2_BIG, cnt);
    for (uint32_t e = lo + t; e < hi; e += S_THREADS) lds_rank_add(hist, (uint32_t)tmp[start + e] & fmask);
    __syncthreads();
    for (uint32_t f = t; f < nf; f += S_THREADS)
      if (hist[f]) atomicAdd(&fcount[b0 + f], hist[f]);
  }
}

static __global__ void __launch_bounds__(1024) k_msm_s2_scan(const uint32_t* __restrict__ cbase, uint32_t F,
                                                             uint32_t T, uint32_t* __restrict__ fcount,
                                                             uint32_t* __restrict__ offsets) {
  extern __shared__ uint32_t hist[];
  __shared__ uint32_t wsum[17];
  const uint32_t H = blockIdx.x, t = threadIdx.x;
  const uint32_t start = cbase[H], cnt = cbase[H + 1] - start;
  if (cnt <= S2_BIG) return;
  const uint32_t b0 = H << F, nf = min(1u << F, T - b0);
  for (uint32_t f = t; f < nf; f += S_THREADS) hist[f] = fcount[b0 + f];
  block_excl_scan(hist, nf, wsum);
  for (uint32_t f = t; f < nf; f += S_THREADS) {
    offsets[b0 + f] = start + hist[f];
    fcount[b0 + f] = start + hist[f];  // now the bucket's write cursor
  }
}

static __global__ void __launch_bounds__(1024) k_msm_s2_scatter(const uint64_t* __restrict__ tmp,
                                                                const uint32_t* __restrict__ cbase,
                                                                const uint32_t* __restrict__ pbase, uint32_t NC,
                                                                uint32_t F, uint32_t T,
                                                                uint32_t* __restrict__ fcursor,
                                                                uint32_t* __restrict__ keys_out,
                                                                uint32_t* __restrict__ vals_out) {
  extern __shared__ uint32_t s2_lds[];
  __shared__ uint32_t sh[2];
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  if (j >= pbase[NC] || pbase[NC] == NC) return;  // no split bins: nothing to do
  s2_locate(pbase, NC, j, sh);
  const uint32_t H = sh[0], p = sh[1];
  const uint32_t start = cbase[H], cnt = cbase[H + 1] - start;
  if (cnt <= S2_BIG) return;
  const uint32_t b0 = H << F, nf = min(1u << F, T - b0), fmask = (1u << F) - 1;
  uint32_t* hist = s2_lds;
  uint32_t* cur = s2_lds + nf;
  for (uint32_t q = t; q < nf; q += S_THREADS) hist[q] = 0;
  __syncthreads();
  const uint32_t lo = p * S2_BIG, hi = min(lo + S2_BIG, cnt);
  for (uint32_t e = lo + t; e < hi; e += S_THREADS) lds_rank_add(hist, (uint32_t)tmp[start + e] & fmask);
  __syncthreads();
  for (uint32_t f = t; f < nf; f += S_THREADS)
    if (hist[f]) cur[f] = atomicAdd(&fcursor[b0 + f], hist[f]);
  __syncthreads();
  for (uint32_t e = lo + t; e < hi; e += S_THREADS) {
    const uint64_t x = tmp[start + e];
    const uint32_t b = (uint32_t)x;
    const uint32_t pos = lds_rank_add(cur, b & fmask);
    keys_out[pos] = b;
    vals_out[pos] = (uint32_t)(x >> 32);
  }
}

int msm_sort_digits(gm_ctx* ctx, const SortGeom& g, size_t n, uint32_t W, uint32_t nb, uint32_t shared_stride,
                    const uint32_t* dig, const uint32_t* ccount, uint32_t* cbase, uint32_t* ccursor, uint32_t* pbase,
                    uint64_t* tmp, uint32_t* fcount, uint32_t* keys_out, uint32_t* vals_out, uint32_t* offsets) {
  if (g.NC == 0 || g.NC > 8192 || g.F > 13) {
    set_error("msm sort: bad geometry");
    return GM_ERR_INVALID;
  }
  hipStream_t st = ctx->stream;
  hipLaunchKernelGGL(k_msm_s1_scan, dim3(1), dim3(S_THREADS), 0, st, ccount, g.NC, g.T, cbase, ccursor, pbase,
                     offsets);
  // coarse bins one window touches: its own nb >> F in the plain layout
  const uint32_t nh = (!shared_stride && (1u << g.F) <= nb) ? nb >> g.F : g.NC;
  hipLaunchKernelGGL(k_msm_s1_scatter, dim3(blocks_for(n, S1_PTS), W), dim3(S_THREADS), 2 * sizeof(uint32_t) * nh, st,
                     dig, (uint32_t)n, nb, shared_stride, g.F, g.NC, nh, ccursor, tmp);
  const uint32_t nfmax = std::min<uint32_t>(1u << g.F, g.T);
  // every coarse bin has >= 1 part; split bins add at most M / S2_BIG more
  const size_t maxparts = (size_t)g.NC + g.M / S2_BIG + 1;
  GM_HIP(hipMemsetAsync(fcount, 0, sizeof(uint32_t) * g.T, st));
  hipLaunchKernelGGL(k_msm_s2_local, dim3((unsigned)maxparts), dim3(S_THREADS),
                     sizeof(uint32_t) * (nfmax + 2 * S2_STAGE), st, tmp, cbase, pbase, g.NC, g.F, g.T, fcount,
                     keys_out, vals_out, offsets);
  hipLaunchKernelGGL(k_msm_s2_scan, dim3(g.NC), dim3(S_THREADS), sizeof(uint32_t) * nfmax, st, cbase, g.F, g.T,
                     fcount, offsets);
  hipLaunchKernelGGL(k_msm_s2_scatter, dim3((unsigned)maxparts), dim3(S_THREADS), 2 * sizeof(uint32_t) * nfmax, st,
                     tmp, cbase, pbase, g.NC, g.F, g.T, fcount, keys_out, vals_out);
  GM_HIP(hipGetLastError());
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
