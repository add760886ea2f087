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

// LDS bytes one workgroup may allocate on `device` (queried once per device)
static size_t device_lds_per_block(int device) {
  static std::mutex mu;
  static std::map<int, size_t> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess) {
    (void)hipGetLastError();
    v = 64 << 10;
  }
  return cache[device] = (size_t)v;
}

static __global__ void __launch_bounds__(1024) k_msm_s1_scan(const uint32_t* __restrict__ ccount, uint32_t NC,
                                                             uint32_t T, uint32_t psz, uint32_t* __restrict__ cbase,
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
    a[q] = cnt > psz ? (cnt + psz - 1) / psz : 1u;
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

// The same partition with coalesced writes: the block's entries are first
// sorted by bin into an LDS stage (rank + the bin's local base), then written out
// in stage order, so consecutive lanes store consecutive 8-B entries of one
// bin's run instead of 64 scattered 8-B stores per wave instruction.  PPT points
// per thread (S_THREADS * PPT entries staged, 8 B each).
template <uint32_t PPT>
static __global__ void __launch_bounds__(1024) k_msm_s1_scatter_st(const uint32_t* __restrict__ dig, uint32_t n,
                                                                   uint32_t nb, uint32_t shared_stride, uint32_t F,
                                                                   uint32_t NC, uint32_t nh,
                                                                   uint32_t* __restrict__ ccursor,
                                                                   uint64_t* __restrict__ tmp) {
  constexpr uint32_t PTS = S_THREADS * PPT;
  extern __shared__ uint64_t s1s_lds[];
  uint64_t* stage = s1s_lds;
  uint32_t* hist = reinterpret_cast<uint32_t*>(s1s_lds + PTS);
  uint32_t* cur = hist + nh;   // global base of the block's run in bin q
  uint32_t* lb = cur + nh;     // local base of bin q in the stage
  uint32_t* wsum = lb + nh;    // 17 words
  const uint32_t t = threadIdx.x, w = blockIdx.y, base = blockIdx.x * PTS;
  const uint32_t wb = shared_stride ? 0u : w * nb;
  const uint32_t h0 = nh == NC ? 0u : wb >> F;
  for (uint32_t q = t; q < nh; q += S_THREADS) hist[q] = 0;
  __syncthreads();
  uint32_t dv[PPT], rk[PPT];
#pragma unroll
  for (uint32_t r = 0; r < PPT; r++) {
    const uint32_t i = base + r * S_THREADS + t;
    dv[r] = i < n ? dig[(size_t)w * n + i] : 0xffffffffu;
    if (dv[r] != 0xffffffffu) rk[r] = lds_rank_add(hist, (((dv[r] & 0x7fffffffu) + wb) >> F) - h0);
  }
  __syncthreads();
  for (uint32_t q = t; q < nh; q += S_THREADS) {
    const uint32_t h = hist[q];
    cur[q] = h ? atomicAdd(&ccursor[h0 + q], h) : 0u;
    lb[q] = h;
  }
  const uint32_t total = block_excl_scan(lb, nh, wsum);  // synchronises
#pragma unroll
  for (uint32_t r = 0; r < PPT; r++) {
    if (dv[r] == 0xffffffffu) continue;
    const uint32_t i = base + r * S_THREADS + t;
    const uint32_t b = (dv[r] & 0x7fffffffu) + wb;
    const uint32_t v = (shared_stride ? w * shared_stride + i : i) | (dv[r] & 0x80000000u);
    stage[lb[(b >> F) - h0] + rk[r]] = ((uint64_t)v << 32) | b;
  }
  __syncthreads();
  for (uint32_t q = t; q < total; q += S_THREADS) {
    const uint64_t e = stage[q];
    const uint32_t h = ((uint32_t)e >> F) - h0;
    tmp[cur[h] + (q - lb[h])] = e;
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

// ---- middle pass of a three-level sort (large MSMs) ------------------------
// Pass 1 then partitions into super-bins s = b >> (F + G) (few enough that a
// pass-1 block writes long runs), and this pass splits every super-bin into its
// 2^G coarse bins H = b >> F, part by part (SM_PART entries): an LDS histogram
// per part and global atomics give the coarse counts, a per-super-bin scan the
// coarse bases (super-bin base + local prefix -- no device-wide scan), and the
// scatter reserves one range per touched coarse bin (SM_PART / 2^G entries per
// run on average).
constexpr uint32_t SM_PART = 16384, SM_IPT = SM_PART / S_THREADS;

static __global__ void __launch_bounds__(1024) k_msm_sm_count(const uint64_t* __restrict__ tmp,
                                                              const uint32_t* __restrict__ sbase,
                                                              const uint32_t* __restrict__ spbase, uint32_t NS,
                                                              uint32_t F, uint32_t G, uint32_t* __restrict__ ccount) {
  __shared__ uint32_t hist[1024], sh[2];
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  if (j >= spbase[NS]) return;
  s2_locate(spbase, NS, j, sh);
  const uint32_t s = sh[0], p = sh[1];
  const uint32_t start = sbase[s], cnt = sbase[s + 1] - start;
  const uint32_t lo = p * SM_PART, hi = min(lo + SM_PART, cnt), ng = 1u << G;
  for (uint32_t q = t; q < ng; q += S_THREADS) hist[q] = 0;
  __syncthreads();
  for (uint32_t e = lo + t; e < hi; e += S_THREADS) lds_rank_add(hist, ((uint32_t)tmp[start + e] >> F) & (ng - 1));
  __syncthreads();
  for (uint32_t q = t; q < ng; q += S_THREADS)
    if (hist[q]) atomicAdd(&ccount[(s << G) + q], hist[q]);
}

// block s: coarse bases / cursors of super-bin s's 2^G coarse bins, and the
// number of final-pass parts of each (cparts; > 1 only above S2_BIG entries)
static __global__ void __launch_bounds__(1024) k_msm_sm_scan(const uint32_t* __restrict__ ccount,
                                                             const uint32_t* __restrict__ sbase, uint32_t G,
                                                             uint32_t NC, uint32_t* __restrict__ cbase,
                                                             uint32_t* __restrict__ ccursor,
                                                             uint32_t* __restrict__ cparts) {
  __shared__ uint32_t a[1024], wsum[17];
  const uint32_t s = blockIdx.x, t = threadIdx.x, H0 = s << G;
  const uint32_t nh = min(1u << G, NC - H0);
  for (uint32_t q = t; q < nh; q += S_THREADS) a[q] = ccount[H0 + q];
  block_excl_scan(a, nh, wsum);
  for (uint32_t q = t; q < nh; q += S_THREADS) {
    const uint32_t c = ccount[H0 + q];
    cbase[H0 + q] = sbase[s] + a[q];
    ccursor[H0 + q] = sbase[s] + a[q];
    cparts[H0 + q] = c > S2_BIG ? (c + S2_BIG - 1) / S2_BIG : 1u;
  }
  if (t == 0 && H0 + nh == NC) cbase[NC] = sbase[s + 1];
}

static __global__ void __launch_bounds__(1024) k_msm_sm_scatter(const uint64_t* __restrict__ tmp,
                                                                const uint32_t* __restrict__ sbase,
                                                                const uint32_t* __restrict__ spbase, uint32_t NS,
                                                                uint32_t F, uint32_t G,
                                                                uint32_t* __restrict__ ccursor,
                                                                uint64_t* __restrict__ tmp2) {
  __shared__ uint32_t hist[1024], cur[1024], sh[2];
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  if (j >= spbase[NS]) return;
  s2_locate(spbase, NS, j, sh);
  const uint32_t s = sh[0], p = sh[1];
  const uint32_t start = sbase[s], cnt = sbase[s + 1] - start;
  const uint32_t lo = p * SM_PART, hi = min(lo + SM_PART, cnt), ng = 1u << G;
  for (uint32_t q = t; q < ng; q += S_THREADS) hist[q] = 0;
  __syncthreads();
  uint64_t x[SM_IPT];
  uint32_t rk[SM_IPT];
#pragma unroll
  for (uint32_t it = 0; it < SM_IPT; it++) {
    const uint32_t e = lo + it * S_THREADS + t;
    if (e < hi) {
      x[it] = tmp[start + e];
      rk[it] = lds_rank_add(hist, ((uint32_t)x[it] >> F) & (ng - 1));
    }
  }
  __syncthreads();
  for (uint32_t q = t; q < ng; q += S_THREADS)
    if (hist[q]) cur[q] = atomicAdd(&ccursor[(s << G) + q], hist[q]);
  __syncthreads();
#pragma unroll
  for (uint32_t it = 0; it < SM_IPT; it++) {
    const uint32_t e = lo + it * S_THREADS + t;
    if (e < hi) tmp2[cur[((uint32_t)x[it] >> F) & (ng - 1)] + rk[it]] = x[it];
  }
}

// Device-wide exclusive scan of n u32 (out[n] = total): block scans of
// SCAN_BLK elements, one block over the block totals, then the fix-up.
constexpr uint32_t SCAN_BLK = 4096;
static __global__ void __launch_bounds__(1024) k_scan_local(const uint32_t* __restrict__ in, uint32_t n,
                                                            uint32_t* __restrict__ out, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t a[SCAN_BLK], wsum[17];
  const uint32_t base = blockIdx.x * SCAN_BLK, len = min(SCAN_BLK, n - base);
  for (uint32_t q = threadIdx.x; q < len; q += S_THREADS) a[q] = in[base + q];
  const uint32_t tot = block_excl_scan(a, len, wsum);
  for (uint32_t q = threadIdx.x; q < len; q += S_THREADS) out[base + q] = a[q];
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}
static __global__ void __launch_bounds__(1024) k_scan_tops(uint32_t* __restrict__ bsum, uint32_t nblk) {
  __shared__ uint32_t a[8192], wsum[17];
  for (uint32_t q = threadIdx.x; q < nblk; q += S_THREADS) a[q] = bsum[q];
  const uint32_t tot = block_excl_scan(a, nblk, wsum);
  for (uint32_t q = threadIdx.x; q < nblk; q += S_THREADS) bsum[q] = a[q];
  if (threadIdx.x == 0) bsum[nblk] = tot;
}
static __global__ void __launch_bounds__(1024) k_scan_add(uint32_t* __restrict__ out, uint32_t n,
                                                          const uint32_t* __restrict__ bsum, uint32_t nblk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += bsum[i / SCAN_BLK];
  if (i == 0) out[n] = bsum[nblk];
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

// The split-bin kernels below run on a capped grid, block-strided over the bins /
// parts: with no split bin (uniform digits) every block returns at once, where a
// block per bin cost ~0.2 ms per launch at 2^24 (213K empty blocks).
constexpr uint32_t S2_SPLIT_GRID = 2048;
static __global__ void __launch_bounds__(1024) k_msm_s2_scan(const uint32_t* __restrict__ cbase,
                                                             const uint32_t* __restrict__ pbase, uint32_t NC,
                                                             uint32_t F, uint32_t T, uint32_t* __restrict__ fcount,
                                                             uint32_t* __restrict__ offsets) {
  extern __shared__ uint32_t hist[];
  __shared__ uint32_t wsum[17];
  if (pbase[NC] == NC) return;  // no split bins
  const uint32_t t = threadIdx.x;
  for (uint32_t H = blockIdx.x; H < NC; H += gridDim.x) {
    const uint32_t start = cbase[H], cnt = cbase[H + 1] - start;
    if (cnt <= S2_BIG) continue;
    const uint32_t b0 = H << F, nf = min(1u << F, T - b0);
    for (uint32_t f = t; f < nf; f += S_THREADS) hist[f] = fcount[b0 + f];
    block_excl_scan(hist, nf, wsum);
    for (uint32_t f = t; f < nf; f += S_THREADS) {
      offsets[b0 + f] = start + hist[f];
      fcount[b0 + f] = start + hist[f];  // now the bucket's write cursor
    }
    __syncthreads();
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
  const uint32_t t = threadIdx.x, parts = pbase[NC];
  if (parts == NC) return;  // no split bins: nothing to do
  for (uint32_t j = blockIdx.x; j < parts; j += gridDim.x) {
    s2_locate(pbase, NC, j, sh);
    const uint32_t H = sh[0], p = sh[1];
    const uint32_t start = cbase[H], cnt = cbase[H + 1] - start;
    __syncthreads();  // every thread has read sh before the next part's s2_locate
    if (cnt <= S2_BIG) continue;
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
    __syncthreads();  // the LDS is reused by the next part
  }
}

int msm_sort_digits(gm_ctx* ctx, Arena& arena, const SortGeom& g, size_t n, uint32_t W, uint32_t nb,
                    uint32_t shared_stride, const uint32_t* dig, const uint32_t* scount, uint32_t* keys_out,
                    uint32_t* vals_out, uint32_t* offsets) {
  if (g.NS == 0 || g.NS > 8192 || g.F > 13 || g.G > 10 || g.NC != (g.T + (1u << g.F) - 1) >> g.F ||
      g.NS != (g.T + (1u << (g.F + g.G)) - 1) >> (g.F + g.G)) {
    set_error("msm sort: bad geometry");
    return GM_ERR_INVALID;
  }
  hipStream_t st = ctx->stream;
  const uint32_t shift = g.F + g.G;  // pass-1 bin = b >> shift (super-bin, or coarse bin when G = 0)
  int rc;
  DevBuf sbase, scursor, spbase, tmp;
  if ((rc = sbase.alloc(arena, 4 * ((size_t)g.NS + 1))) || (rc = scursor.alloc(arena, 4 * (size_t)g.NS)) ||
      (rc = spbase.alloc(arena, 4 * ((size_t)g.NS + 1))) || (rc = tmp.alloc(arena, 8 * g.M)))
    return rc;
  hipLaunchKernelGGL(k_msm_s1_scan, dim3(1), dim3(S_THREADS), 0, st, scount, g.NS, g.T, g.G ? SM_PART : S2_BIG,
                     sbase.as<uint32_t>(), scursor.as<uint32_t>(), spbase.as<uint32_t>(), offsets);
  // bins one pass-1 block touches: its window's own nb >> shift in the plain layout
  const uint32_t nh = (!shared_stride && (1u << shift) <= nb) ? nb >> shift : g.NS;
  // staged (coalesced-write) pass 1 while its LDS fits: 64 KB of entries plus
  // three words per touched bin (up to ~112 KB at 4,096 bins: gfx950 has 160 KB
  // per workgroup; a device with less takes the direct scatter)
  const size_t lds = 8 * (size_t)S1_PTS + sizeof(uint32_t) * (3 * (size_t)nh + 17);
  if (nh <= 4096 && lds <= device_lds_per_block(ctx->device)) {
    hipLaunchKernelGGL(k_msm_s1_scatter_st<S1_PPT>, dim3(blocks_for(n, S1_PTS), W), dim3(S_THREADS), lds, st, dig,
                       (uint32_t)n, nb, shared_stride, shift, g.NS, nh, scursor.as<uint32_t>(), tmp.as<uint64_t>());
    GM_HIP(hipGetLastError());
  } else {
    hipLaunchKernelGGL(k_msm_s1_scatter, dim3(blocks_for(n, S1_PTS), W), dim3(S_THREADS), 2 * sizeof(uint32_t) * nh,
                       st, dig, (uint32_t)n, nb, shared_stride, shift, g.NS, nh, scursor.as<uint32_t>(),
                       tmp.as<uint64_t>());
  }
  // final pass input: coarse-binned entries with their bases / part table
  const uint64_t* fin = tmp.as<uint64_t>();
  const uint32_t *cbase = sbase.as<uint32_t>(), *pbase = spbase.as<uint32_t>();
  if (g.G) {
    DevBuf ccount, cb, ccur, cparts, pb, bsum, tmp2;
    const uint32_t nblk = (g.NC + SCAN_BLK - 1) / SCAN_BLK;
    if ((rc = ccount.alloc(arena, 4 * (size_t)g.NC)) || (rc = cb.alloc(arena, 4 * ((size_t)g.NC + 1))) ||
        (rc = ccur.alloc(arena, 4 * (size_t)g.NC)) || (rc = cparts.alloc(arena, 4 * (size_t)g.NC)) ||
        (rc = pb.alloc(arena, 4 * ((size_t)g.NC + 1))) || (rc = bsum.alloc(arena, 4 * ((size_t)nblk + 1))) ||
        (rc = tmp2.alloc(arena, 8 * g.M)))
      return rc;
    if (nblk > 8192) {
      set_error("msm sort: too many coarse bins");
      return GM_ERR_INVALID;
    }
    const size_t mparts = (size_t)g.NS + g.M / SM_PART + 1;
    GM_HIP(hipMemsetAsync(ccount.p, 0, 4 * (size_t)g.NC, st));
    hipLaunchKernelGGL(k_msm_sm_count, dim3((unsigned)mparts), dim3(S_THREADS), 0, st, tmp.as<uint64_t>(),
                       sbase.as<uint32_t>(), spbase.as<uint32_t>(), g.NS, g.F, g.G, ccount.as<uint32_t>());
    hipLaunchKernelGGL(k_msm_sm_scan, dim3(g.NS), dim3(S_THREADS), 0, st, ccount.as<uint32_t>(), sbase.as<uint32_t>(),
                       g.G, g.NC, cb.as<uint32_t>(), ccur.as<uint32_t>(), cparts.as<uint32_t>());
    hipLaunchKernelGGL(k_scan_local, dim3(nblk), dim3(S_THREADS), 0, st, cparts.as<uint32_t>(), g.NC,
                       pb.as<uint32_t>(), bsum.as<uint32_t>());
    hipLaunchKernelGGL(k_scan_tops, dim3(1), dim3(S_THREADS), 0, st, bsum.as<uint32_t>(), nblk);
    hipLaunchKernelGGL(k_scan_add, dim3(blocks_for(g.NC, 256)), dim3(256), 0, st, pb.as<uint32_t>(), g.NC,
                       bsum.as<uint32_t>(), nblk);
    hipLaunchKernelGGL(k_msm_sm_scatter, dim3((unsigned)mparts), dim3(S_THREADS), 0, st, tmp.as<uint64_t>(),
                       sbase.as<uint32_t>(), spbase.as<uint32_t>(), g.NS, g.F, g.G, ccur.as<uint32_t>(),
                       tmp2.as<uint64_t>());
    fin = tmp2.as<uint64_t>();
    cbase = cb.as<uint32_t>();
    pbase = pb.as<uint32_t>();
  }
  DevBuf fcount;
  if ((rc = fcount.alloc(arena, 4 * (size_t)g.T))) return rc;
  const uint32_t nfmax = std::min<uint32_t>(1u << g.F, g.T);
  // every coarse bin has >= 1 part; split bins add at most M / S2_BIG more
  const size_t maxparts = (size_t)g.NC + g.M / S2_BIG + 1;
  GM_HIP(hipMemsetAsync(fcount.p, 0, sizeof(uint32_t) * g.T, st));
  hipLaunchKernelGGL(k_msm_s2_local, dim3((unsigned)maxparts), dim3(S_THREADS),
                     sizeof(uint32_t) * (nfmax + 2 * S2_STAGE), st, fin, cbase, pbase, g.NC, g.F, g.T,
                     fcount.as<uint32_t>(), keys_out, vals_out, offsets);
  hipLaunchKernelGGL(k_msm_s2_scan, dim3(std::min<uint32_t>(g.NC, S2_SPLIT_GRID)), dim3(S_THREADS),
                     sizeof(uint32_t) * nfmax, st, cbase, pbase, g.NC, g.F, g.T, fcount.as<uint32_t>(), offsets);
  hipLaunchKernelGGL(k_msm_s2_scatter, dim3((unsigned)std::min<size_t>(maxparts, S2_SPLIT_GRID)), dim3(S_THREADS),
                     2 * sizeof(uint32_t) * nfmax, st, fin, cbase, pbase, g.NC, g.F, g.T, fcount.as<uint32_t>(),
                     keys_out, vals_out);
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
  best.narrow = precomp_narrow(best.c, best.W, bits);
  return best;
}

}  // namespace gm
