// Pippenger bucket MSM on gfx950 -- replaces iciclegnark MsmOnDevice /
// MsmG2OnDevice (backend/groth16/bn254/icicle/icicle.go:302,315,332,355,382).
//
// Pipeline (one HIP stream, all state in HBM):
//   1. k_msm_hist     Montgomery -> canonical scalar, signed c-bit digits for all
//                     W windows, histogram of (window, |digit|) buckets.
//   2. exclusive scan of the histogram (hipcub) -> bucket offsets.
//   3. k_msm_scatter  recompute digits, counting-sort scatter of
//                     (point index | sign<<31) into bucket order.
//   4. k_msm_accum    one thread per bucket: XYZZ accumulation of its points
//                     (mixed adds, gathered affine points, sign applied on load).
//   5. k_msm_seg      bucket reduction sum_b b*B_b, per segment of L buckets:
//                     running sums (T_s, S_s).
//   6. k_msm_segmul   R_s = T_s + (s*L) * S_s.
//   7. k_msm_winsum   per-window tree reduction of R_s in LDS.
//   8. host: Horner over windows sum_w 2^(c w) W_w (W tiny), XYZZ -> Jacobian.
//
// Exact group arithmetic: the result is independent of summation order, so the
// atomics-based counting sort needs no determinism.
#include <hipcub/hipcub.hpp>

#include "curves.hpp"
#include "msm.hpp"
#include "runtime.hpp"

namespace gm {

// ---------------------------------------------------------------------------
// scalar digits
// ---------------------------------------------------------------------------
template <class Fr>
GM_DEV uint32_t window_bits(const FeG<Fr>& k, uint32_t bit, uint32_t mask) {
  const uint32_t idx = bit >> 5, sh = bit & 31;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < Fr::NG; i++) {
    lo = (idx == (uint32_t)i) ? k.w[i] : lo;
    hi = (idx + 1 == (uint32_t)i) ? k.w[i] : hi;
  }
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  return (uint32_t)(v >> sh) & mask;
}

// gnark Montgomery fr.Element -> canonical integer as packed u32 words
template <class Fr>
GM_DEV FeG<Fr> load_scalar_canonical(const uint32_t* __restrict__ s, uint32_t i) {
  return fe_pack(fe_gnark_to_canonical(fe_load_g<Fr>(s, i)));
}

// Signed digit recoding: raw = bits + carry; raw > 2^(c-1) -> digit raw - 2^c.
// Digits lie in [-(2^(c-1) - 1), 2^(c-1)]; bucket index = |digit| - 1.
template <class Fr>
__global__ void __launch_bounds__(256) k_msm_hist(const uint32_t* __restrict__ scalars, uint32_t n,
                                                  uint32_t c, uint32_t W,
                                                  uint32_t* __restrict__ counts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const FeG<Fr> k = load_scalar_canonical<Fr>(scalars, i);
  const uint32_t nb = 1u << (c - 1), mask = (1u << c) - 1;
  uint32_t carry = 0;
  for (uint32_t w = 0; w < W; w++) {
    uint32_t raw = window_bits(k, w * c, mask) + carry;
    uint32_t d;
    if (raw > nb) {
      d = (1u << c) - raw;
      carry = 1;
    } else {
      d = raw;
      carry = 0;
    }
    if (d) atomicAdd(&counts[w * nb + d - 1], 1u);
  }
}

template <class Fr>
__global__ void __launch_bounds__(256) k_msm_scatter(const uint32_t* __restrict__ scalars,
                                                     uint32_t n, uint32_t c, uint32_t W,
                                                     uint32_t* __restrict__ cursor,
                                                     const uint32_t* __restrict__ bucket_end,
                                                     uint32_t* __restrict__ sorted,
                                                     uint32_t* __restrict__ err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const FeG<Fr> k = load_scalar_canonical<Fr>(scalars, i);
  const uint32_t nb = 1u << (c - 1), mask = (1u << c) - 1;
  uint32_t carry = 0;
  for (uint32_t w = 0; w < W; w++) {
    uint32_t raw = window_bits(k, w * c, mask) + carry;
    uint32_t d, neg;
    if (raw > nb) {
      d = (1u << c) - raw;
      carry = 1;
      neg = 1;
    } else {
      d = raw;
      carry = 0;
      neg = 0;
    }
    if (d) {
      const uint32_t b = w * nb + d - 1;
      const uint32_t pos = atomicAdd(&cursor[b], 1u);
      if (pos < bucket_end[b])
        sorted[pos] = i | (neg << 31);
      else
        atomicOr(err, 1u);  // histogram / scatter disagreement: never write out of range
    }
  }
}

// Digit keys for a radix sort: key = global bucket index w*nb + |d|-1 (or the
// sentinel `total` for a zero digit, which sorts past every bucket), value =
// point index | sign << 31.  Window-major: entry (w, i) at w*n + i.
template <class Fr>
__global__ void __launch_bounds__(256) k_msm_keys(const uint32_t* __restrict__ scalars, uint32_t n,
                                                  uint32_t c, uint32_t W, uint32_t* __restrict__ keys,
                                                  uint32_t* __restrict__ vals) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const FeG<Fr> k = load_scalar_canonical<Fr>(scalars, i);
  const uint32_t nb = 1u << (c - 1), mask = (1u << c) - 1, total = W * nb;
  uint32_t carry = 0;
  for (uint32_t w = 0; w < W; w++) {
    const uint32_t raw = window_bits(k, w * c, mask) + carry;
    uint32_t d, neg;
    if (raw > nb) {
      d = (1u << c) - raw;
      carry = 1;
      neg = 1;
    } else {
      d = raw;
      carry = 0;
      neg = 0;
    }
    const size_t e = (size_t)w * n + i;
    keys[e] = d ? w * nb + d - 1 : total;
    vals[e] = i | (neg << 31);
  }
}

// offsets[b] = first sorted position with key >= b, for b in [0, total].
__global__ void __launch_bounds__(256) k_msm_offsets(const uint32_t* __restrict__ keys, size_t M,
                                                     uint32_t total, uint32_t* __restrict__ offsets) {
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= M) return;
  const uint32_t k = keys[q];
  const uint32_t kp = q ? keys[q - 1] : 0xffffffffu;  // -1
  if (k != kp) {
    const uint32_t lo = kp == 0xffffffffu ? 0 : kp + 1;
    const uint32_t hi = k < total ? k : total;
    for (uint32_t b = lo; b <= hi; b++) offsets[b] = (uint32_t)q;
  }
  if (q == M - 1 && k < total)
    for (uint32_t b = k + 1; b <= total; b++) offsets[b] = (uint32_t)M;
}

// ---------------------------------------------------------------------------
// points: gnark layout -> internal layout (once per MSM, into workspace)
// ---------------------------------------------------------------------------
template <class F>
__global__ void __launch_bounds__(256) k_msm_convert_points(const uint32_t* __restrict__ src, size_t n,
                                                            Affine<F>* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dst[i] = load_affine_gnark<F>(src + i * 2 * Coord<F>::WORDS);
}

template <class F>
__global__ void __launch_bounds__(128) k_msm_accum(const Affine<F>* __restrict__ points,
                                                   uint32_t n,
                                                   const uint32_t* __restrict__ sorted,
                                                   const uint32_t* __restrict__ offsets,
                                                   uint32_t total_buckets,
                                                   XYZZ<F>* __restrict__ buckets,
                                                   uint32_t* __restrict__ err) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= total_buckets) return;
  const uint32_t s = offsets[b], e = offsets[b + 1];
  XYZZ<F> acc = xyzz_inf<F>();
  for (uint32_t q = s; q < e; q++) {
    const uint32_t v = sorted[q];
    const uint32_t idx = v & 0x7fffffffu;
    if (idx >= n) {
      atomicOr(err, 2u);
      continue;
    }
    Affine<F> P = points[idx];
    if (v >> 31) P.y = fe_neg(P.y);
    xyzz_add_aff(acc, P);
  }
  buckets[b] = acc;
}

// Load-balanced accumulation over the sorted entry list: thread t owns entries
// [t*K, t*K+K).  A bucket whose whole range lies in the thread's slice is
// written straight to `buckets`; the (at most two) buckets cut by the slice
// edges go to part_first[t] / part_last[t] and are merged by k_msm_fixup.
// Skewed scalar distributions (one huge bucket) therefore cost the same as
// uniform ones in this phase.
template <class F>
GM_DEV void accum_emit(uint32_t b, const XYZZ<F>& acc, bool is_first, bool is_last, uint32_t start,
                       uint32_t end, uint32_t t, const uint32_t* __restrict__ offsets,
                       XYZZ<F>* __restrict__ buckets, XYZZ<F>* __restrict__ part_first,
                       XYZZ<F>* __restrict__ part_last) {
  const uint32_t bs = offsets[b], be = offsets[b + 1];
  if (bs >= start && be <= end) {
    buckets[b] = acc;
  } else {
    if (is_first) part_first[t] = acc;
    if (is_last) part_last[t] = acc;
  }
}

template <class F>
__global__ void __launch_bounds__(128) k_msm_accum_seg(const Affine<F>* __restrict__ points, uint32_t n,
                                                       const uint32_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ vals,
                                                       const uint32_t* __restrict__ offsets, uint32_t total,
                                                       uint32_t K, XYZZ<F>* __restrict__ buckets,
                                                       XYZZ<F>* __restrict__ part_first,
                                                       XYZZ<F>* __restrict__ part_last,
                                                       uint32_t* __restrict__ err) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t Mv = offsets[total];  // valid (non-zero-digit) entries
  const uint32_t start = t * K;
  if (start >= Mv) return;
  const uint32_t end = min(start + K, Mv);
  uint32_t cur = keys[start];
  bool first = true;
  XYZZ<F> acc = xyzz_inf<F>();
  uint32_t v = vals[start];
  uint32_t idx = v & 0x7fffffffu;
  if (idx >= n) {
    atomicOr(err, 2u);
    return;
  }
  Affine<F> P = points[idx];
  for (uint32_t q = start; q < end; q++) {
    const uint32_t k = keys[q];
    // prefetch the next point while this add runs
    uint32_t vn = 0;
    Affine<F> Pn;
    if (q + 1 < end) {
      vn = vals[q + 1];
      const uint32_t in = vn & 0x7fffffffu;
      if (in >= n) {
        atomicOr(err, 2u);
        return;
      }
      Pn = points[in];
    }
    if (k != cur) {
      accum_emit(cur, acc, first, false, start, end, t, offsets, buckets, part_first, part_last);
      first = false;
      acc = xyzz_inf<F>();
      cur = k;
    }
    if (v >> 31) P.y = fe_neg(P.y);
    xyzz_add_aff(acc, P);
    v = vn;
    P = Pn;
  }
  accum_emit(cur, acc, first, true, start, end, t, offsets, buckets, part_first, part_last);
}

// Merge the partial sums of buckets cut by slice edges (bucket b spans slices t0..t1).
template <class F>
__global__ void __launch_bounds__(128) k_msm_fixup(const uint32_t* __restrict__ offsets, uint32_t total,
                                                   uint32_t K, XYZZ<F>* __restrict__ buckets,
                                                   const XYZZ<F>* __restrict__ part_first,
                                                   const XYZZ<F>* __restrict__ part_last) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= total) return;
  const uint32_t bs = offsets[b], be = offsets[b + 1];
  if (be == bs) return;
  const uint32_t t0 = bs / K, t1 = (be - 1) / K;
  if (t0 == t1) return;
  XYZZ<F> acc = part_last[t0];
  for (uint32_t t = t0 + 1; t < t1; t++) acc = xyzz_add(acc, part_first[t]);
  acc = xyzz_add(acc, part_first[t1]);
  buckets[b] = acc;
}

// Segment running sums.  Segment s of window w covers bucket array indices
// j in [s*L, s*L + L) (bucket weight j+1):
//   S_s = sum_j B_j,   T_s = sum_j (j - s*L + 1) B_j
template <class F>
__global__ void __launch_bounds__(128) k_msm_seg(const XYZZ<F>* __restrict__ buckets,
                                                 uint32_t nb, uint32_t L, uint32_t nseg,
                                                 uint32_t W, XYZZ<F>* __restrict__ segT,
                                                 XYZZ<F>* __restrict__ segS) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= W * nseg) return;
  const uint32_t w = t / nseg, s = t % nseg;
  const XYZZ<F>* B = buckets + (size_t)w * nb + (size_t)s * L;
  XYZZ<F> S = xyzz_inf<F>(), T = xyzz_inf<F>();
  for (int j = (int)L - 1; j >= 0; j--) {
    S = xyzz_add(S, B[j]);
    T = xyzz_add(T, S);
  }
  segT[t] = T;
  segS[t] = S;
}

// R_s = T_s + (s*L) * S_s
template <class F>
__global__ void __launch_bounds__(128) k_msm_segmul(XYZZ<F>* __restrict__ segT,
                                                    const XYZZ<F>* __restrict__ segS, uint32_t L,
                                                    uint32_t nseg, uint32_t W) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= W * nseg) return;
  const uint32_t s = t % nseg;
  XYZZ<F> m = xyzz_mul_small(segS[t], s * L);
  segT[t] = xyzz_add(segT[t], m);
}

// Per-window reduction of nseg R_s values: block per window.
template <class F, int TPB>
__global__ void __launch_bounds__(TPB) k_msm_winsum(const XYZZ<F>* __restrict__ R, uint32_t nseg,
                                                    uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  XYZZ<F>* sm = reinterpret_cast<XYZZ<F>*>(smem_raw);
  const uint32_t w = blockIdx.x;
  XYZZ<F> acc = xyzz_inf<F>();
  for (uint32_t s = threadIdx.x; s < nseg; s += TPB) acc = xyzz_add(acc, R[(size_t)w * nseg + s]);
  sm[threadIdx.x] = acc;
  __syncthreads();
  for (int half = TPB / 2; half > 0; half >>= 1) {
    if ((int)threadIdx.x < half) sm[threadIdx.x] = xyzz_add(sm[threadIdx.x], sm[threadIdx.x + half]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    // window sum in gnark layout (X, Y, ZZ, ZZZ) for the host finish
    uint32_t* o = out + (size_t)w * 4 * Coord<F>::WORDS;
    const XYZZ<F> r = sm[0];
    Coord<F>::store_gnark(o, r.x);
    Coord<F>::store_gnark(o + Coord<F>::WORDS, r.y);
    Coord<F>::store_gnark(o + 2 * Coord<F>::WORDS, r.zz);
    Coord<F>::store_gnark(o + 3 * Coord<F>::WORDS, r.zzz);
  }
}

// ---------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------
static int choose_window(size_t n) {
  int lg = 0;
  while ((size_t(1) << (lg + 1)) <= n) lg++;
  int c = lg - 4;
  if (c < 8) c = 8;
  if (c > 20) c = 20;
  return c;
}

template <class C, bool G2>
int msm_device(gm_ctx* ctx, const void* scalars_dev, const void* points_dev, size_t n,
               typename GroupSel<C, G2>::HF (&jac_out)[3], bool points_internal) {
  using DF = typename GroupSel<C, G2>::DF;
  using HF = typename GroupSel<C, G2>::HF;
  using HJ = host::Jac<HF>;
  hipStream_t st = ctx->stream;
  if (n == 0) {
    HJ inf = HJ::inf();
    jac_out[0] = inf.x;
    jac_out[1] = inf.y;
    jac_out[2] = inf.z;
    return GM_OK;
  }
  if (n >= (size_t(1) << 31)) {
    set_error("msm: n must be < 2^31");
    return GM_ERR_INVALID;
  }
  const uint32_t c = ctx->msm_c_override ? (uint32_t)ctx->msm_c_override : (uint32_t)choose_window(n);
  const uint32_t W = (C::FR_BITS + 1 + c - 1) / c;  // ceil((bits+1)/c): top signed digit never carries
  const uint32_t nb = 1u << (c - 1);
  const uint32_t total = W * nb;
  const uint32_t L = nb >= 64 ? 8 : 1;
  const uint32_t nseg = nb / L;
  int rc;

  Arena arena(ctx);
  constexpr int WORDS = Coord<DF>::WORDS;  // u32 words of one gnark-layout coordinate
  DevBuf counts, offsets, sorted, buckets, segT, segS, wsum, scan_tmp, errw, ipts, keys_in, keys_out;
  if ((rc = errw.alloc(arena, 16))) return rc;
  GM_HIP(hipMemsetAsync(errw.p, 0, 16, st));
  // counts doubles as the unsorted value array of the radix sort
  if ((rc = counts.alloc(arena, sizeof(uint32_t) * (size_t)W * n))) return rc;
  if ((rc = keys_in.alloc(arena, sizeof(uint32_t) * (size_t)W * n))) return rc;
  if ((rc = keys_out.alloc(arena, sizeof(uint32_t) * (size_t)W * n))) return rc;
  if ((rc = offsets.alloc(arena, sizeof(uint32_t) * (total + 1)))) return rc;
  if ((rc = sorted.alloc(arena, sizeof(uint32_t) * (size_t)W * n))) return rc;
  if ((rc = buckets.alloc(arena, sizeof(XYZZ<DF>) * (size_t)total))) return rc;
  if ((rc = segT.alloc(arena, sizeof(XYZZ<DF>) * (size_t)W * nseg))) return rc;
  if ((rc = segS.alloc(arena, sizeof(XYZZ<DF>) * (size_t)W * nseg))) return rc;
  if ((rc = wsum.alloc(arena, sizeof(uint32_t) * 4 * WORDS * W))) return rc;
  const Affine<DF>* pts_internal = reinterpret_cast<const Affine<DF>*>(points_dev);
  if (!points_internal) {
    if ((rc = ipts.alloc(arena, sizeof(Affine<DF>) * n))) return rc;
    ProfScope ps(ctx, "msm_convert_points");
    hipLaunchKernelGGL(k_msm_convert_points<DF>, dim3(blocks_for(n, 256)), dim3(256), 0, st,
                       reinterpret_cast<const uint32_t*>(points_dev), n, ipts.as<Affine<DF>>());
    pts_internal = ipts.as<Affine<DF>>();
  }

  const uint32_t* sc = reinterpret_cast<const uint32_t*>(scalars_dev);
  const size_t M = (size_t)W * n;
  if (M >= (size_t(1) << 31)) {
    set_error("msm: n * windows must be < 2^31");
    return GM_ERR_INVALID;
  }
  {
    ProfScope ps(ctx, "msm_keys");
    hipLaunchKernelGGL(k_msm_keys<typename C::Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, st, sc,
                       (uint32_t)n, c, W, keys_in.as<uint32_t>(), counts.as<uint32_t>());
  }
  GM_HIP(hipGetLastError());
  int end_bit = 1;
  while ((1ull << end_bit) <= total) end_bit++;
  size_t tmp_bytes = 0;
  GM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys_in.as<uint32_t>(), keys_out.as<uint32_t>(),
                                            counts.as<uint32_t>(), sorted.as<uint32_t>(), (int)M, 0, end_bit, st));
  if ((rc = scan_tmp.alloc(arena, tmp_bytes))) return rc;
  {
    ProfScope ps(ctx, "msm_sort");
    GM_HIP(hipcub::DeviceRadixSort::SortPairs(scan_tmp.p, tmp_bytes, keys_in.as<uint32_t>(),
                                              keys_out.as<uint32_t>(), counts.as<uint32_t>(),
                                              sorted.as<uint32_t>(), (int)M, 0, end_bit, st));
  }
  {
    ProfScope ps(ctx, "msm_offsets");
    hipLaunchKernelGGL(k_msm_offsets, dim3(blocks_for(M, 256)), dim3(256), 0, st, keys_out.as<uint32_t>(), M,
                       total, offsets.as<uint32_t>());
  }
  GM_HIP(hipGetLastError());
  {
    const uint32_t K = ctx->msm_slice ? (uint32_t)ctx->msm_slice : 64u;
    const size_t nslices = (M + K - 1) / K;
    DevBuf pfirst, plast;
    if ((rc = pfirst.alloc(arena, sizeof(XYZZ<DF>) * nslices))) return rc;
    if ((rc = plast.alloc(arena, sizeof(XYZZ<DF>) * nslices))) return rc;
    GM_HIP(hipMemsetAsync(buckets.p, 0, sizeof(XYZZ<DF>) * (size_t)total, st));  // all-zero XYZZ = infinity
    ProfScope ps(ctx, G2 ? "msm_accum_g2" : "msm_accum_g1");
    hipLaunchKernelGGL(k_msm_accum_seg<DF>, dim3(blocks_for(nslices, 128)), dim3(128), 0, st, pts_internal,
                       (uint32_t)n, keys_out.as<uint32_t>(), sorted.as<uint32_t>(), offsets.as<uint32_t>(), total,
                       K, buckets.as<XYZZ<DF>>(), pfirst.as<XYZZ<DF>>(), plast.as<XYZZ<DF>>(),
                       errw.as<uint32_t>());
    hipLaunchKernelGGL(k_msm_fixup<DF>, dim3(blocks_for(total, 128)), dim3(128), 0, st, offsets.as<uint32_t>(),
                       total, K, buckets.as<XYZZ<DF>>(), pfirst.as<XYZZ<DF>>(), plast.as<XYZZ<DF>>());
  }
  {
    ProfScope ps(ctx, "msm_bucket_reduce");
    hipLaunchKernelGGL(k_msm_seg<DF>, dim3(blocks_for((size_t)W * nseg, 128)), dim3(128), 0, st,
                       buckets.as<XYZZ<DF>>(), nb, L, nseg, W, segT.as<XYZZ<DF>>(), segS.as<XYZZ<DF>>());
    hipLaunchKernelGGL(k_msm_segmul<DF>, dim3(blocks_for((size_t)W * nseg, 128)), dim3(128), 0, st,
                       segT.as<XYZZ<DF>>(), segS.as<XYZZ<DF>>(), L, nseg, W);
    constexpr int TPB = 128;
    hipLaunchKernelGGL((k_msm_winsum<DF, TPB>), dim3(W), dim3(TPB), sizeof(XYZZ<DF>) * TPB, st,
                       segT.as<XYZZ<DF>>(), nseg, wsum.as<uint32_t>());
  }
  GM_HIP(hipGetLastError());
  uint32_t herr = 0;
  GM_HIP(hipMemcpyAsync(&herr, errw.p, 4, hipMemcpyDeviceToHost, st));
  std::vector<HF> hw(4 * W);
  static_assert(sizeof(HF) == 4 * WORDS, "host/device layout mismatch");
  GM_HIP(hipMemcpyAsync(hw.data(), wsum.p, sizeof(uint32_t) * 4 * WORDS * W, hipMemcpyDeviceToHost, st));
  GM_HIP(hipStreamSynchronize(st));
  if (herr) {
    set_error("msm: internal consistency check failed (code " + std::to_string(herr) + ")");
    return GM_ERR_DEVICE;
  }
  // Horner over windows
  HJ acc = HJ::inf();
  for (int w = (int)W - 1; w >= 0; w--) {
    if (!acc.is_inf())
      for (uint32_t i = 0; i < c; i++) acc = host::jdbl(acc);
    HJ ww = host::xyzz_to_jac(hw[4 * w + 0], hw[4 * w + 1], hw[4 * w + 2], hw[4 * w + 3]);
    acc = host::jadd(acc, ww);
  }
  jac_out[0] = acc.x;
  jac_out[1] = acc.y;
  jac_out[2] = acc.z;
  return GM_OK;
}

template <class C, bool G2>
size_t msm_internal_point_bytes() {
  return sizeof(Affine<typename GroupSel<C, G2>::DF>);
}

template <class C, bool G2>
int msm_prepare_points(gm_ctx* ctx, const void* gnark_points, size_t n, void* dst) {
  using DF = typename GroupSel<C, G2>::DF;
  if (n == 0) return GM_OK;
  hipLaunchKernelGGL(k_msm_convert_points<DF>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                     reinterpret_cast<const uint32_t*>(gnark_points), n, reinterpret_cast<Affine<DF>*>(dst));
  GM_HIP(hipGetLastError());
  return GM_OK;
}

#define GM_MSM_PREP_INST(C, G2)                                                   \
  template size_t msm_internal_point_bytes<C, G2>();                             \
  template int msm_prepare_points<C, G2>(gm_ctx*, const void*, size_t, void*);
GM_MSM_PREP_INST(CurveBN254, false)
GM_MSM_PREP_INST(CurveBN254, true)
GM_MSM_PREP_INST(CurveBLS12377, false)
GM_MSM_PREP_INST(CurveBLS12377, true)

template int msm_device<CurveBN254, false>(gm_ctx*, const void*, const void*, size_t,
                                          CurveBN254::HG1F (&)[3], bool);
template int msm_device<CurveBN254, true>(gm_ctx*, const void*, const void*, size_t,
                                          CurveBN254::HG2F (&)[3], bool);
template int msm_device<CurveBLS12377, false>(gm_ctx*, const void*, const void*, size_t,
                                          CurveBLS12377::HG1F (&)[3], bool);
template int msm_device<CurveBLS12377, true>(gm_ctx*, const void*, const void*, size_t,
                                          CurveBLS12377::HG2F (&)[3], bool);

}  // namespace gm
