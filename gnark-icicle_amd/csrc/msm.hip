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
#include <cstdlib>

#include "curves.hpp"
#include "msm.hpp"
#include "runtime.hpp"

namespace gm {

// ---------------------------------------------------------------------------
// scalar digits
// ---------------------------------------------------------------------------
template <class Fr>
GM_DEV uint32_t window_bits(const Fe<Fr>& k, uint32_t bit, uint32_t mask) {
  const uint32_t idx = bit >> 5, sh = bit & 31;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < Fr::N; i++) {
    lo = (idx == (uint32_t)i) ? k.v[i] : lo;
    hi = (idx + 1 == (uint32_t)i) ? k.v[i] : hi;
  }
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  return (uint32_t)(v >> sh) & mask;
}

template <class Fr>
GM_DEV Fe<Fr> load_scalar_canonical(const uint32_t* __restrict__ s, uint32_t i) {
  Fe<Fr> k;
  const uint4* p = reinterpret_cast<const uint4*>(s + (size_t)i * Fr::N);
#pragma unroll
  for (int q = 0; q < Fr::N / 4; q++) {
    uint4 v = p[q];
    k.v[4 * q + 0] = v.x;
    k.v[4 * q + 1] = v.y;
    k.v[4 * q + 2] = v.z;
    k.v[4 * q + 3] = v.w;
  }
  return fe_from_mont(k);
}

// Signed digit recoding: raw = bits + carry; raw > 2^(c-1) -> digit raw - 2^c.
// Digits lie in [-(2^(c-1) - 1), 2^(c-1)]; bucket index = |digit| - 1.
template <class Fr>
__global__ void __launch_bounds__(256) k_msm_hist(const uint32_t* __restrict__ scalars, uint32_t n,
                                                  uint32_t c, uint32_t W,
                                                  uint32_t* __restrict__ counts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<Fr> k = load_scalar_canonical<Fr>(scalars, i);
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
  const Fe<Fr> k = load_scalar_canonical<Fr>(scalars, i);
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

// ---------------------------------------------------------------------------
// point loads (gnark affine layout, 16-byte vector loads)
// ---------------------------------------------------------------------------
template <class F>
GM_DEV Affine<F> load_affine(const Affine<F>* __restrict__ pts, uint32_t idx) {
  static_assert(sizeof(Affine<F>) % 16 == 0, "affine point must be 16B multiple");
  constexpr int Q = sizeof(Affine<F>) / 16;
  const uint4* src = reinterpret_cast<const uint4*>(pts + idx);
  Affine<F> r;
  uint4* dst = reinterpret_cast<uint4*>(&r);
#pragma unroll
  for (int q = 0; q < Q; q++) dst[q] = src[q];
  return r;
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
    Affine<F> P = load_affine(points, idx);
    if (v >> 31) P.y = fe_neg(P.y);
    xyzz_add_aff(acc, P);
  }
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
                                                    XYZZ<F>* __restrict__ out) {
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
  if (threadIdx.x == 0) out[w] = sm[0];
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
               typename GroupSel<C, G2>::HF (&jac_out)[3]) {
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
  DevBuf counts, offsets, sorted, buckets, segT, segS, wsum, scan_tmp, errw;
  if ((rc = errw.alloc(arena, 16))) return rc;
  GM_HIP(hipMemsetAsync(errw.p, 0, 16, st));
  if ((rc = counts.alloc(arena, sizeof(uint32_t) * (total + 1)))) return rc;
  if ((rc = offsets.alloc(arena, sizeof(uint32_t) * (total + 1)))) return rc;
  if ((rc = sorted.alloc(arena, sizeof(uint32_t) * (size_t)W * n))) return rc;
  if ((rc = buckets.alloc(arena, sizeof(XYZZ<DF>) * (size_t)total))) return rc;
  if ((rc = segT.alloc(arena, sizeof(XYZZ<DF>) * (size_t)W * nseg))) return rc;
  if ((rc = segS.alloc(arena, sizeof(XYZZ<DF>) * (size_t)W * nseg))) return rc;
  if ((rc = wsum.alloc(arena, sizeof(XYZZ<DF>) * W))) return rc;

  GM_HIP(hipMemsetAsync(counts.p, 0, sizeof(uint32_t) * (total + 1), st));
  const uint32_t* sc = reinterpret_cast<const uint32_t*>(scalars_dev);
  {
    ProfScope ps(ctx, "msm_hist");
    hipLaunchKernelGGL(k_msm_hist<typename C::Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, st, sc,
                       (uint32_t)n, c, W, counts.as<uint32_t>());
  }
  GM_HIP(hipGetLastError());
  size_t tmp_bytes = 0;
  GM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, counts.as<uint32_t>(),
                                          offsets.as<uint32_t>(), total + 1, st));
  if ((rc = scan_tmp.alloc(arena, tmp_bytes))) return rc;
  {
    ProfScope ps(ctx, "msm_scan");
    GM_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp.p, tmp_bytes, counts.as<uint32_t>(),
                                            offsets.as<uint32_t>(), total + 1, st));
  }
  // cursor = offsets (reuse counts buffer)
  GM_HIP(hipMemcpyAsync(counts.p, offsets.p, sizeof(uint32_t) * (total + 1), hipMemcpyDeviceToDevice, st));
  {
    ProfScope ps(ctx, "msm_scatter");
    hipLaunchKernelGGL(k_msm_scatter<typename C::Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, st, sc,
                       (uint32_t)n, c, W, counts.as<uint32_t>(), offsets.as<uint32_t>() + 1,
                       sorted.as<uint32_t>(), errw.as<uint32_t>());
  }
  {
    ProfScope ps(ctx, G2 ? "msm_accum_g2" : "msm_accum_g1");
    hipLaunchKernelGGL(k_msm_accum<DF>, dim3(blocks_for(total, 128)), dim3(128), 0, st,
                       reinterpret_cast<const Affine<DF>*>(points_dev), (uint32_t)n,
                       sorted.as<uint32_t>(), offsets.as<uint32_t>(), total, buckets.as<XYZZ<DF>>(),
                       errw.as<uint32_t>());
  }
  {
    ProfScope ps(ctx, "msm_bucket_reduce");
    hipLaunchKernelGGL(k_msm_seg<DF>, dim3(blocks_for((size_t)W * nseg, 128)), dim3(128), 0, st,
                       buckets.as<XYZZ<DF>>(), nb, L, nseg, W, segT.as<XYZZ<DF>>(), segS.as<XYZZ<DF>>());
    hipLaunchKernelGGL(k_msm_segmul<DF>, dim3(blocks_for((size_t)W * nseg, 128)), dim3(128), 0, st,
                       segT.as<XYZZ<DF>>(), segS.as<XYZZ<DF>>(), L, nseg, W);
    constexpr int TPB = 128;
    hipLaunchKernelGGL((k_msm_winsum<DF, TPB>), dim3(W), dim3(TPB), sizeof(XYZZ<DF>) * TPB, st,
                       segT.as<XYZZ<DF>>(), nseg, wsum.as<XYZZ<DF>>());
  }
  GM_HIP(hipGetLastError());
  if (getenv("GM_DEBUG_MSM")) {
    GM_HIP(hipStreamSynchronize(st));
    std::vector<HF> hb(4 * (size_t)total);
    GM_HIP(hipMemcpy(hb.data(), buckets.p, sizeof(XYZZ<DF>) * total, hipMemcpyDeviceToHost));
    size_t nonzero = 0;
    for (size_t b = 0; b < total; b++) nonzero += !hb[4 * b + 2].is_zero();
    std::vector<uint32_t> off(total + 1);
    GM_HIP(hipMemcpy(off.data(), offsets.p, 4 * (total + 1), hipMemcpyDeviceToHost));
    std::vector<HF> ht(4 * (size_t)W * nseg);
    GM_HIP(hipMemcpy(ht.data(), segT.p, sizeof(XYZZ<DF>) * W * nseg, hipMemcpyDeviceToHost));
    size_t nzT = 0;
    for (size_t b = 0; b < (size_t)W * nseg; b++) nzT += !ht[4 * b + 2].is_zero();
    std::vector<uint32_t> hs(8 * std::min<size_t>(n, 4));
    GM_HIP(hipMemcpy(hs.data(), scalars_dev, 4 * hs.size(), hipMemcpyDeviceToHost));
    uint32_t e2 = 0;
    GM_HIP(hipMemcpy(&e2, errw.p, 4, hipMemcpyDeviceToHost));
    fprintf(stderr, "[msm dbg] n=%zu c=%u W=%u entries=%u nonzero_buckets=%zu nonzero_R=%zu err=%u s0=%08x%08x\n",
            n, c, W, off[total], nonzero, nzT, e2, hs[1], hs[0]);
  }
  uint32_t herr = 0;
  GM_HIP(hipMemcpyAsync(&herr, errw.p, 4, hipMemcpyDeviceToHost, st));
  std::vector<HF> hw(4 * W);
  static_assert(sizeof(HF) * 4 == sizeof(XYZZ<DF>), "host/device layout mismatch");
  GM_HIP(hipMemcpyAsync(hw.data(), wsum.p, sizeof(XYZZ<DF>) * W, hipMemcpyDeviceToHost, st));
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

template int msm_device<CurveBN254, false>(gm_ctx*, const void*, const void*, size_t,
                                           CurveBN254::HG1F (&)[3]);
template int msm_device<CurveBN254, true>(gm_ctx*, const void*, const void*, size_t,
                                          CurveBN254::HG2F (&)[3]);
template int msm_device<CurveBLS12377, false>(gm_ctx*, const void*, const void*, size_t,
                                              CurveBLS12377::HG1F (&)[3]);
template int msm_device<CurveBLS12377, true>(gm_ctx*, const void*, const void*, size_t,
                                             CurveBLS12377::HG2F (&)[3]);

}  // namespace gm
