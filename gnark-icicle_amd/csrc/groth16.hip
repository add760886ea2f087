// Groth16 prover on one or several MI355X GPUs -- replaces the device block of
// icicle_bn254.Prove (backend/groth16/bn254/icicle/icicle.go:133-422),
// re-derived from the current CPU prover groth16_bn254.Prove
// (backend/groth16/bn254/prove.go:62-325) as SURVEY.md §0.3 prescribes: only
// computeH, the compaction and the five MSMs move to the device; the O(1)
// finishing adds (prove.go:195-305) run on the host.
//
// One proof = five MSM sums over the key's (sharded) point arrays:
//   A  = <wA, pk.G1.A>,  B = <wB, pk.G1.B>,  B2 = <wB, pk.G2.B>,
//   K  = <wK, pk.G1.K>,  Z = <h[:n-1], pk.G1.Z>
// g16_sums_t computes them on one device; an HSource supplies h (computeH on
// this device from resident or host-staged a/b/c, or slices distributed by
// another device of a gm_multi).  Sums of several shards / devices add up.
#include <atomic>
#include <cstdint>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "curves.hpp"
#include "msm.hpp"
#include "ntt.hpp"
#include "groth16.hpp"
#include "runtime.hpp"

using namespace gm;

namespace gm {

// A copy between the buffers of two gm_multi devices takes the peer path
// (hipMemcpyPeerAsync over xGMI) when the devices differ.  GM_MULTI_FORCE_PEER=1
// (test knob, read per call) takes it for equal devices too, so a one-GPU box
// runs the peer branches of the multi-device prover (hipMemcpyPeerAsync with
// equal devices is a plain device-to-device copy).
static bool cross_device(int a, int b) {
  if (a != b) return true;
  const char* f = getenv("GM_MULTI_FORCE_PEER");
  return f && atoi(f) != 0;
}

int check_curve_id(int curve) {
  if (curve != GM_BN254 && curve != GM_BLS12_377) {
    set_error("unknown curve id");
    return GM_ERR_INVALID;
  }
  return GM_OK;
}

namespace {
// dst[i] = src[idx[i]] (Fr, 32 bytes) -- device-side scalar compaction
__global__ void k_gather_fr(const uint4* __restrict__ src, const uint32_t* __restrict__ idx, size_t n,
                            uint4* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t j = idx[i];
  dst[2 * i] = src[2 * j];
  dst[2 * i + 1] = src[2 * j + 1];
}

// [lo, hi) of rank's contiguous shard of n items (gnark_mi355x.shard_range)
void shard_of(size_t n, int rank, int world, size_t* lo, size_t* hi) {
  const size_t q = n / (size_t)world, r = n % (size_t)world;
  *lo = (size_t)rank * q + std::min((size_t)rank, r);
  *hi = *lo + q + ((size_t)rank < r ? 1 : 0);
}

// [lo, hi) of part k of n items split in proportion to weights w
void shard_weighted(size_t n, const std::vector<double>& w, int k, size_t* lo, size_t* hi) {
  double tot = 0, before = 0;
  for (size_t i = 0; i < w.size(); i++) {
    tot += w[i];
    if ((int)i < k) before += w[i];
  }
  *lo = (size_t)((double)n * before / tot);
  *hi = k + 1 == (int)w.size() ? n : (size_t)((double)n * (before + w[k]) / tot);
}

}  // namespace

size_t internal_point_bytes(int curve, bool g2) {
  if (curve == GM_BN254)
    return g2 ? msm_internal_point_bytes<CurveBN254, true>() : msm_internal_point_bytes<CurveBN254, false>();
  return g2 ? msm_internal_point_bytes<CurveBLS12377, true>() : msm_internal_point_bytes<CurveBLS12377, false>();
}

void pk_release(gm_g16_pk* pk) {
  stage_spare_release(pk);
  for (void* q : {pk->A, pk->B, pk->Z, pk->K, pk->B2, pk->idxA, pk->idxB, pk->idxK})
    if (q) hipFree(q);
  delete pk;
}

void wire_plan_choice(size_t span, size_t nbA, size_t nbB, size_t nbK, bool out[3]) {
  const char* env = getenv("GM_G16_WIRE_PLAN");  // read per key (tests flip it)
  const bool on = !env || atoi(env) != 0;
  const size_t cnt[3] = {nbA, nbB, nbK};
  int k = 0;
  for (int x = 0; x < 3; x++) {
    out[x] = on && span > 0 && cnt[x] <= span && 32 * cnt[x] >= 31 * span;
    k += out[x];
  }
  if (k < 2)
    for (int x = 0; x < 3; x++) out[x] = false;
}

void wire_plan_maps(size_t span, const uint32_t* const idx[3], const size_t cnt[3], bool want[3],
                    std::vector<uint32_t> map[3]) {
  int k = 0;
  for (int x = 0; x < 3; x++) {
    if (!want[x]) continue;
    map[x].assign(span, MSM_SKIP);
    for (size_t j = 0; j < cnt[x] && want[x]; j++) {
      const uint32_t w = idx[x][j];
      if (w >= span || map[x][w] != MSM_SKIP) want[x] = false;  // a wire used twice: own plan
      else map[x][w] = (uint32_t)j;
    }
    k += want[x];
  }
  if (k < 2)
    for (int x = 0; x < 3; x++) want[x] = false;  // not worth a shared plan
}

namespace {
// Wire-indexed copy of a compacted internal point array (and its window
// copies): dst[w * span + i] = src[w * cnt + map[i]], infinity (all zero)
// where wire i has no point.  q = 16-byte chunks per point.
__global__ void k_expand_points(const uint4* __restrict__ src, size_t cnt, const uint32_t* __restrict__ map,
                                size_t span, size_t total, uint32_t q, uint4* __restrict__ dst) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const size_t p = t / q, k = t - p * q;
  const size_t w = p / span, i = p - w * span;
  const uint32_t m = map[i];
  dst[t] = m == MSM_SKIP ? make_uint4(0, 0, 0, 0) : src[((size_t)w * cnt + m) * q + k];
}
}  // namespace

int prepare_points_into(gm_ctx* ctx, int curve, bool g2, const void* gnark_dev, size_t count,
                        const MsmPrecomp* pre, void* dst) {
  if (pre) {
    if (curve == GM_BN254)
      return g2 ? msm_precompute_points<CurveBN254, true>(ctx, gnark_dev, count, *pre, dst)
                : msm_precompute_points<CurveBN254, false>(ctx, gnark_dev, count, *pre, dst);
    return g2 ? msm_precompute_points<CurveBLS12377, true>(ctx, gnark_dev, count, *pre, dst)
              : msm_precompute_points<CurveBLS12377, false>(ctx, gnark_dev, count, *pre, dst);
  }
  if (curve == GM_BN254)
    return g2 ? msm_prepare_points<CurveBN254, true>(ctx, gnark_dev, count, dst)
              : msm_prepare_points<CurveBN254, false>(ctx, gnark_dev, count, dst);
  return g2 ? msm_prepare_points<CurveBLS12377, true>(ctx, gnark_dev, count, dst)
            : msm_prepare_points<CurveBLS12377, false>(ctx, gnark_dev, count, dst);
}

// Uploads the [lo, hi) slices of the key's point arrays (h's pointers address
// the first point of each slice, or `src` fetches them) and the matching slices
// of the compaction maps (setupDevicePointers, icicle.go:31-130; the maps
// replace icicle.go:231-278's host filtering, prove.go:157-178 / 243-245).
int pk_upload_ranges(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, unsigned flags, const Ranges& rg,
                     gm_g16_pk** out, const PointSource* src) {
  auto* pk = new gm_g16_pk();
  pk->curve = curve;
  pk->n = h->domain_size;
  pk->nb_wires = h->nb_wires;
  pk->nb_public = h->nb_public;
  pk->nbA = rg.hiA - rg.loA;
  pk->nbB = rg.hiB - rg.loB;
  pk->nbK = rg.hiK - rg.loK;
  pk->zlo = rg.loZ;
  pk->nbZ = rg.hiZ - rg.loZ;
  pk->precomp = (flags & GM_PK_PRECOMPUTE) != 0;
  const bool precomp_auto = !pk->precomp && (flags & GM_PK_PRECOMPUTE_AUTO);
  const int frbits = curve == GM_BN254 ? CurveBN254::FR_BITS : CurveBLS12377::FR_BITS;
  auto fail = [&](int code) {
    pk_release(pk);
    return code;
  };
  // compaction maps (prove.go:157-178: drop wire i when InfinityA[i] / InfinityB[i];
  // K: the k_wires survivors of filterHeap, prove.go:243-245, or nb_public + i)
  std::vector<uint32_t> ia, ib, ik;
  for (size_t i = 0; i < pk->nb_wires; i++) {
    if (!h->infA[i]) ia.push_back((uint32_t)i);
    if (!h->infB[i]) ib.push_back((uint32_t)i);
  }
  for (size_t i = 0; i < h->nbK; i++) {
    const size_t w = h->k_wires ? (size_t)h->k_wires[i] : pk->nb_public + i;
    if (w >= pk->nb_wires || w < pk->nb_public) {
      set_error("pk upload: K wire index out of range");
      return fail(GM_ERR_INVALID);
    }
    ik.push_back((uint32_t)w);
  }
  if (ia.size() != h->nbA || ib.size() != h->nbB || pk->nb_public + h->nbK > pk->nb_wires) {
    set_error("pk upload: infinity masks inconsistent with nbA/nbB/nbK");
    return fail(GM_ERR_INVALID);
  }
  // wire range this key's slices read
  pk->wlo = 0;
  pk->whi = pk->nb_wires;
  if (rg.rebase) {
    size_t lo = SIZE_MAX, hi = 0;
    auto span = [&](const std::vector<uint32_t>& v, size_t a, size_t b) {
      for (size_t i = a; i < b; i++) {
        lo = std::min(lo, (size_t)v[i]);
        hi = std::max(hi, (size_t)v[i] + 1);
      }
    };
    span(ia, rg.loA, rg.hiA);
    span(ib, rg.loB, rg.hiB);
    span(ik, rg.loK, rg.hiK);
    if (hi <= lo) lo = hi = 0;
    pk->wlo = lo;
    pk->whi = hi;
    for (auto* v : {&ia, &ib, &ik})
      for (auto& x : *v) x -= (x >= lo ? (uint32_t)lo : x);  // entries outside the slice are never read
  }
  // Shared wire plan: arrays covering (nearly) every wire of the span are
  // stored wire-indexed (expanded, infinity where a wire has no point), so one
  // plan over the wires addresses all of them directly; window geometry and
  // stride are the plan's.  The others keep their own compacted layout.
  const size_t span = pk->whi - pk->wlo;
  std::vector<uint32_t> wmap[3];
  {
    const uint32_t* idx[3] = {ia.data() + rg.loA, ib.data() + rg.loB, ik.data() + rg.loK};
    const size_t cnt[3] = {pk->nbA, pk->nbB, pk->nbK};
    wire_plan_choice(span, pk->nbA, pk->nbB, pk->nbK, pk->wshare);
    wire_plan_maps(span, idx, cnt, pk->wshare, wmap);
  }
  // GM_PK_PRECOMPUTE_AUTO: the window copies when they fit the device (the
  // final arrays plus the largest array's transient upload buffers within
  // GM_PK_PRECOMPUTE_FRAC of the free memory)
  if (precomp_auto) {
    const MsmPrecomp pw = msm_choose_precomp(span, frbits);
    auto bytes_of = [&](size_t cnt, bool shared, bool g2) {
      const MsmPrecomp p = shared ? pw : msm_choose_precomp(cnt, frbits);
      return (double)internal_point_bytes(curve, g2) * (double)p.W * (double)(shared ? span : cnt);
    };
    const double arr[5] = {bytes_of(pk->nbA, pk->wshare[0], false), bytes_of(pk->nbB, pk->wshare[1], false),
                           bytes_of(pk->nbK, pk->wshare[2], false), bytes_of(pk->nbZ, false, false),
                           bytes_of(pk->nbB, pk->wshare[1], true)};
    double need = 0, largest = 0;
    for (double b : arr) {
      need += b;
      largest = std::max(largest, b);
    }
    need += largest / 8;  // gnark-layout staging of the largest array
    // the streamed (dump) path builds a shared array's compacted precomputed copy
    // before expanding it: one more array at the upload's peak
    if (src && (pk->wshare[0] || pk->wshare[1] || pk->wshare[2])) need += largest;
    // computeH's two n-element tables, built at the end of the upload (pk_prepare_h)
    need += 2.0 * 36.0 * (double)pk->n;
    size_t fr = 0, tot = 0;
    const char* fenv = getenv("GM_PK_PRECOMPUTE_FRAC");
    const double frac = fenv ? atof(fenv) : 0.6;
    pk->precomp = hipMemGetInfo(&fr, &tot) == hipSuccess && need <= frac * (double)fr;
  }
  if (pk->precomp) {
    const MsmPrecomp pw = msm_choose_precomp(span, frbits);
    auto geom = [&](size_t cnt, bool shared) {
      MsmPrecomp p = shared ? pw : msm_choose_precomp(cnt, frbits);
      p.stride = shared ? span : cnt;
      return p;
    };
    pk->preA = geom(pk->nbA, pk->wshare[0]);
    pk->preB = geom(pk->nbB, pk->wshare[1]);
    pk->preK = geom(pk->nbK, pk->wshare[2]);
    pk->preZ = msm_choose_precomp(pk->nbZ, frbits);
    pk->preW = pw;
    pk->preW.stride = span;
  }
  const size_t g1b = 2 * fp_bytes(curve), g2b = 4 * fp_bytes(curve);
  auto up = [&](const void* src, size_t bytes, void** dst) -> int {
    hipError_t e = hipMalloc(dst, bytes ? bytes : 16);
    if (e != hipSuccess) {
      set_error(std::string("pk upload hipMalloc: ") + hipGetErrorString(e));
      return GM_ERR_OOM;
    }
    if (bytes) {
      e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        set_error(std::string("pk upload hipMemcpy: ") + hipGetErrorString(e));
        return GM_ERR_DEVICE;
      }
    }
    return GM_OK;
  };
  // gnark-layout points -> device-internal layout, once (plus the W-1
  // window-shifted copies with GM_PK_PRECOMPUTE, msm_precompute_points)
  // emap: wire map of an expanded (shared-plan) array, else null
  auto up_compact = [&](int which, const void* hsrc, size_t count, bool g2, const MsmPrecomp& pre,
                        void** dst) -> int {
    const size_t copies = pk->precomp ? pre.W : 1;
    hipError_t e = hipMalloc(dst, internal_point_bytes(curve, g2) * (count ? count * copies : 1));
    if (e != hipSuccess) {
      set_error(std::string("pk upload hipMalloc: ") + hipGetErrorString(e));
      return GM_ERR_OOM;
    }
    if (src) return (*src)(which, count, g2, pk->precomp ? &pre : nullptr, *dst);
    void* tmp = nullptr;
    int r = up(hsrc, (g2 ? g2b : g1b) * count, &tmp);
    if (r) {
      if (tmp) hipFree(tmp);
      return r;
    }
    r = prepare_points_into(ctx, curve, g2, tmp, count, pk->precomp ? &pre : nullptr, *dst);
    hipStreamSynchronize(ctx->stream);
    hipFree(tmp);
    return r;
  };
  // Wire-indexed (shared-plan) array from host memory: the gnark-layout points
  // are expanded to the wire span first (infinity = (0, 0) where a wire has no
  // point), then converted / precomputed straight into the final array -- no
  // precomputed compacted copy is ever materialised (peak = final + span gnark
  // points, not twice the final size).
  auto up_expanded_gnark = [&](const void* hsrc, size_t count, bool g2, const MsmPrecomp& pre, void** dst,
                               const std::vector<uint32_t>& emap) -> int {
    const size_t gpb = g2 ? g2b : g1b;
    void *tmp = nullptr, *wide = nullptr, *dmap = nullptr;
    auto done = [&](int r) {
      for (void* q : {tmp, wide, dmap})
        if (q) hipFree(q);
      return r;
    };
    int r = up(hsrc, gpb * count, &tmp);
    if (r) return done(r);
    if ((r = up(emap.data(), 4 * span, &dmap))) return done(r);
    if (hipMalloc(&wide, gpb * (span ? span : 1)) != hipSuccess) {
      set_error("pk upload: hipMalloc of an expanded array failed");
      return done(GM_ERR_OOM);
    }
    const size_t q = gpb / 16, total = span * q;
    if (span)
      hipLaunchKernelGGL(k_expand_points, dim3(blocks_for(total, 256)), dim3(256), 0, ctx->stream, (const uint4*)tmp,
                         count, (const uint32_t*)dmap, span, total, (uint32_t)q, (uint4*)wide);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess) {
      set_error("pk upload: expanding a point array failed");
      return done(GM_ERR_DEVICE);
    }
    hipFree(tmp);
    tmp = nullptr;
    const size_t copies = pk->precomp ? pre.W : 1;
    if (hipMalloc(dst, internal_point_bytes(curve, g2) * (span ? span * copies : 1)) != hipSuccess) {
      set_error("pk upload hipMalloc: out of device memory");
      return done(GM_ERR_OOM);
    }
    r = prepare_points_into(ctx, curve, g2, wide, span, pk->precomp ? &pre : nullptr, *dst);
    if (hipStreamSynchronize(ctx->stream) != hipSuccess && !r) r = GM_ERR_DEVICE;
    return done(r);
  };
  auto up_pts = [&](int which, const void* hsrc, size_t count, bool g2, const MsmPrecomp& pre, void** dst,
                    const std::vector<uint32_t>* emap) -> int {
    if (!emap) return up_compact(which, hsrc, count, g2, pre, dst);
    if (!src) return up_expanded_gnark(hsrc, count, g2, pre, dst, *emap);
    MsmPrecomp pc = pre;  // streamed (dump): compacted first (stride = count), then expanded to the span
    pc.stride = count;
    void* tmp = nullptr;
    int r = up_compact(which, hsrc, count, g2, pc, &tmp);
    const size_t copies = pk->precomp ? pre.W : 1;
    const size_t ipb = internal_point_bytes(curve, g2), total = span * copies * (ipb / 16);
    void* dmap = nullptr;
    if (r == GM_OK && (hipMalloc(dst, ipb * (span ? span * copies : 1)) != hipSuccess ||
                       hipMalloc(&dmap, 4 * (span ? span : 1)) != hipSuccess)) {
      set_error("pk upload: hipMalloc of an expanded array failed");
      r = GM_ERR_OOM;
    }
    if (r == GM_OK && span) {
      if (hipMemcpy(dmap, emap->data(), 4 * span, hipMemcpyHostToDevice) != hipSuccess) r = GM_ERR_DEVICE;
      if (r == GM_OK)
        hipLaunchKernelGGL(k_expand_points, dim3(blocks_for(total, 256)), dim3(256), 0, ctx->stream,
                           (const uint4*)tmp, count, (const uint32_t*)dmap, span, total, (uint32_t)(ipb / 16),
                           (uint4*)*dst);
      if (r == GM_OK && (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess))
        r = GM_ERR_DEVICE;
      if (r) set_error("pk upload: expanding a point array failed");
    }
    if (tmp) hipFree(tmp);
    if (dmap) hipFree(dmap);
    return r;
  };
  auto em = [&](int x) { return pk->wshare[x] ? &wmap[x] : nullptr; };
  int rc;
  if ((rc = up_pts(PK_A, h->g1_A, pk->nbA, false, pk->preA, &pk->A, em(0))) ||
      (rc = up_pts(PK_B, h->g1_B, pk->nbB, false, pk->preB, &pk->B, em(1))) ||
      (rc = up_pts(PK_Z, h->g1_Z, pk->nbZ, false, pk->preZ, &pk->Z, nullptr)) ||
      (rc = up_pts(PK_K, h->g1_K, pk->nbK, false, pk->preK, &pk->K, em(2))) ||
      (rc = up_pts(PK_B2, h->g2_B, pk->nbB, true, pk->preB, &pk->B2, em(1))))
    return fail(rc);
  if ((rc = up(ia.data() + rg.loA, 4 * pk->nbA, &pk->idxA)) || (rc = up(ib.data() + rg.loB, 4 * pk->nbB, &pk->idxB)) ||
      (rc = up(ik.data() + rg.loK, 4 * pk->nbK, &pk->idxK)))
    return fail(rc);
  auto cp = [](std::vector<uint8_t>& v, const void* s, size_t b) {
    v.resize(b);
    memcpy(v.data(), s, b);
  };
  cp(pk->alpha, h->g1_alpha, g1b);
  cp(pk->beta, h->g1_beta, g1b);
  cp(pk->delta, h->g1_delta, g1b);
  cp(pk->beta2, h->g2_beta, g2b);
  cp(pk->delta2, h->g2_delta, g2b);
  pk_prepare_h(ctx, pk);
  *out = pk;
  return GM_OK;
}

void pk_prepare_h(gm_ctx* ctx, const gm_g16_pk* pk) {
  const std::string saved = last_error();
  const int rc = pk->curve == GM_BN254 ? compute_h_prepare<CurveBN254>(ctx, pk->n)
                                       : compute_h_prepare<CurveBLS12377>(ctx, pk->n);
  if (rc) {  // e.g. out of memory: the first prove builds them (or reports it); the upload succeeded
    (void)hipGetLastError();
    set_error(saved);
  }
}

namespace {

// ---------------------------------------------------------------------------
// Sources of h (the bit-reversed computeH output, icicle.go:453-513 /
// prove.go:356-399) for the Z MSM.  poll() is called between the A/B/K MSMs
// (which need no h) and launches work whose inputs have arrived; z_scalars()
// makes the main stream wait for this key's slice of h and returns it.
// ---------------------------------------------------------------------------
struct HSource {
  virtual ~HSource() {}
  virtual int poll() { return GM_OK; }
  virtual int z_scalars(const void** zs) = 0;
};

// computeH on the context's auxiliary stream, overlapped with the MSMs (whose
// sorts, reductions and host round trips leave the VALUs idle).
// r1: a, b, c are first evaluated from the wires by the device-resident R1CS
// (gm_g16_prove_r1cs), on the same stream as computeH.
template <class C>
int launch_compute_h(gm_ctx* ctx, void* a, void* b, void* c, size_t nc, size_t n, hipEvent_t wait_for,
                     hipEvent_t done, const gm_r1cs* r1 = nullptr, const void* wires = nullptr) {
  // n == 0: only the R1CS evaluation (no done event); computeH follows later
  auto body = [&]() -> int {
    int rc;
    if (r1 && (rc = r1cs_eval_device(ctx, r1, wires, a, b, c))) return rc;
    return n ? compute_h_device<C>(ctx, a, b, c, nc, n) : GM_OK;
  };
  if (wait_for) GM_HIP(hipStreamWaitEvent(ctx->aux, wait_for, 0));
  hipStream_t main = ctx->stream;
  ctx->stream = ctx->aux;
  int rc = body();
  ctx->stream = main;
  if (rc) return rc;
  if (done) GM_HIP(hipEventRecord(done, ctx->aux));
  return GM_OK;
}

struct EventPair {
  hipEvent_t a = nullptr, b = nullptr;
  int create() {
    GM_HIP(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    GM_HIP(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    return GM_OK;
  }
  ~EventPair() {
    if (a) hipEventDestroy(a);
    if (b) hipEventDestroy(b);
  }
};

// a, b, c already on the device (queued on the main stream): computeH starts at once.
template <class C>
struct DeviceH : HSource {
  gm_ctx* ctx;
  gm_g16_pk* pk;
  void *a, *b, *c;
  size_t nc;
  const gm_r1cs* r1 = nullptr;  // set: a, b, c evaluated from `wires` first
  const void* wires = nullptr;
  EventPair ev;  // a: inputs ready (main stream), b: h ready
  bool launched = false;
  DeviceH(gm_ctx* x, gm_g16_pk* k, void* a_, void* b_, void* c_, size_t n_) : ctx(x), pk(k), a(a_), b(b_), c(c_), nc(n_) {}
  // computeH is queued at the first poll(), i.e. after the shared wire plan's
  // digits / sort (g16_sums_t polls once the plan is queued) and ordered after
  // it: the LDS-heavy sort passes and NTT passes slow each other down (r03
  // timeline: k_msm_s2_local 1.2 -> 14.5 ms beside the NTT) while the
  // VALU-bound accumulation shares the chip with them at no extra cost.
  // The R1CS evaluation (a
  // latency-bound gather, 0.65 ms alone at 2^24 but 18 ms beside the
  // accumulation) is not deferred: it runs on the auxiliary stream next to the
  // digit pass.
  int start() {
    int rc;
    if ((rc = ev.create())) return rc;
    if (r1) {
      GM_HIP(hipEventRecord(ev.a, ctx->stream));
      if ((rc = launch_compute_h<C>(ctx, a, b, c, nc, 0, ev.a, nullptr, r1, wires))) return rc;
      r1 = nullptr;
    }
    return GM_OK;
  }
  int launch() {
    if (launched) return GM_OK;
    launched = true;
    GM_HIP(hipEventRecord(ev.a, ctx->stream));
    return launch_compute_h<C>(ctx, a, b, c, nc, pk->n, ev.a, ev.b, r1, wires);
  }
  int poll() override { return launch(); }
  int z_scalars(const void** zs) override {
    int rc;
    if ((rc = launch())) return rc;
    GM_HIP(hipStreamWaitEvent(ctx->stream, ev.b, 0));
    *zs = (const char*)a + 32 * pk->zlo;
    return GM_OK;
  }
  ~DeviceH() override { hipStreamSynchronize(ctx->aux); }
};

// The context's pinned H2D ring (HostStagedH), created on first use or ahead of
// it (pk_prepare_h); false when pinned memory or an event is not available (the
// copies then take the pageable path instead of failing the prove).
bool h2d_ring_ensure(gm_ctx* ctx) {
  bool ok = true;
  for (int i = 0; i < gm_ctx::H2D_SLOTS && ok; i++) {
    if (!ctx->h2d_pin[i] && hipHostMalloc(&ctx->h2d_pin[i], gm_ctx::H2D_SLOT, hipHostMallocDefault) != hipSuccess) {
      ctx->h2d_pin[i] = nullptr;
      ok = false;
    }
    if (ok && !ctx->h2d_ev[i] && hipEventCreateWithFlags(&ctx->h2d_ev[i], hipEventDisableTiming) != hipSuccess) {
      ctx->h2d_ev[i] = nullptr;
      ok = false;
    }
  }
  (void)hipGetLastError();  // a failed allocation is not the caller's error
  return ok;
}

// The context's a / b / c input buffer of host-input proves (gm_ctx::in_abc),
// grown to 3 n elements.
int in_abc_reserve(gm_ctx* ctx, size_t n) {
  const size_t abc = 3 * 32 * n;
  if (ctx->in_abc_cap >= abc) return GM_OK;
  void* old = ctx->in_abc;
  ctx->in_abc = nullptr;  // released below; never left pointing at freed memory
  ctx->in_abc_cap = 0;
  if (old) GM_HIP(hipFree(old));
  if (hipMalloc(&ctx->in_abc, abc) != hipSuccess) {
    ctx->in_abc = nullptr;
    set_error("prove: hipMalloc of the a/b/c input buffer failed");
    return GM_ERR_OOM;
  }
  ctx->in_abc_cap = abc;
  return GM_OK;
}

// a, b, c in host memory: a helper thread copies them on the context's copy
// stream (pageable hipMemcpyAsync runs at ~56 GB/s on the box but blocks the
// calling thread) while the main thread runs the A/B/K MSMs; each vector's
// computeH chain is launched on the auxiliary stream at the first poll() after
// that vector's copies are queued, the fused tail once all three are.  `after_h`
// (multi-device) runs right after the tail is queued.
template <class C>
struct HostStagedH : HSource {
  gm_ctx* ctx;
  gm_g16_pk* pk;
  void *da, *db, *dc;
  const void *ha, *hb, *hc;
  size_t nc;
  EventPair ev;             // b: h ready
  hipEvent_t vev[3] = {};   // a / b / c copied (copy stream)
  std::thread th;
  std::atomic<int> nq{0};   // vectors whose copies are queued (vev recorded)
  std::atomic<int> copy_rc{GM_OK};
  std::string copy_err;
  int chained = 0;          // computeH chains queued (a, b, c in order)
  bool launched = false;
  std::function<int()> after_h;
  HostStagedH(gm_ctx* x, gm_g16_pk* k, void* a_, void* b_, void* c_, const void* ha_, const void* hb_,
              const void* hc_, size_t n_)
      : ctx(x), pk(k), da(a_), db(b_), dc(c_), ha(ha_), hb(hb_), hc(hc_), nc(n_) {}
  int start() {
    int rc;
    if ((rc = ev.create())) return rc;
    for (hipEvent_t& e : vev) GM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // A pageable copy issued
    // from this thread while the MSMs ran could stall until an accumulation kernel
    // ended (fresh process: copies after the B2 MSM, 2^24 prove 199 ms instead of
    // ~167, profiles/r04s_g16_host_slow_copies.txt); through the context's pinned
    // ring (memcpy into a 32 MiB slot, then an async copy from pinned memory) the
    // DMA does not wait for the kernels.  The slot fill is split over
    // H2D_FILL_THREADS (4) threads: with one, a 32 MiB fill took 1.55 ms against
    // the DMA's 0.59 ms and a, b, c arrived only ~75 ms into a 2^24 prove
    // (profiles/r05i_host_prove_timeline.txt).
    th = std::thread([this] {
      int r = GM_OK;
      if (hipSetDevice(ctx->device) != hipSuccess) r = GM_ERR_DEVICE;
      const void* src[3] = {ha, hb, hc};
      void* dst[3] = {da, db, dc};
      // the ring is created on first use; when pinned memory (or an event) is not
      // available the copies take the pageable path instead of failing the prove
      const bool ring = r == GM_OK && h2d_ring_ensure(ctx);
      bool used[gm_ctx::H2D_SLOTS] = {};
      int slot = 0;
      for (int k = 0; k < 3 && r == GM_OK; k++) {
        if (ring) {
          for (size_t off = 0; off < 32 * nc && r == GM_OK; off += gm_ctx::H2D_SLOT) {
            const size_t len = std::min(gm_ctx::H2D_SLOT, 32 * nc - off);
            if (used[slot] && hipEventSynchronize(ctx->h2d_ev[slot]) != hipSuccess) r = GM_ERR_DEVICE;
            if (r) break;
            par_memcpy(ctx->h2d_pin[slot], (const char*)src[k] + off, len, H2D_FILL_THREADS);
            if (hipMemcpyAsync((char*)dst[k] + off, ctx->h2d_pin[slot], len, hipMemcpyHostToDevice, ctx->copy) !=
                    hipSuccess ||
                hipEventRecord(ctx->h2d_ev[slot], ctx->copy) != hipSuccess)
              r = GM_ERR_DEVICE;
            used[slot] = true;
            slot = (slot + 1) % gm_ctx::H2D_SLOTS;
          }
        } else if (nc && hipMemcpyAsync(dst[k], src[k], 32 * nc, hipMemcpyHostToDevice, ctx->copy) != hipSuccess) {
          r = GM_ERR_DEVICE;
        }
        if (r == GM_OK && hipEventRecord(vev[k], ctx->copy) != hipSuccess) r = GM_ERR_DEVICE;
        if (r == GM_OK) nq = k + 1;  // vector k may be chained
      }
      if (r) copy_err = "staged a/b/c upload failed";
      copy_rc = r;
    });
    return GM_OK;
  }
  // computeH in pieces as the inputs arrive: the chain of vector k (pad, INTT,
  // coset NTT) waits only for k's copies, the fused tail for all three
  // (on ctx->aux, as launch_compute_h).  block: wait for every copy to be queued.
  int launch(bool block) {
    if (launched) return GM_OK;
    if (block && th.joinable()) th.join();
    if (copy_rc) {
      if (th.joinable()) th.join();
      set_error(copy_err);
      return copy_rc;
    }
    const int q = nq.load();
    if (chained >= q && !(block && q == 3)) return GM_OK;
    const hipStream_t hst = ctx->aux;
    void* vec[3] = {da, db, dc};
    {
      StreamSwap sw(ctx, hst);
      for (; chained < q; chained++) {
        GM_HIP(hipStreamWaitEvent(hst, vev[chained], 0));
        if (int rc = compute_h_chain<C>(ctx, vec[chained], nc, pk->n)) return rc;
      }
      if (chained < 3) return GM_OK;
      if (int rc = compute_h_finish<C>(ctx, da, db, dc, pk->n)) return rc;
      GM_HIP(hipEventRecord(ev.b, hst));
    }
    launched = true;
    if (th.joinable()) th.join();
    return after_h ? after_h() : GM_OK;
  }
  int poll() override { return launch(false); }
  int z_scalars(const void** zs) override {
    int rc;
    if ((rc = launch(true))) return rc;
    GM_HIP(hipStreamWaitEvent(ctx->stream, ev.b, 0));
    *zs = (const char*)da + 32 * pk->zlo;
    return GM_OK;
  }
  ~HostStagedH() override {
    if (th.joinable()) th.join();
    hipStreamSynchronize(ctx->copy);
    hipStreamSynchronize(ctx->aux);
    hipStreamSynchronize(ctx->stream);
    for (hipEvent_t e : vev)
      if (e) hipEventDestroy(e);
  }
};

// h slice delivered by another device (gm_multi): wait until the producer has
// queued the peer copy into `dst`, then for that copy itself.
struct SharedH {
  std::mutex mu;
  std::condition_variable cv;
  bool ready = false;
  int rc = GM_OK;
  hipEvent_t done = nullptr;  // on the producer's auxiliary stream, after the peer copies
};
struct RemoteH : HSource {
  SharedH* sh;
  const void* dst;
  RemoteH(SharedH* s, const void* d) : sh(s), dst(d) {}
  int z_scalars(const void** zs) override {
    std::unique_lock<std::mutex> lk(sh->mu);
    sh->cv.wait(lk, [&] { return sh->ready; });
    if (sh->rc) {
      set_error("h producer device failed");
      return sh->rc;
    }
    GM_HIP(hipEventSynchronize(sh->done));
    *zs = dst;
    return GM_OK;
  }
};

// ---------------------------------------------------------------------------
// computeH split across the devices of a gm_multi (the a, b, c
// INTT + coset-NTT chains are independent).  Device 1 runs b's chain (and c's
// with two devices), device 2 c's; each sends its result into device 0's
// buffer (xGMI peer copy) and signals a ChainDone.  Device 0 runs a's chain,
// then -- once b and c have arrived -- the fused pointwise + coset INTT, and
// distributes the h slices.  Every device also runs its MSM shards meanwhile.
// ---------------------------------------------------------------------------
struct ChainDone {
  std::mutex mu;
  std::condition_variable cv;
  bool recorded = false;  // `ev` recorded after the peer copies (or failure)
  int rc = GM_OK;
  hipEvent_t ev = nullptr;  // on the producer's auxiliary stream
  void signal(int r) {
    std::lock_guard<std::mutex> lk(mu);
    recorded = true;
    rc = r;
    cv.notify_all();
  }
  // 1 = arrived, 0 = not yet (non-blocking), < 0 = producer failed
  int ready(bool block) {
    std::unique_lock<std::mutex> lk(mu);
    if (block) cv.wait(lk, [&] { return recorded; });
    if (!recorded) return 0;
    if (rc) {
      set_error("computeH chain device failed");
      return rc;
    }
    lk.unlock();
    if (block) return hipEventSynchronize(ev) == hipSuccess ? 1 : GM_ERR_DEVICE;
    const hipError_t q = hipEventQuery(ev);
    return q == hipSuccess ? 1 : (q == hipErrorNotReady ? 0 : GM_ERR_DEVICE);
  }
};

// runs `f` with the context's main stream replaced by its auxiliary stream
template <class F>
int on_aux(gm_ctx* ctx, F&& f) {
  hipStream_t main = ctx->stream;
  ctx->stream = ctx->aux;
  int rc = f();
  ctx->stream = main;
  return rc;
}

// Producer side (devices 1, 2): h slice from device 0 like RemoteH, plus the
// chains of the host vectors it was given.
template <class C>
struct ChainRemoteH : RemoteH {
  gm_ctx* ctx;
  int dev0;
  size_t nc, n;
  struct Job {
    const void* host;  // solution.B / .C
    void* local;       // on this device
    void* dst;         // device 0's buffer
    ChainDone* done;
  };
  std::vector<Job> jobs;
  hipEvent_t copied = nullptr;
  std::thread th;
  std::atomic<bool> queued{false};
  std::atomic<int> copy_rc{GM_OK};
  bool launched = false;
  ChainRemoteH(SharedH* s, const void* d, gm_ctx* c, int dev0_, size_t nc_, size_t n_)
      : RemoteH(s, d), ctx(c), dev0(dev0_), nc(nc_), n(n_) {}
  int start() {
    GM_HIP(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
    th = std::thread([this] {
      int r = hipSetDevice(ctx->device) == hipSuccess ? GM_OK : GM_ERR_DEVICE;
      for (auto& j : jobs)
        if (r == GM_OK && nc && hipMemcpyAsync(j.local, j.host, 32 * nc, hipMemcpyHostToDevice, ctx->copy) != hipSuccess)
          r = GM_ERR_DEVICE;
      if (r == GM_OK && hipEventRecord(copied, ctx->copy) != hipSuccess) r = GM_ERR_DEVICE;
      copy_rc = r;
      queued = true;
    });
    return GM_OK;
  }
  int launch(bool block) {
    if (launched || jobs.empty()) return GM_OK;  // devices 3.. run no chain
    if (!block && !queued.load()) return GM_OK;
    if (th.joinable()) th.join();
    launched = true;
    int rc = copy_rc;
    if (rc == GM_OK)
      rc = on_aux(ctx, [&]() -> int {
        GM_HIP(hipStreamWaitEvent(ctx->stream, copied, 0));
        for (auto& j : jobs) {
          int r = compute_h_chain<C>(ctx, j.local, nc, n);
          if (r) return r;
          if (!cross_device(ctx->device, dev0))
            GM_HIP(hipMemcpyAsync(j.dst, j.local, 32 * n, hipMemcpyDeviceToDevice, ctx->stream));
          else
            GM_HIP(hipMemcpyPeerAsync(j.dst, dev0, j.local, ctx->device, 32 * n, ctx->stream));
        }
        for (auto& j : jobs) GM_HIP(hipEventRecord(j.done->ev, ctx->stream));
        return GM_OK;
      });
    for (auto& j : jobs) j.done->signal(rc);
    if (rc) set_error("computeH chain: " + std::string(gm_last_error()));
    return rc;
  }
  int poll() override { return launch(false); }
  int z_scalars(const void** zs) override {
    int rc;
    if ((rc = launch(true))) return rc;
    return RemoteH::z_scalars(zs);
  }
  ~ChainRemoteH() override {
    if (th.joinable()) th.join();
    if (!launched)
      for (auto& j : jobs) j.done->signal(GM_ERR_DEVICE);  // never leave device 0 waiting (no-op without jobs)
    hipStreamSynchronize(ctx->copy);
    hipStreamSynchronize(ctx->aux);
    if (copied) hipEventDestroy(copied);
  }
};

// Device 0 side: a's chain as soon as a is on the device, the fused tail once
// b and c have arrived, then `after_h` (the h slices to the other devices).
template <class C>
struct SplitH : HSource {
  gm_ctx* ctx;
  gm_g16_pk* pk;
  void *da, *db, *dc;
  const void* ha;
  size_t nc;
  std::vector<ChainDone*> remote;
  EventPair ev;  // a: a copied (copy stream), b: h ready (aux)
  std::thread th;
  std::atomic<bool> queued{false};
  std::atomic<int> copy_rc{GM_OK};
  int stage = 0;  // 0: nothing launched, 1: a's chain launched, 2: tail launched
  std::function<int()> after_h;
  SplitH(gm_ctx* x, gm_g16_pk* k, void* a_, void* b_, void* c_, const void* ha_, size_t n_)
      : ctx(x), pk(k), da(a_), db(b_), dc(c_), ha(ha_), nc(n_) {}
  int start() {
    int rc;
    if ((rc = ev.create())) return rc;
    th = std::thread([this] {
      int r = hipSetDevice(ctx->device) == hipSuccess ? GM_OK : GM_ERR_DEVICE;
      if (r == GM_OK && nc && hipMemcpyAsync(da, ha, 32 * nc, hipMemcpyHostToDevice, ctx->copy) != hipSuccess)
        r = GM_ERR_DEVICE;
      if (r == GM_OK && hipEventRecord(ev.a, ctx->copy) != hipSuccess) r = GM_ERR_DEVICE;
      copy_rc = r;
      queued = true;
    });
    return GM_OK;
  }
  int advance(bool block) {
    int rc;
    if (stage == 0) {
      if (!block && !queued.load()) return GM_OK;
      if (th.joinable()) th.join();
      if (copy_rc) {
        set_error("staged a upload failed");
        return copy_rc;
      }
      rc = on_aux(ctx, [&]() -> int {
        GM_HIP(hipStreamWaitEvent(ctx->stream, ev.a, 0));
        return compute_h_chain<C>(ctx, da, nc, pk->n);
      });
      if (rc) return rc;
      stage = 1;
    }
    if (stage == 1) {
      for (ChainDone* d : remote) {
        const int r = d->ready(block);
        if (r < 0) return r;
        if (r == 0) return GM_OK;  // not yet: a later poll
      }
      rc = on_aux(ctx, [&]() -> int {
        int r = compute_h_finish<C>(ctx, da, db, dc, pk->n);
        if (r) return r;
        GM_HIP(hipEventRecord(ev.b, ctx->stream));
        return GM_OK;
      });
      if (rc) return rc;
      stage = 2;
      if (after_h && (rc = after_h())) return rc;
    }
    return GM_OK;
  }
  int poll() override { return advance(false); }
  int z_scalars(const void** zs) override {
    int rc;
    if ((rc = advance(true))) return rc;
    GM_HIP(hipStreamWaitEvent(ctx->stream, ev.b, 0));
    *zs = (const char*)da + 32 * pk->zlo;
    return GM_OK;
  }
  ~SplitH() override {
    if (th.joinable()) th.join();
    hipStreamSynchronize(ctx->copy);
    hipStreamSynchronize(ctx->aux);
  }
};

template <class C>
struct G16Sums {
  typename C::HG1F A[3], B[3], K[3], Z[3];
  typename C::HG2F B2[3];
};

// The five MSM sums of one key (slice) on one device.  on_ab(A, B) runs on the
// host as soon as A and B are known (the prover starts the cross terms then).
template <class C>
int g16_sums_t(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, HSource& hs, G16Sums<C>& out,
               const std::function<void(const G16Sums<C>&)>& on_ab) {
  hipStream_t st = ctx->stream;
  int rc;
  Arena arena(ctx);
  const MsmPrecomp* pA = pk->precomp ? &pk->preA : nullptr;
  const MsmPrecomp* pB = pk->precomp ? &pk->preB : nullptr;
  const MsmPrecomp* pK = pk->precomp ? &pk->preK : nullptr;
  const MsmPrecomp* pZ = pk->precomp ? &pk->preZ : nullptr;
  const MsmPrecomp* pX[3] = {pA, pB, pK};
  const size_t nX[3] = {pk->nbA, pk->nbB, pk->nbK};
  const void* idxX[3] = {pk->idxA, pk->idxB, pk->idxK};
  // Scalars of the arrays with their own plan: device-side compaction
  // (icicle.go:231-278 do this on the host + H2D)
  DevBuf wX[3];
  {
    ProfScope ps(ctx, "gather_scalars");
    for (int x = 0; x < 3; x++) {
      if (pk->wshare[x]) continue;
      if ((rc = wX[x].alloc(arena, 32 * (nX[x] ? nX[x] : 1)))) return rc;
      if (nX[x])
        hipLaunchKernelGGL(k_gather_fr, dim3(blocks_for(nX[x], 256)), dim3(256), 0, st, (const uint4*)wires_dev,
                           (const uint32_t*)idxX[x], nX[x], (uint4*)wX[x].p);
    }
  }
  GM_HIP(hipGetLastError());
  // The shared wire plan: ONE digit / sort plan over the wire slice serves the
  // A, B, B2 and K MSMs of the wire-indexed arrays (pk_upload_ranges).
  MsmPlan planX[3];
  bool have[3] = {false, false, false};
  if (pk->wshare[0] || pk->wshare[1] || pk->wshare[2]) {
    MsmPlan planW;
    const MsmPrecomp* pW = pk->precomp ? &pk->preW : nullptr;
    if ((rc = msm_plan<C>(ctx, arena, wires_dev, pk->whi - pk->wlo, pW, planW))) return rc;
    for (int x = 0; x < 3; x++) {
      if (!pk->wshare[x]) continue;
      planX[x] = planW;  // the array is wire-indexed: the plan's entries address it directly
      have[x] = true;
    }
  }
  // launch array x's MSM into `slot`: on the shared plan, or plan + launch
  auto launch_x = [&](int x, Arena& slot, void* pts, MsmTail& t) -> int {
    if (have[x]) return msm_launch<C, false>(ctx, slot, planX[x], pts, t);
    return msm_device_launch<C, false>(ctx, slot, wX[x].p, pts, nX[x], true, pX[x], t);
  };
  // The five MSMs run pipelined two deep: the host tail of one (readback checks
  // and Horner, msm_finish) overlaps the device work of the next, each MSM in
  // one of the context's two slot arenas.  The G1 and G2 B-MSMs
  // (prove.go:217,293) share scalars and layout: one plan, in slot 1.
  // Slot 1's MSMs (B, B2, Z) queue on a second stream (GM_G16_MSM_STREAMS=1),
  // ordered after the plans / gathers: one MSM's bucket reduction (latency-bound,
  // one or two waves per SIMD) then runs beside the next one's accumulation
  // instead of before it.
  // (read per prove: the parity tests flip it).  The stream is the prove's own
  // (gm_ctx::g16_stream), not an async-MSM slot stream, so a pending
  // gm_msm_async never serialises the prove's MSMs behind it.
  const char* two_env = getenv("GM_G16_MSM_STREAMS");
  const bool two = two_env && atoi(two_env) != 0;
  hipStream_t st1 = st;
  if (two) {
    if (!ctx->g16_stream) GM_HIP(hipStreamCreateWithFlags(&ctx->g16_stream, hipStreamNonBlocking));
    st1 = ctx->g16_stream;
    hipEvent_t ev;
    GM_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const hipError_t e1 = hipEventRecord(ev, st);  // the gathers and the shared plan
    const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(st1, ev, 0) : e1;
    hipEventDestroy(ev);
    GM_HIP(e2);
  }
  SlotArena s0(ctx), s1(ctx);
  MsmTail tA, tB, tB2, tK, tZ;
  if ((rc = hs.poll()) || (rc = s0.take())) return rc;
  if ((rc = launch_x(0, *s0.a, pk->A, tA))) return rc;
  if ((rc = hs.poll()) || (rc = s1.take())) return rc;
  {
    StreamSwap sw(ctx, st1);
    if (!have[1]) {
      if ((rc = msm_plan<C>(ctx, *s1.a, wX[1].p, pk->nbB, pB, planX[1]))) return rc;
    }
    if ((rc = msm_launch<C, false>(ctx, *s1.a, planX[1], pk->B, tB))) return rc;
  }
  if ((rc = msm_finish<C, false>(ctx, tA, out.A))) return rc;
  s0.release();
  if ((rc = hs.poll())) return rc;
  {
    StreamSwap sw(ctx, st1);
    if ((rc = msm_launch<C, true>(ctx, *s1.a, planX[1], pk->B2, tB2)) ||
        (rc = msm_finish<C, false>(ctx, tB, out.B)))
      return rc;
  }
  if (on_ab) on_ab(out);
  if ((rc = hs.poll()) || (rc = s0.take())) return rc;
  if ((rc = launch_x(2, *s0.a, pk->K, tK))) return rc;
  {
    StreamSwap sw(ctx, st1);
    if ((rc = msm_finish<C, true>(ctx, tB2, out.B2))) return rc;
  }
  s1.release();
  const void* zs = nullptr;
  {
    StreamSwap sw(ctx, st1);  // Z waits for h on its own stream
    if ((rc = hs.z_scalars(&zs)) || (rc = s1.take())) return rc;
    if ((rc = msm_device_launch<C, false>(ctx, *s1.a, zs, pk->Z, pk->nbZ, true, pZ, tZ))) return rc;
  }
  if ((rc = msm_finish<C, false>(ctx, tK, out.K))) return rc;
  s0.release();
  StreamSwap sw(ctx, st1);
  return msm_finish<C, false>(ctx, tZ, out.Z);
}

// Host finishing of icicle.go:280-391 / prove.go:183-305 from the raw sums:
//   Ar  = A + alpha + [r]delta
//   Bs1 = B + beta + [s]delta
//   Krs = K + [-rs]delta + Z + [s]Ar + [r]Bs1
//   Bs  = B2 + [s]delta2 + beta2
// The four scalar multiplications that do not depend on the device results run
// on a host thread started before the MSMs (begin()); [s]Ar and [r]Bs1 on a
// second one as soon as A and B are known (cross()).
template <class C>
struct G16Finish {
  using HF1 = typename C::HG1F;
  using HF2 = typename C::HG2F;
  using HFr = typename C::HFr;
  using J1 = host::Jac<HF1>;
  using J2 = host::Jac<HF2>;
  host::Aff<HF1> alpha, beta, delta;
  host::Aff<HF2> beta2, delta2;
  host::F<HFr> rc_, sc_, krc;
  J1 d0, d1, d2, ar, bs1, s_ar, r_bs1;
  J2 sd2;
  std::thread t_deltas, t_cross;

  G16Finish(const uint8_t* alpha_, const uint8_t* beta_, const uint8_t* delta_, const uint8_t* beta2_,
            const uint8_t* delta2_, const void* r_mont, const void* s_mont) {
    memcpy(&alpha, alpha_, sizeof(alpha));
    memcpy(&beta, beta_, sizeof(beta));
    memcpy(&delta, delta_, sizeof(delta));
    memcpy(&beta2, beta2_, sizeof(beta2));
    memcpy(&delta2, delta2_, sizeof(delta2));
    host::F<HFr> r, s;
    memcpy(r.v, r_mont, 32);
    memcpy(s.v, s_mont, 32);
    const host::F<HFr> kr = -(r * s);  // _kr = -(r s) (prove.go:189)
    rc_ = host::from_mont(r);
    sc_ = host::from_mont(s);
    krc = host::from_mont(kr);
  }
  // [r]delta, [s]delta, [kr]delta (BatchScalarMultiplicationG1, prove.go:195), [s]delta2
  void begin() {
    t_deltas = std::thread([this] {
      const J1 dj = host::to_jac(delta);
      d0 = host::jmul(dj, rc_.v, 4);
      d1 = host::jmul(dj, sc_.v, 4);
      d2 = host::jmul(dj, krc.v, 4);
      sd2 = host::jmul(host::to_jac(delta2), sc_.v, 4);
    });
  }
  void cross(const HF1 (&A)[3], const HF1 (&B)[3]) {
    if (t_deltas.joinable()) t_deltas.join();
    ar = host::jadd(host::jadd_aff(J1{A[0], A[1], A[2]}, alpha), d0);
    bs1 = host::jadd(host::jadd_aff(J1{B[0], B[1], B[2]}, beta), d1);
    t_cross = std::thread([this] {
      s_ar = host::jmul(ar, sc_.v, 4);
      r_bs1 = host::jmul(bs1, rc_.v, 4);
    });
  }
  void join() {
    if (t_deltas.joinable()) t_deltas.join();
    if (t_cross.joinable()) t_cross.join();
  }
  void finish(const G16Sums<C>& s, void* ar_out, void* bs_out, void* krs_out) {
    if (!t_cross.joinable() && !crossed) cross(s.A, s.B);
    join();
    J1 krs = host::jadd(J1{s.K[0], s.K[1], s.K[2]}, d2);
    krs = host::jadd(krs, J1{s.Z[0], s.Z[1], s.Z[2]});
    krs = host::jadd(krs, s_ar);
    krs = host::jadd(krs, r_bs1);
    J2 bs = host::jadd(J2{s.B2[0], s.B2[1], s.B2[2]}, sd2);
    bs = host::jadd_aff(bs, beta2);
    const host::Aff<HF1> ara = host::to_aff(ar), krsa = host::to_aff(krs);
    const host::Aff<HF2> bsa = host::to_aff(bs);
    memcpy(ar_out, &ara, sizeof(ara));
    memcpy(krs_out, &krsa, sizeof(krsa));
    memcpy(bs_out, &bsa, sizeof(bsa));
  }
  bool crossed = false;
  ~G16Finish() { join(); }
};

template <class C>
G16Finish<C>* make_finish(const gm_g16_pk* pk, const void* r, const void* s) {
  return new G16Finish<C>(pk->alpha.data(), pk->beta.data(), pk->delta.data(), pk->beta2.data(), pk->delta2.data(),
                          r, s);
}

// One device, whole key.  host_abc: a, b, c are host pointers staged on the copy
// stream; else device buffers (queued on the main stream).
template <class C>
int g16_prove_t(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a, void* b, void* c, const void* ha,
                const void* hb, const void* hc, size_t nc, const void* r, const void* s, void* ar_out, void* bs_out,
                void* krs_out, const gm_r1cs* r1 = nullptr) {
  std::unique_ptr<G16Finish<C>> fin(make_finish<C>(pk, r, s));
  fin->begin();
  std::unique_ptr<HSource> hs;
  int rc;
  if (ha) {
    auto* x = new HostStagedH<C>(ctx, pk, a, b, c, ha, hb, hc, nc);
    hs.reset(x);
    rc = x->start();
  } else {
    auto* x = new DeviceH<C>(ctx, pk, a, b, c, nc);
    x->r1 = r1;
    x->wires = wires_dev;
    hs.reset(x);
    rc = x->start();
  }
  if (rc) return rc;
  G16Sums<C> sums;
  auto on_ab = [&](const G16Sums<C>& sm) {
    fin->cross(sm.A, sm.B);
    fin->crossed = true;
  };
  if ((rc = g16_sums_t<C>(ctx, pk, wires_dev, *hs, sums, on_ab))) return rc;
  fin->finish(sums, ar_out, bs_out, krs_out);
  return GM_OK;
}

template <class C>
void sums_to_bytes(const G16Sums<C>& s, uint8_t* out) {
  constexpr size_t J1 = sizeof(s.A);
  memcpy(out, s.A, J1);
  memcpy(out + J1, s.B, J1);
  memcpy(out + 2 * J1, s.K, J1);
  memcpy(out + 3 * J1, s.Z, J1);
  memcpy(out + 4 * J1, s.B2, sizeof(s.B2));
}
template <class C>
void bytes_to_sums(const uint8_t* in, G16Sums<C>& s) {
  constexpr size_t J1 = sizeof(s.A);
  memcpy(s.A, in, J1);
  memcpy(s.B, in + J1, J1);
  memcpy(s.K, in + 2 * J1, J1);
  memcpy(s.Z, in + 3 * J1, J1);
  memcpy(s.B2, in + 4 * J1, sizeof(s.B2));
}
template <class C>
void add_sums(G16Sums<C>& acc, const G16Sums<C>& x) {
  using J1 = host::Jac<typename C::HG1F>;
  using J2 = host::Jac<typename C::HG2F>;
  auto add1 = [](typename C::HG1F (&a)[3], const typename C::HG1F (&b)[3]) {
    const J1 r = host::jadd(J1{a[0], a[1], a[2]}, J1{b[0], b[1], b[2]});
    a[0] = r.x;
    a[1] = r.y;
    a[2] = r.z;
  };
  add1(acc.A, x.A);
  add1(acc.B, x.B);
  add1(acc.K, x.K);
  add1(acc.Z, x.Z);
  const J2 r = host::jadd(J2{acc.B2[0], acc.B2[1], acc.B2[2]}, J2{x.B2[0], x.B2[1], x.B2[2]});
  acc.B2[0] = r.x;
  acc.B2[1] = r.y;
  acc.B2[2] = r.z;
}

}  // namespace
}  // namespace gm

// ===========================================================================
// single-device C-ABI
// ===========================================================================
extern "C" {

int gm_g16_pk_upload(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, gm_g16_pk** out) {
  return gm_g16_pk_upload_ex(ctx, curve, h, 0u, out);
}

int gm_g16_pk_upload_ex(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, unsigned flags, gm_g16_pk** out) {
  return gm_g16_pk_upload_shard(ctx, curve, h, flags, 0, 1, out);
}

int gm_g16_pk_upload_shard(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, unsigned flags, int rank, int world,
                           gm_g16_pk** out) {
  if (int rc = check_curve_id(curve)) return rc;
  if (flags & ~(unsigned)(GM_PK_PRECOMPUTE | GM_PK_PRECOMPUTE_AUTO)) {
    set_error("pk upload: unknown flags");
    return GM_ERR_INVALID;
  }
  if (!ctx || !h || !out || h->domain_size < 2) return GM_ERR_INVALID;
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("pk upload: bad rank / world");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  Ranges rg;
  shard_of(h->nbA, rank, world, &rg.loA, &rg.hiA);
  shard_of(h->nbB, rank, world, &rg.loB, &rg.hiB);
  shard_of(h->nbK, rank, world, &rg.loK, &rg.hiK);
  shard_of(h->domain_size - 1, rank, world, &rg.loZ, &rg.hiZ);
  rg.rebase = false;
  return pk_upload_ranges(ctx, curve, h, flags, rg, out, nullptr);
}

int gm_g16_pk_precomputed(const gm_g16_pk* pk, int* out) {
  if (!pk || !out) return GM_ERR_INVALID;
  *out = pk->precomp ? 1 : 0;
  return GM_OK;
}

int gm_g16_pk_free(gm_ctx* ctx, gm_g16_pk* pk) {
  if (!pk) return GM_OK;
  gm::CtxLock g(ctx);
  hipSetDevice(ctx->device);
  pk_release(pk);
  return GM_OK;
}

int gm_g16_prove_device(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a, void* b, void* c, size_t nc,
                        const void* r, const void* s, void* ar_out, void* bs_out, void* krs_out) {
  if (!ctx || !pk || !r || !s || !ar_out || !bs_out || !krs_out) return GM_ERR_INVALID;
  if (nc > pk->n) {
    set_error("prove: more constraints than the domain size");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = pk->curve == GM_BN254 ? g16_prove_t<CurveBN254>(ctx, pk, wires_dev, a, b, c, nullptr, nullptr, nullptr,
                                                           nc, r, s, ar_out, bs_out, krs_out)
                                 : g16_prove_t<CurveBLS12377>(ctx, pk, wires_dev, a, b, c, nullptr, nullptr, nullptr,
                                                              nc, r, s, ar_out, bs_out, krs_out);
  prof_collect(ctx);
  return rc;
}

// Host inputs (the icicle.go:204-412 scope, H2D included): the wires are
// copied first (every MSM needs them), a / b / c on the copy stream by a helper
// thread while the A/B/K MSMs run.
int gm_g16_prove(gm_ctx* ctx, gm_g16_pk* pk, const void* wires, const void* a, const void* b, const void* c,
                 size_t nc, const void* r, const void* s, void* ar_out, void* bs_out, void* krs_out) {
  if (!ctx || !pk || !wires || !a || !b || !c || !r || !s || !ar_out || !bs_out || !krs_out) return GM_ERR_INVALID;
  if (nc > pk->n) {
    set_error("prove: more constraints than the domain size");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  Arena arena(ctx);
  DevBuf w;
  int rc;
  if ((rc = w.alloc(arena, 32 * pk->nb_wires))) return rc;
  // a / b / c: the context's input allocation (gm_ctx::in_abc), not the arena
  if ((rc = in_abc_reserve(ctx, pk->n))) return rc;
  char* const da = (char*)ctx->in_abc;
  char* const db = da + 32 * pk->n;
  char* const dc = db + 32 * pk->n;
  GM_HIP(hipMemcpyAsync(w.p, wires, 32 * pk->nb_wires, hipMemcpyHostToDevice, ctx->stream));
  rc = pk->curve == GM_BN254 ? g16_prove_t<CurveBN254>(ctx, pk, w.p, da, db, dc, a, b, c, nc, r, s, ar_out,
                                                       bs_out, krs_out)
                             : g16_prove_t<CurveBLS12377>(ctx, pk, w.p, da, db, dc, a, b, c, nc, r, s, ar_out,
                                                          bs_out, krs_out);
  prof_collect(ctx);
  return rc;
}

// Wires alone in host memory, the R1CS resident (gm_r1cs_upload): the wires
// are copied, a / b / c evaluated on the device (auxiliary stream, ahead of
// computeH) while the A/B/K MSMs run on the main stream.
}  // extern "C"

// Proof from device-resident wires and a device-resident R1CS: a, b, c are
// evaluated into the caller's n-element buffers (gm_g16_prove_r1cs, staged
// wires: gm_g16_stage_prove_r1cs).  The key / system match is checked by the callers.
int gm::g16_prove_r1cs_device(gm_ctx* ctx, gm_g16_pk* pk, const gm_r1cs* r1, const void* wires_dev, void* a,
                              void* b, void* c, const void* r, const void* s, void* ar_out, void* bs_out,
                              void* krs_out) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  const size_t nc = r1cs_nb_constraints(r1);
  int rc = pk->curve == GM_BN254
               ? g16_prove_t<CurveBN254>(ctx, pk, wires_dev, a, b, c, nullptr, nullptr, nullptr, nc, r, s, ar_out,
                                         bs_out, krs_out, r1)
               : g16_prove_t<CurveBLS12377>(ctx, pk, wires_dev, a, b, c, nullptr, nullptr, nullptr, nc, r, s,
                                            ar_out, bs_out, krs_out, r1);
  prof_collect(ctx);
  return rc;
}

bool gm::r1cs_matches_key(const gm_g16_pk* pk, const gm_r1cs* r1) {
  return r1cs_nb_constraints(r1) <= pk->n && r1cs_nb_wires(r1) == pk->nb_wires && pk->wlo == 0 &&
         pk->whi == pk->nb_wires;
}

extern "C" {

int gm_g16_prove_r1cs(gm_ctx* ctx, gm_g16_pk* pk, const gm_r1cs* r1, const void* wires, const void* r,
                      const void* s, void* ar_out, void* bs_out, void* krs_out) {
  if (!ctx || !pk || !r1 || !wires || !r || !s || !ar_out || !bs_out || !krs_out) return GM_ERR_INVALID;
  if (!r1cs_matches_key(pk, r1)) {
    set_error("prove_r1cs: constraint system does not match the proving key (constraints <= n, same wires, "
              "whole key)");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  Arena arena(ctx);
  DevBuf w, da, db, dc;
  int rc;
  if ((rc = w.alloc(arena, 32 * pk->nb_wires)) || (rc = da.alloc(arena, 32 * pk->n)) ||
      (rc = db.alloc(arena, 32 * pk->n)) || (rc = dc.alloc(arena, 32 * pk->n)))
    return rc;
  GM_HIP(hipMemcpyAsync(w.p, wires, 32 * pk->nb_wires, hipMemcpyHostToDevice, ctx->stream));
  return gm::g16_prove_r1cs_device(ctx, pk, r1, w.p, da.p, db.p, dc.p, r, s, ar_out, bs_out, krs_out);
}

// ---- sharded Groth16 (one process per GPU) --------------------
int gm_g16_partial_bytes(int curve, size_t* out) {
  if (int rc = check_curve_id(curve)) return rc;
  if (out) *out = 4 * 3 * fp_bytes(curve) + 3 * 2 * fp_bytes(curve);
  return GM_OK;
}

int gm_g16_prove_partial(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a_dev, void* b_dev, void* c_dev,
                         size_t nc, void* partial_out) {
  if (!ctx || !pk || !partial_out) return GM_ERR_INVALID;
  if (nc > pk->n) {
    set_error("prove: more constraints than the domain size");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  auto run = [&](auto tag) -> int {
    using C = decltype(tag);
    DeviceH<C> hs(ctx, pk, a_dev, b_dev, c_dev, nc);
    int rc;
    if ((rc = hs.start())) return rc;
    G16Sums<C> sums;
    if ((rc = g16_sums_t<C>(ctx, pk, wires_dev, hs, sums, nullptr))) return rc;
    sums_to_bytes<C>(sums, (uint8_t*)partial_out);
    return GM_OK;
  };
  int rc = pk->curve == GM_BN254 ? run(CurveBN254()) : run(CurveBLS12377());
  prof_collect(ctx);
  return rc;
}

int gm_g16_finish(int curve, const gm_g16_pk_host* h, const void* sums, const void* r, const void* s, void* ar_out,
                  void* bs_out, void* krs_out) {
  if (int rc = check_curve_id(curve)) return rc;
  if (!h || !sums || !r || !s || !ar_out || !bs_out || !krs_out) return GM_ERR_INVALID;
  auto run = [&](auto tag) {
    using C = decltype(tag);
    G16Finish<C> fin((const uint8_t*)h->g1_alpha, (const uint8_t*)h->g1_beta, (const uint8_t*)h->g1_delta,
                     (const uint8_t*)h->g2_beta, (const uint8_t*)h->g2_delta, r, s);
    fin.begin();
    G16Sums<C> sm;
    bytes_to_sums<C>((const uint8_t*)sums, sm);
    fin.finish(sm, ar_out, bs_out, krs_out);
  };
  if (curve == GM_BN254) run(CurveBN254());
  else run(CurveBLS12377());
  return GM_OK;
}

}  // extern "C"

// ===========================================================================
// single-process multi-device C-ABI (gm_multi)
// ===========================================================================
struct gm_multi {
  std::vector<gm_ctx*> ctx;
};

struct gm_g16_pk_multi {
  int curve;
  std::vector<gm_g16_pk*> pk;  // pk[d] on ctx[d]
};

extern "C" {

int gm_multi_init(const int* device_ids, int count, gm_multi** out) {
  if (!device_ids || count < 1 || !out) return GM_ERR_INVALID;
  auto* m = new gm_multi();
  for (int d = 0; d < count; d++) {
    gm_ctx* c = nullptr;
    if (int rc = gm_init(device_ids[d], &c)) {
      for (gm_ctx* x : m->ctx) gm_destroy(x);
      delete m;
      return rc;
    }
    m->ctx.push_back(c);
  }
  // direct xGMI copies device 0 -> d for the h slices (ignored when unsupported:
  // HIP then stages peer copies itself)
  for (int d = 1; d < count; d++) {
    const int d0 = device_ids[0], dd = device_ids[d];
    if (dd == d0) continue;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, dd, d0) == hipSuccess && can) {
      hipSetDevice(dd);
      hipDeviceEnablePeerAccess(d0, 0);
      hipSetDevice(d0);
      hipDeviceEnablePeerAccess(dd, 0);
      (void)hipGetLastError();
    }
  }
  *out = m;
  return GM_OK;
}

int gm_multi_destroy(gm_multi* m) {
  if (!m) return GM_OK;
  for (gm_ctx* c : m->ctx) gm_destroy(c);
  delete m;
  return GM_OK;
}

int gm_multi_size(const gm_multi* m, int* count) {
  if (!m || !count) return GM_ERR_INVALID;
  *count = (int)m->ctx.size();
  return GM_OK;
}

int gm_multi_context(gm_multi* m, int index, gm_ctx** out) {
  if (!m || !out || index < 0 || index >= (int)m->ctx.size()) return GM_ERR_INVALID;
  *out = m->ctx[index];
  return GM_OK;
}

int gm_g16_pk_upload_multi(gm_multi* m, int curve, const gm_g16_pk_host* h, unsigned flags, gm_g16_pk_multi** out) {
  if (!m || !h || !out || h->domain_size < 2) return GM_ERR_INVALID;
  if (int rc = check_curve_id(curve)) return rc;
  const int nd = (int)m->ctx.size();
  // device 0 also runs computeH (~19 ms at 2^24): it takes a smaller share of
  // the MSM work (GM_MULTI_SHARE0 = its weight relative to the others' 1.0)
  // devices 0-2 also run computeH (split: one a / b / c chain each, device 0
  // the tail and the h distribution; ~5 ms per chain, ~2.5 ms tail at 2^24):
  // they take smaller MSM shares (weights relative to the others' 1.0; an
  // estimate from the one-GPU timeline)
  std::vector<double> w(nd, 1.0);
  if (nd > 1) {
    w[0] = 0.7;
    for (int d = 1; d < std::min(nd, 3); d++) w[d] = 0.85;
  }
  auto* mp = new gm_g16_pk_multi();
  mp->curve = curve;
  mp->pk.assign(nd, nullptr);
  std::vector<int> rcs(nd, GM_OK);
  std::vector<std::string> errs(nd);
  std::vector<std::thread> th;
  for (int d = 0; d < nd; d++) {
    th.emplace_back([&, d] {
      gm_ctx* ctx = m->ctx[d];
      gm::CtxLock g(ctx);
      if (hipSetDevice(ctx->device) != hipSuccess) {
        rcs[d] = GM_ERR_DEVICE;
        errs[d] = "hipSetDevice failed";
        return;
      }
      Ranges rg;
      shard_weighted(h->nbA, w, d, &rg.loA, &rg.hiA);
      shard_weighted(h->nbB, w, d, &rg.loB, &rg.hiB);
      shard_weighted(h->nbK, w, d, &rg.loK, &rg.hiK);
      shard_weighted(h->domain_size - 1, w, d, &rg.loZ, &rg.hiZ);
      rg.rebase = true;
      gm_g16_pk_host hs = *h;
      const size_t g1b = 2 * fp_bytes(curve), g2b = 4 * fp_bytes(curve);
      hs.g1_A = (const uint8_t*)h->g1_A + g1b * rg.loA;
      hs.g1_B = (const uint8_t*)h->g1_B + g1b * rg.loB;
      hs.g1_K = (const uint8_t*)h->g1_K + g1b * rg.loK;
      hs.g1_Z = (const uint8_t*)h->g1_Z + g1b * rg.loZ;
      hs.g2_B = (const uint8_t*)h->g2_B + g2b * rg.loB;
      rcs[d] = pk_upload_ranges(ctx, curve, &hs, flags, rg, &mp->pk[d], nullptr);
      if (rcs[d]) errs[d] = gm_last_error();
    });
  }
  for (auto& t : th) t.join();
  for (int d = 0; d < nd; d++)
    if (rcs[d]) {
      set_error("device " + std::to_string(d) + ": " + errs[d]);
      for (int e = 0; e < nd; e++)
        if (mp->pk[e]) gm_g16_pk_free(m->ctx[e], mp->pk[e]);
      delete mp;
      return rcs[d];
    }
  *out = mp;
  return GM_OK;
}

int gm_g16_pk_free_multi(gm_multi* m, gm_g16_pk_multi* mp) {
  if (!m || !mp) return GM_OK;
  for (size_t d = 0; d < mp->pk.size() && d < m->ctx.size(); d++)
    if (mp->pk[d]) gm_g16_pk_free(m->ctx[d], mp->pk[d]);
  delete mp;
  return GM_OK;
}

}  // extern "C"

namespace gm {
namespace {

// All devices of `m` prove one proof: device d uploads only the wires its key
// slices read ([wlo, whi)), runs its A/B/B2/K MSMs; device 0 additionally gets
// a / b / c, runs computeH and copies each device's slice of h to it (xGMI peer
// copies); every device then runs its Z slice.  The per-device sums are added
// and finished on the host.
template <class C>
int g16_prove_multi_t(gm_multi* m, gm_g16_pk_multi* mp, const uint8_t* wires, const void* ha, const void* hb,
                      const void* hc, size_t nc, const void* r, const void* s, void* ar_out, void* bs_out,
                      void* krs_out) {
  const int nd = (int)m->ctx.size();
  gm_g16_pk* pk0 = mp->pk[0];
  std::unique_ptr<G16Finish<C>> fin(make_finish<C>(pk0, r, s));
  fin->begin();
  SharedH sh;
  std::vector<G16Sums<C>> sums(nd);
  std::vector<int> rcs(nd, GM_OK);
  std::vector<std::string> errs(nd);
  // per-device h slice buffers, allocated up front so device 0 can address them
  std::vector<std::unique_ptr<Arena>> arenas;
  std::vector<void*> hz(nd, nullptr);
  for (int d = 0; d < nd; d++) {
    gm_ctx* ctx = m->ctx[d];
    GM_HIP(hipSetDevice(ctx->device));
    arenas.emplace_back(new Arena(ctx));
    if (d > 0) {
      DevBuf b;
      if (int rc = b.alloc(*arenas[d], 32 * (mp->pk[d]->nbZ ? mp->pk[d]->nbZ : 1))) return rc;
      hz[d] = b.p;
    }
  }
  // device 0's b / c buffers (peer-copy targets of the chains on devices 1, 2;
  // one device: its own staged b, c)
  void* d0bc[2] = {nullptr, nullptr};
  const bool split = nd >= 2;
  {
    GM_HIP(hipSetDevice(m->ctx[0]->device));
    DevBuf b, c;
    const size_t n = mp->pk[0]->n;
    if (int rc = b.alloc(*arenas[0], 32 * n)) return rc;
    if (int rc = c.alloc(*arenas[0], 32 * n)) return rc;
    d0bc[0] = b.p;
    d0bc[1] = c.p;
  }
  // chain placement: b on device 1, c on device 2 (device 1 with two devices)
  ChainDone chain_done[2];
  const int chain_dev[2] = {split ? 1 : -1, nd >= 3 ? 2 : (split ? 1 : -1)};
  for (int k = 0; k < 2 && split; k++) {
    GM_HIP(hipSetDevice(m->ctx[chain_dev[k]]->device));
    GM_HIP(hipEventCreateWithFlags(&chain_done[k].ev, hipEventDisableTiming));
  }
  struct EvFree {
    ChainDone* cd;
    ~EvFree() {
      for (int k = 0; k < 2; k++)
        if (cd[k].ev) hipEventDestroy(cd[k].ev);
    }
  } ev_free{chain_done};
  EventPair dist;
  GM_HIP(hipSetDevice(m->ctx[0]->device));
  if (int rc = dist.create()) return rc;
  sh.done = dist.a;
  auto worker = [&](int d) {
    gm_ctx* ctx = m->ctx[d];
    gm_g16_pk* pk = mp->pk[d];
    auto fail = [&](int rc) {
      rcs[d] = rc;
      errs[d] = gm_last_error();
      if (d == 0) {
        std::lock_guard<std::mutex> lk(sh.mu);
        if (!sh.ready) {
          sh.ready = true;
          sh.rc = rc;
          sh.cv.notify_all();
        }
      }
    };
    gm::CtxLock g(ctx);
    if (hipSetDevice(ctx->device) != hipSuccess) {
      if (d == chain_dev[0]) chain_done[0].signal(GM_ERR_DEVICE);
      if (d == chain_dev[1]) chain_done[1].signal(GM_ERR_DEVICE);
      return fail(GM_ERR_DEVICE);
    }
    Arena arena(ctx);
    DevBuf w, da;
    const size_t nw = pk->whi - pk->wlo;
    int rc;
    // a device that owns a chain must signal it even when it fails early
    std::unique_ptr<HSource> hs;
    if (d > 0) {
      auto* x = new ChainRemoteH<C>(&sh, hz[d], ctx, m->ctx[0]->device, nc, pk->n);
      const void* hv[2] = {hb, hc};
      for (int k = 0; k < 2; k++) {
        if (chain_dev[k] != d) continue;
        DevBuf loc;
        if ((rc = loc.alloc(arena, 32 * pk->n))) {
          chain_done[k].signal(rc);
          continue;
        }
        x->jobs.push_back({hv[k], loc.p, d0bc[k], &chain_done[k]});
      }
      hs.reset(x);
      if (!x->jobs.empty() && (rc = x->start())) return fail(rc);
    }
    if ((rc = w.alloc(arena, 32 * (nw ? nw : 1)))) return fail(rc);
    if (nw && hipMemcpyAsync(w.p, wires + 32 * pk->wlo, 32 * nw, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
      return fail(GM_ERR_DEVICE);
    if (d == 0 && !split) {  // one device: computeH whole, inputs staged from the host
      if ((rc = da.alloc(arena, 32 * pk->n))) return fail(rc);
      auto* x = new HostStagedH<C>(ctx, pk, da.p, d0bc[0], d0bc[1], ha, hb, hc, nc);
      hs.reset(x);
      x->after_h = [&]() -> int {
        GM_HIP(hipEventRecord(sh.done, ctx->aux));
        std::lock_guard<std::mutex> lk(sh.mu);
        sh.ready = true;
        sh.cv.notify_all();
        return GM_OK;
      };
      if ((rc = x->start())) return fail(rc);
    } else if (d == 0) {
      if ((rc = da.alloc(arena, 32 * pk->n))) return fail(rc);
      auto* x = new SplitH<C>(ctx, pk, da.p, d0bc[0], d0bc[1], ha, nc);
      x->remote = {&chain_done[0], &chain_done[1]};
      hs.reset(x);
      x->after_h = [&, x]() -> int {
        // h is produced on ctx0->aux after x->ev.b: copy the slices there too
        for (int e = 1; e < nd; e++) {
          gm_g16_pk* pe = mp->pk[e];
          if (!pe->nbZ) continue;
          const void* src = (const char*)x->da + 32 * pe->zlo;
          const int dev_e = m->ctx[e]->device;
          if (!cross_device(dev_e, ctx->device))
            GM_HIP(hipMemcpyAsync(hz[e], src, 32 * pe->nbZ, hipMemcpyDeviceToDevice, ctx->aux));
          else
            GM_HIP(hipMemcpyPeerAsync(hz[e], dev_e, src, ctx->device, 32 * pe->nbZ, ctx->aux));
        }
        GM_HIP(hipEventRecord(sh.done, ctx->aux));
        std::lock_guard<std::mutex> lk(sh.mu);
        sh.ready = true;
        sh.cv.notify_all();
        return GM_OK;
      };
      if ((rc = x->start())) return fail(rc);
    }
    if ((rc = g16_sums_t<C>(ctx, pk, w.p, *hs, sums[d], nullptr))) return fail(rc);
    if (d == 0) {
      // make sure h was produced (and distributed) even if device 0 has no Z slice
      const void* zs;
      if ((rc = hs->z_scalars(&zs))) return fail(rc);
    }
  };
  std::vector<std::thread> th;
  for (int d = 0; d < nd; d++) th.emplace_back(worker, d);
  for (auto& t : th) t.join();
  for (int d = 0; d < nd; d++) {
    hipSetDevice(m->ctx[d]->device);
    hipStreamSynchronize(m->ctx[d]->aux);
    hipStreamSynchronize(m->ctx[d]->copy);
  }
  for (int d = 0; d < nd; d++)
    if (rcs[d]) {
      set_error("device " + std::to_string(d) + ": " + errs[d]);
      return rcs[d];
    }
  G16Sums<C> tot = sums[0];
  for (int d = 1; d < nd; d++) add_sums<C>(tot, sums[d]);
  fin->finish(tot, ar_out, bs_out, krs_out);
  // release the h slice buffers in LIFO order
  while (!arenas.empty()) arenas.pop_back();
  return GM_OK;
}

}  // namespace
}  // namespace gm

extern "C" {

int gm_g16_prove_multi(gm_multi* m, gm_g16_pk_multi* mp, const void* wires, const void* a, const void* b,
                       const void* c, size_t nc, const void* r, const void* s, void* ar_out, void* bs_out,
                       void* krs_out) {
  if (!m || !mp || !wires || !a || !b || !c || !r || !s || !ar_out || !bs_out || !krs_out) return GM_ERR_INVALID;
  if (mp->pk.size() != m->ctx.size()) {
    set_error("prove_multi: key uploaded to a different device set");
    return GM_ERR_INVALID;
  }
  if (nc > mp->pk[0]->n) {
    set_error("prove: more constraints than the domain size");
    return GM_ERR_INVALID;
  }
  int rc = mp->curve == GM_BN254
               ? g16_prove_multi_t<CurveBN254>(m, mp, (const uint8_t*)wires, a, b, c, nc, r, s, ar_out, bs_out, krs_out)
               : g16_prove_multi_t<CurveBLS12377>(m, mp, (const uint8_t*)wires, a, b, c, nc, r, s, ar_out, bs_out,
                                                  krs_out);
  for (gm_ctx* x : m->ctx) prof_collect(x);
  return rc;
}

}  // extern "C"
