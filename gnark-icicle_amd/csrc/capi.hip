// C-ABI implementation (include/gnark_mi355x.h): context, memory, MSM, KZG,
// NTT / computeH, host group helpers and synthetic inputs.  The Groth16 prover
// entry points live in groth16.hip.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <string>
#include <vector>

#include "curves.hpp"
#include "groth16.hpp"
#include "msm.hpp"
#include "ntt.hpp"
#include "runtime.hpp"

namespace gm {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
std::string last_error() { return g_last_error; }

// ---------------------------------------------------------------------------
// synthetic-input kernels (bench / tests)
// ---------------------------------------------------------------------------
GM_DEV uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// n Montgomery (gnark-layout) scalars: random canonical value below 2^BITS,
// reduced once (2^BITS < 2r for both scalar fields), then x*Rg.
template <class Fr>
__global__ void k_random_scalars(uint32_t* out, size_t n, uint64_t seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t st = seed ^ (0xD1B54A32D192ED03ull * (i + 1));
  FeG<Fr> g;
  for (int q = 0; q < Fr::NG / 2; q++) {
    uint64_t v = splitmix64(st);
    g.w[2 * q] = (uint32_t)v;
    g.w[2 * q + 1] = (uint32_t)(v >> 32);
  }
  const int top = Fr::BITS - 32 * (Fr::NG - 1);
  g.w[Fr::NG - 1] &= (top >= 32) ? 0xffffffffu : ((1u << top) - 1);
  Fe<Fr> k = fe_unpack<Fr>(g);
  fe_reduce_once(k);
  feg_store<Fr>(out + i * Fr::NG, fe_pack(fe_canonical_to_gnark(k)));
}

// gnark-layout affine point passed by value
template <class F>
struct GPoint {
  uint32_t w[2 * Coord<F>::WORDS];
};

// out[i] = [k_i] base (gnark-layout affine), double-and-add over the canonical scalar.
template <class Fr, class F>
__global__ void __launch_bounds__(128) k_batch_mul_base(const uint32_t* __restrict__ scalars,
                                                        size_t n, GPoint<F> base_g,
                                                        uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const FeG<Fr> k = fe_pack(fe_gnark_to_canonical(fe_load_g<Fr>(scalars, i)));
  const Affine<F> base = load_affine_gnark<F>(base_g.w);
  XYZZ<F> acc = xyzz_inf<F>();
  for (int w = Fr::NG - 1; w >= 0; w--) {
    for (int b = 31; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      if ((k.w[w] >> b) & 1) xyzz_add_aff(acc, base);
    }
  }
  Affine<F> r;
  if (xyzz_is_inf(acc)) {
    r.x = FOps<F>::zero();
    r.y = FOps<F>::zero();
  } else {
    F t = fe_inv(fe_mul(acc.zz, acc.zzz));
    r.x = fe_mul(acc.x, fe_mul(t, acc.zzz));  // X / ZZ
    r.y = fe_mul(acc.y, fe_mul(t, acc.zz));   // Y / ZZZ
  }
  store_affine_gnark<F>(out + i * 2 * Coord<F>::WORDS, r);
}

// ---------------------------------------------------------------------------
// dispatch helpers
// ---------------------------------------------------------------------------
template <class C, bool G2>
static int msm_to_host(gm_ctx* ctx, const void* sc, const void* pts, size_t n, void* out_jac,
                       void* out_aff) {
  using HF = typename GroupSel<C, G2>::HF;
  HF j[3];
  int rc = msm_device<C, G2>(ctx, sc, pts, n, j);
  if (rc) return rc;
  if (out_jac) memcpy(out_jac, j, sizeof(j));
  if (out_aff) {
    host::Aff<HF> a = host::to_aff(host::Jac<HF>{j[0], j[1], j[2]});
    memcpy(out_aff, &a, sizeof(a));
  }
  return GM_OK;
}

static int check_curve(int curve) {
  if (curve != GM_BN254 && curve != GM_BLS12_377) {
    set_error("unknown curve id");
    return GM_ERR_INVALID;
  }
  return GM_OK;
}

size_t fp_bytes(int curve) { return curve == GM_BN254 ? 32 : 48; }

void orphan_pending_msms(gm_ctx* ctx);  // below gm_msm_pending

}  // namespace gm

using namespace gm;

extern "C" {

const char* gm_last_error(void) { return g_last_error.c_str(); }
int gm_version(void) { return 2; }

int gm_device_count(int* count) {
  if (!count) return GM_ERR_INVALID;
  GM_HIP(hipGetDeviceCount(count));
  return GM_OK;
}

int gm_init(int device, gm_ctx** out) {
  if (!out) return GM_ERR_INVALID;
  int ndev = 0;
  GM_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("gm_init: device index out of range");
    return GM_ERR_INVALID;
  }
  GM_HIP(hipSetDevice(device));
  auto* c = new gm_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking);
  if (e != hipSuccess) {
    set_error(std::string("hipStreamCreate: ") + hipGetErrorString(e));
    delete c;
    return GM_ERR_DEVICE;
  }
  *out = c;
  return GM_OK;
}

int gm_destroy(gm_ctx* ctx) {
  if (!ctx) return GM_OK;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  if (ctx->aux) hipStreamSynchronize(ctx->aux);
  if (ctx->copy) hipStreamSynchronize(ctx->copy);
  for (hipStream_t s : ctx->slot_stream)
    if (s) hipStreamSynchronize(s);
  if (ctx->g16_stream) hipStreamSynchronize(ctx->g16_stream);
  orphan_pending_msms(ctx);
  // stages parked with keys of this context (their keys may outlive it)
  while (!ctx->spare_keys.empty()) stage_spare_release(ctx->spare_keys.back());
  for (auto& pr : ctx->pending_reads) hipEventDestroy(pr.second);
  ctx->pending_reads.clear();
  ntt_domains_free(ctx);
  std::vector<gm::ArenaState*> arenas{&ctx->arena};
  for (gm::ArenaState& sa : ctx->slots) arenas.push_back(&sa);
  for (gm::ArenaState* a : arenas) {
    for (auto& ch : a->chunks) hipFree(ch.base);
    a->chunks.clear();
  }
  for (void* p : ctx->tail_pinned)
    if (p) hipHostFree(p);
  for (auto e : ctx->event_pool) hipEventDestroy(e);
  for (auto& p : ctx->pending) {
    hipEventDestroy(p.a);
    hipEventDestroy(p.b);
  }
  for (hipStream_t s : ctx->slot_stream)
    if (s) hipStreamDestroy(s);
  if (ctx->g16_stream) hipStreamDestroy(ctx->g16_stream);
  if (ctx->acc_tail) hipEventDestroy(ctx->acc_tail);
  if (ctx->stamp_dev) hipFree(ctx->stamp_dev);
  hipStreamDestroy(ctx->stream);
  if (ctx->aux) hipStreamDestroy(ctx->aux);
  if (ctx->copy) hipStreamDestroy(ctx->copy);
  if (ctx->pinned) hipHostFree(ctx->pinned);
  if (ctx->in_abc) hipFree(ctx->in_abc);
  for (int i = 0; i < gm_ctx::H2D_SLOTS; i++) {
    if (ctx->h2d_pin[i]) hipHostFree(ctx->h2d_pin[i]);
    if (ctx->h2d_ev[i]) hipEventDestroy(ctx->h2d_ev[i]);
  }
  delete ctx;
  return GM_OK;
}

int gm_trim(gm_ctx* ctx) {
  if (!ctx) return GM_ERR_INVALID;
  gm::CtxLock g(ctx);
  if (!ctx->live_msms.empty()) {
    set_error("gm_trim: MSMs are pending on this context (gm_msm_wait them first)");
    return GM_ERR_INVALID;
  }
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->aux) GM_HIP(hipStreamSynchronize(ctx->aux));
  if (ctx->copy) GM_HIP(hipStreamSynchronize(ctx->copy));
  for (hipStream_t st : ctx->slot_stream)
    if (st) GM_HIP(hipStreamSynchronize(st));
  if (ctx->g16_stream) GM_HIP(hipStreamSynchronize(ctx->g16_stream));
  std::vector<gm::ArenaState*> arenas{&ctx->arena};
  for (gm::ArenaState& sa : ctx->slots) arenas.push_back(&sa);
  for (gm::ArenaState* a : arenas) {
    for (auto& ch : a->chunks) hipFree(ch.base);
    a->chunks.clear();
    a->cur_chunk = a->cur_top = 0;
  }
  if (ctx->in_abc) hipFree(ctx->in_abc);
  ctx->in_abc = nullptr;
  ctx->in_abc_cap = 0;
  while (!ctx->spare_keys.empty()) stage_spare_release(ctx->spare_keys.back());  // parked stages
  for (int i = 0; i < gm_ctx::H2D_SLOTS; i++) {
    if (ctx->h2d_pin[i]) hipHostFree(ctx->h2d_pin[i]);
    ctx->h2d_pin[i] = nullptr;
  }
  ntt_domains_free(ctx);
  return GM_OK;
}

int gm_synchronize(gm_ctx* ctx) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}

int gm_profile_enable(gm_ctx* ctx, int on) {
  gm::CtxLock g(ctx);
  ctx->profiling = on != 0;
  if (ctx->profiling) {
    GM_HIP(hipSetDevice(ctx->device));
    gm::stamp_ensure(ctx);  // best effort: without the ring only the event brackets are recorded
    (void)hipGetLastError();
  }
  return GM_OK;
}
int gm_profile_reset(gm_ctx* ctx) {
  gm::CtxLock g(ctx);
  hipStreamSynchronize(ctx->stream);
  prof_collect(ctx);
  stamp_collect(ctx);
  ctx->stats.clear();
  return GM_OK;
}
int gm_profile_get(gm_ctx* ctx, const char* name, double* total_ms, uint64_t* count) {
  gm::CtxLock g(ctx);
  hipStreamSynchronize(ctx->stream);
  prof_collect(ctx);
  stamp_collect(ctx);
  auto it = ctx->stats.find(name);
  if (it == ctx->stats.end()) {
    *total_ms = 0;
    *count = 0;
    return GM_OK;
  }
  *total_ms = it->second.total_ms;
  *count = it->second.count;
  return GM_OK;
}
int gm_profile_dump(gm_ctx* ctx, char* buf, size_t cap) {
  gm::CtxLock g(ctx);
  hipStreamSynchronize(ctx->stream);
  prof_collect(ctx);
  stamp_collect(ctx);
  std::string s;
  for (auto& kv : ctx->stats)
    s += kv.first + " " + std::to_string(kv.second.total_ms) + " " + std::to_string(kv.second.count) + "\n";
  if (cap) {
    size_t m = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), m);
    buf[m] = 0;
  }
  return GM_OK;
}
int gm_set_msm_window(gm_ctx* ctx, int c) {
  if (c != 0 && (c < 2 || c > 24)) return GM_ERR_INVALID;
  ctx->msm_c_override = c;
  return GM_OK;
}

int gm_set_msm_glv(gm_ctx* ctx, int mode) {
  if (!ctx || mode < -1 || mode > 1) return GM_ERR_INVALID;
  gm::CtxLock g(ctx);
  ctx->msm_glv = mode;
  return GM_OK;
}

// ---- memory -----------------------------------------------------------------
int gm_malloc(gm_ctx* ctx, size_t bytes, void** dev_out) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  hipError_t e = hipMalloc(dev_out, bytes ? bytes : 16);
  if (e != hipSuccess) {
    set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return GM_ERR_OOM;
  }
  return GM_OK;
}
int gm_free(gm_ctx* ctx, void* dev) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  GM_HIP(hipFree(dev));
  return GM_OK;
}
int gm_memcpy_h2d(gm_ctx* ctx, void* dev, const void* host, size_t bytes) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
int gm_memcpy_d2h(gm_ctx* ctx, void* host, const void* dev, size_t bytes) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
int gm_memcpy_d2d(gm_ctx* ctx, void* dst, const void* src, size_t bytes) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
int gm_copy_to_device(gm_ctx* ctx, const void* host, size_t bytes, void** dev_out) {
  int rc = gm_malloc(ctx, bytes, dev_out);
  if (rc) return rc;
  return gm_memcpy_h2d(ctx, *dev_out, host, bytes);
}
int gm_copy_points_to_device(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n,
                             void** dev_out) {
  if (int rc = check_curve(curve)) return rc;
  return gm_copy_to_device(ctx, host_points, n * fp_bytes(curve) * (g2 ? 4 : 2), dev_out);
}

// ---- MSM ------------------------------------------------------------------------
int gm_msm(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* points_dev,
           size_t n, void* out_jac, void* out_affine) {
  if (!ctx) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc;
  if (curve == GM_BN254)
    rc = g2 ? msm_to_host<CurveBN254, true>(ctx, scalars_dev, points_dev, n, out_jac, out_affine)
            : msm_to_host<CurveBN254, false>(ctx, scalars_dev, points_dev, n, out_jac, out_affine);
  else
    rc = g2 ? msm_to_host<CurveBLS12377, true>(ctx, scalars_dev, points_dev, n, out_jac, out_affine)
            : msm_to_host<CurveBLS12377, false>(ctx, scalars_dev, points_dev, n, out_jac, out_affine);
  prof_collect(ctx);
  return rc;
}

}  // extern "C"

bool gm::msm_glv_on(const gm_ctx* ctx, bool g2, size_t n) {
  if (ctx && ctx->msm_glv >= 0) return ctx->msm_glv != 0;
  // Default: GLV up to 2^21 points.  Measured (r03, same box, sync MSMs): at
  // 2^20 it halves the bucket reduction (BN254 G1 2.26 -> 2.14 ms, G2 7.65 ->
  // 6.51 ms); at 2^22 (BLS12-377) the reduction is a small share while the 2n
  // virtual points double the gathered point set (G1 14.2 -> 15.8 ms, G2 56.6
  // -> 62.1 ms).  gm_set_msm_glv overrides it per context.
  if (n > (size_t(1) << 21)) return false;
  return true;
}

// MsmTail's pinned readback buffer goes back to its context (msm.hpp)
void gm::MsmTail::release_stage() {
  if (stage_ctx) tail_pinned_release(stage_ctx, stage_idx);
  stage_ctx = nullptr;
  stage_idx = -1;
  stage = nullptr;
}

struct gm_msm_pending {
  gm_ctx* ctx;  // nullptr once gm_destroy orphaned the handle
  int curve, g2;
  hipStream_t st = nullptr;  // stream the MSM runs on (slot stream or ctx->stream)
  gm::SlotArena slot;
  gm::MsmTail tail;
  explicit gm_msm_pending(gm_ctx* c) : ctx(c), slot(c) {}
};

// gm_destroy with MSMs pending (its streams already synchronised): every pending
// handle gives its slot arena and pinned readback buffer back to the context and
// is marked orphaned; the caller's later gm_msm_wait reports it and frees it.
void gm::orphan_pending_msms(gm_ctx* ctx) {
  for (gm_msm_pending* p : ctx->live_msms) {
    p->tail.release_stage();
    p->slot.release();
    p->ctx = nullptr;
  }
  ctx->live_msms.clear();
}

namespace {
template <class C, bool G2>
int msm_wait_t(gm_msm_pending* p, void* out_jac, void* out_aff) {
  using HF = typename GroupSel<C, G2>::HF;
  HF j[3];
  int rc = msm_finish<C, G2>(p->ctx, p->tail, j);
  if (rc) return rc;
  if (out_jac) memcpy(out_jac, j, sizeof(j));
  if (out_aff) {
    host::Aff<HF> a = host::to_aff(host::Jac<HF>{j[0], j[1], j[2]});
    memcpy(out_aff, &a, sizeof(a));
  }
  return GM_OK;
}
}  // namespace

extern "C" {

int gm_msm_async(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* points_dev, size_t n,
                 gm_msm_pending** out) {
  if (!ctx || !out) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  // no CtxLock: nothing is queued on ctx->stream here (gm_ctx::pending_reads)
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  auto* p = new gm_msm_pending(ctx);
  p->curve = curve;
  p->g2 = g2 ? 1 : 0;
  int rc = p->slot.take();
  // One stream per slot: one MSM's fixup / reduction / readback overlaps the
  // next one's conversion and sort (profiles/r04m_hwq_ab.txt, r05r_slot_stream_ab.txt).
  // It starts after the work already queued on ctx->stream (the inputs).
  hipEvent_t inputs_read = nullptr;
  p->st = ctx->stream;
  if (rc == GM_OK) {
    hipStream_t& ss = ctx->slot_stream[p->slot.k];
    // The slot streams run at the highest stream priority: the runtime keeps a
    // separate pool of hardware queues per priority, so with the default four
    // queues they do not share one with ctx->stream / aux / copy or each other,
    // and the next MSM's conversion and sort start beside this one's reduction
    // (bench 2^20: 599-605 -> 632-645 Mpoints/s with the change below,
    // profiles/r05r_slot_stream_ab.txt).
    if (!ss) {
      int least = 0, greatest = 0;
      GM_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
      GM_HIP(hipStreamCreateWithPriority(&ss, hipStreamNonBlocking, greatest));
    }
    // Ordered after the work already queued on ctx->stream (the inputs) -- by a
    // marker only when that stream still has work: a packet on ctx->stream waits
    // behind everything in its hardware queue, which may be shared with a slot
    // stream running the previous MSM.
    const hipError_t q = hipStreamQuery(ctx->stream);
    (void)hipGetLastError();  // hipErrorNotReady is an answer, not an error
    if (q != hipSuccess) {
      hipEvent_t ev;
      GM_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      GM_HIP(hipEventRecord(ev, ctx->stream));
      GM_HIP(hipStreamWaitEvent(ss, ev, 0));
      GM_HIP(hipEventDestroy(ev));
    }
    p->st = ss;
    // work queued later on ctx->stream (synchronous calls that may overwrite the
    // scalars or points in place) waits until this MSM has read them: the event is
    // recorded after the digits and the point conversion, before the accumulation
    GM_HIP(hipEventCreateWithFlags(&inputs_read, hipEventDisableTiming));
  }
  {
    // The in-flight MSMs' accumulations run one after another (gm_ctx::acc_tail):
    // each launch then runs with the chip's wave slots free of the previous
    // one, so its start / stop stamps bracket its own execution (the bench's
    // kernel time; without the order a launch was stamped while it waited for the
    // previous accumulation's slots).  Same box: 621-624 against 624-630
    // Mpoints/s unordered (profiles/r06c_acc_chain_ab.txt).
    ctx->acc_chain = p->st != ctx->stream;  // slot streams only
    StreamSwap sw(ctx, p->st);
    struct ChainOff {
      gm_ctx* c;
      ~ChainOff() { c->acc_chain = false; }
    } chain_off{ctx};
    if (rc == GM_OK) {
      Arena& a = *p->slot.a;
      const void* sc = scalars_dev;
      const void* pt = points_dev;
      if (curve == GM_BN254)
        rc = g2 ? msm_device_launch<CurveBN254, true>(ctx, a, sc, pt, n, false, nullptr, p->tail, inputs_read)
                : msm_device_launch<CurveBN254, false>(ctx, a, sc, pt, n, false, nullptr, p->tail, inputs_read);
      else
        rc = g2 ? msm_device_launch<CurveBLS12377, true>(ctx, a, sc, pt, n, false, nullptr, p->tail, inputs_read)
                : msm_device_launch<CurveBLS12377, false>(ctx, a, sc, pt, n, false, nullptr, p->tail, inputs_read);
    }
  }
  if (inputs_read && rc) hipEventDestroy(inputs_read);
  if (rc) {
    delete p;
    return rc;
  }
  // ctx->stream waits on it at the next call that may queue work there (CtxLock)
  if (inputs_read) ctx->pending_reads.push_back({p, inputs_read});
  ctx->live_msms.push_back(p);
  *out = p;
  return GM_OK;
}

int gm_msm_wait(gm_msm_pending* p, void* out_jac, void* out_affine) {
  if (!p) return GM_ERR_INVALID;
  gm_ctx* ctx = p->ctx;
  if (!ctx) {
    delete p;
    set_error("gm_msm_wait: the context was destroyed while this MSM was pending");
    return GM_ERR_INVALID;
  }
  std::lock_guard<std::recursive_mutex> g(ctx->mu);  // nothing queued on ctx->stream
  auto& live = ctx->live_msms;
  live.erase(std::remove(live.begin(), live.end(), p), live.end());
  // a finished MSM has read its inputs: ctx->stream need not wait for it
  auto& pr = ctx->pending_reads;
  for (auto it = pr.begin(); it != pr.end();)
    if (it->first == p) {
      hipEventDestroy(it->second);
      it = pr.erase(it);
    } else {
      ++it;
    }
  GM_HIP(hipSetDevice(ctx->device));
  int rc;
  StreamSwap sw(ctx, p->st);  // a long-span redo runs on the MSM's own stream
  if (p->curve == GM_BN254)
    rc = p->g2 ? msm_wait_t<CurveBN254, true>(p, out_jac, out_affine) : msm_wait_t<CurveBN254, false>(p, out_jac, out_affine);
  else
    rc = p->g2 ? msm_wait_t<CurveBLS12377, true>(p, out_jac, out_affine)
               : msm_wait_t<CurveBLS12377, false>(p, out_jac, out_affine);
  prof_collect(ctx);
  delete p;
  return rc;
}

int gm_msm_host_scalars(gm_ctx* ctx, int curve, int g2, const void* scalars_host,
                        const void* points_dev, size_t n, void* out_jac, void* out_affine) {
  if (!ctx || (n && !scalars_host)) return GM_ERR_INVALID;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  Arena arena(ctx);
  DevBuf s;
  int rc;
  if ((rc = s.alloc(arena, 32 * n))) return rc;
  GM_HIP(hipMemcpyAsync(s.p, scalars_host, 32 * n, hipMemcpyHostToDevice, ctx->stream));
  return gm_msm(ctx, curve, g2, s.p, points_dev, n, out_jac, out_affine);
}

int gm_points_upload(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n, void** out) {
  if (!ctx || !out) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  const size_t gb = fp_bytes(curve) * (g2 ? 4 : 2) * n;
  const size_t ib = n * (curve == GM_BN254 ? (g2 ? msm_internal_point_bytes<CurveBN254, true>()
                                                 : msm_internal_point_bytes<CurveBN254, false>())
                                           : (g2 ? msm_internal_point_bytes<CurveBLS12377, true>()
                                                 : msm_internal_point_bytes<CurveBLS12377, false>()));
  Arena arena(ctx);
  DevBuf tmp;
  int rc;
  if ((rc = tmp.alloc(arena, gb))) return rc;
  hipError_t e = hipMalloc(out, ib ? ib : 16);
  if (e != hipSuccess) {
    set_error(std::string("gm_points_upload hipMalloc: ") + hipGetErrorString(e));
    return GM_ERR_OOM;
  }
  GM_HIP(hipMemcpyAsync(tmp.p, host_points, gb, hipMemcpyHostToDevice, ctx->stream));
  if (curve == GM_BN254)
    rc = g2 ? msm_prepare_points<CurveBN254, true>(ctx, tmp.p, n, *out)
            : msm_prepare_points<CurveBN254, false>(ctx, tmp.p, n, *out);
  else
    rc = g2 ? msm_prepare_points<CurveBLS12377, true>(ctx, tmp.p, n, *out)
            : msm_prepare_points<CurveBLS12377, false>(ctx, tmp.p, n, *out);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}

extern "C++" {
template <class C, bool G2>
static int msm_prepared_t(gm_ctx* ctx, const void* sc, const void* pts, size_t n, void* out_jac, void* out_aff,
                          const MsmPrecomp* pre = nullptr) {
  using HF = typename GroupSel<C, G2>::HF;
  HF j[3];
  int rc = msm_device<C, G2>(ctx, sc, pts, n, j, true, pre);
  if (rc) return rc;
  if (out_jac) memcpy(out_jac, j, sizeof(j));
  if (out_aff) {
    host::Aff<HF> a = host::to_aff(host::Jac<HF>{j[0], j[1], j[2]});
    memcpy(out_aff, &a, sizeof(a));
  }
  return GM_OK;
}
}  // extern "C++"

int gm_msm_prepared(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* prepared, size_t n,
                    void* out_jac, void* out_affine) {
  if (!ctx) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc;
  if (curve == GM_BN254)
    rc = g2 ? msm_prepared_t<CurveBN254, true>(ctx, scalars_dev, prepared, n, out_jac, out_affine)
            : msm_prepared_t<CurveBN254, false>(ctx, scalars_dev, prepared, n, out_jac, out_affine);
  else
    rc = g2 ? msm_prepared_t<CurveBLS12377, true>(ctx, scalars_dev, prepared, n, out_jac, out_affine)
            : msm_prepared_t<CurveBLS12377, false>(ctx, scalars_dev, prepared, n, out_jac, out_affine);
  prof_collect(ctx);
  return rc;
}

// ---- fixed-base precomputed point sets -------------------------------------------
static int make_precomp(int curve, size_t n, int window, MsmPrecomp* out) {
  const int bits = curve == GM_BN254 ? CurveBN254::FR_BITS : CurveBLS12377::FR_BITS;
  if (window == 0) {
    *out = msm_choose_precomp(n, bits);
    return GM_OK;
  }
  if (window < 2 || window > 24) {
    set_error("precompute: window must be 0 (auto) or in [2, 24]");
    return GM_ERR_INVALID;
  }
  out->c = (uint32_t)window;
  out->W = (uint32_t)((bits + 1 + window - 1) / window);
  out->narrow = precomp_narrow(out->c, out->W, bits);
  out->stride = n;
  return GM_OK;
}

int gm_precompute_layout(int curve, size_t n, int window, int* c_out, int* copies_out) {
  if (int rc = check_curve(curve)) return rc;
  MsmPrecomp p;
  if (int rc = make_precomp(curve, n, window, &p)) return rc;
  if (c_out) *c_out = (int)p.c;
  if (copies_out) *copies_out = (int)p.W;
  return GM_OK;
}

int gm_points_upload_precomputed(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n, int window,
                                 void** out) {
  if (!ctx || !out) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  MsmPrecomp pre;
  if (int rc = make_precomp(curve, n, window, &pre)) return rc;
  if ((size_t)pre.W * n >= (size_t(1) << 31)) {
    set_error("precompute: copies * n must be < 2^31");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  const size_t gb = fp_bytes(curve) * (g2 ? 4 : 2) * n;
  const size_t ib = (size_t)pre.W * n *
                    (curve == GM_BN254 ? (g2 ? msm_internal_point_bytes<CurveBN254, true>()
                                             : msm_internal_point_bytes<CurveBN254, false>())
                                       : (g2 ? msm_internal_point_bytes<CurveBLS12377, true>()
                                             : msm_internal_point_bytes<CurveBLS12377, false>()));
  Arena arena(ctx);
  DevBuf tmp;
  int rc;
  if ((rc = tmp.alloc(arena, gb ? gb : 16))) return rc;
  hipError_t e = hipMalloc(out, ib ? ib : 16);
  if (e != hipSuccess) {
    set_error(std::string("gm_points_upload_precomputed hipMalloc: ") + hipGetErrorString(e));
    return GM_ERR_OOM;
  }
  if (gb) GM_HIP(hipMemcpyAsync(tmp.p, host_points, gb, hipMemcpyHostToDevice, ctx->stream));
  if (curve == GM_BN254)
    rc = g2 ? msm_precompute_points<CurveBN254, true>(ctx, tmp.p, n, pre, *out)
            : msm_precompute_points<CurveBN254, false>(ctx, tmp.p, n, pre, *out);
  else
    rc = g2 ? msm_precompute_points<CurveBLS12377, true>(ctx, tmp.p, n, pre, *out)
            : msm_precompute_points<CurveBLS12377, false>(ctx, tmp.p, n, pre, *out);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}

int gm_msm_precomputed(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* prepared,
                       size_t prepared_n, int window, size_t n, void* out_jac, void* out_affine) {
  if (!ctx) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  if (n > prepared_n) {
    set_error("msm_precomputed: n exceeds the prepared point count");
    return GM_ERR_INVALID;
  }
  MsmPrecomp pre;
  if (int rc = make_precomp(curve, prepared_n, window, &pre)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc;
  if (curve == GM_BN254)
    rc = g2 ? msm_prepared_t<CurveBN254, true>(ctx, scalars_dev, prepared, n, out_jac, out_affine, &pre)
            : msm_prepared_t<CurveBN254, false>(ctx, scalars_dev, prepared, n, out_jac, out_affine, &pre);
  else
    rc = g2 ? msm_prepared_t<CurveBLS12377, true>(ctx, scalars_dev, prepared, n, out_jac, out_affine, &pre)
            : msm_prepared_t<CurveBLS12377, false>(ctx, scalars_dev, prepared, n, out_jac, out_affine, &pre);
  prof_collect(ctx);
  return rc;
}

int gm_kzg_commit(gm_ctx* ctx, int curve, const void* srs, size_t srs_len, const void* coeffs_host, size_t n,
                  void* digest_affine) {
  if (!ctx || !digest_affine) return GM_ERR_INVALID;
  if (n > srs_len) {
    set_error("kzg commit: polynomial larger than the SRS");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  Arena arena(ctx);
  DevBuf s;
  int rc;
  if ((rc = s.alloc(arena, 32 * (n ? n : 1)))) return rc;
  if (n) GM_HIP(hipMemcpyAsync(s.p, coeffs_host, 32 * n, hipMemcpyHostToDevice, ctx->stream));
  return gm_msm_prepared(ctx, curve, 0, s.p, srs, n, nullptr, digest_affine);
}

// ---- NTT --------------------------------------------------------------------------
int gm_ntt(gm_ctx* ctx, int curve, void* data_dev, size_t n, int inverse, int dit, int coset) {
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? ntt_device<CurveBN254>(ctx, data_dev, n, inverse, dit, coset)
                             : ntt_device<CurveBLS12377>(ctx, data_dev, n, inverse, dit, coset);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}
int gm_poly_ops(gm_ctx* ctx, int curve, void* a, const void* b, const void* c, size_t n,
                const void* den_host) {
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? poly_ops_device<CurveBN254>(ctx, a, b, c, n, den_host)
                             : poly_ops_device<CurveBLS12377>(ctx, a, b, c, n, den_host);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}
int gm_reverse_scalars(gm_ctx* ctx, int curve, void* data_dev, size_t n) {
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? reverse_device<CurveBN254>(ctx, data_dev, n)
                             : reverse_device<CurveBLS12377>(ctx, data_dev, n);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}
int gm_groth16_compute_h(gm_ctx* ctx, int curve, void* a, void* b, void* c, size_t len, size_t n) {
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? compute_h_device<CurveBN254>(ctx, a, b, c, len, n)
                             : compute_h_device<CurveBLS12377>(ctx, a, b, c, len, n);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}

// ---- host group helpers ---------------------------------------------------------------
extern "C++" {
template <class HF>
static void jac_add_t(const void* p, const void* q, void* out) {
  host::Jac<HF> a, b;
  memcpy(&a, p, sizeof(a));
  memcpy(&b, q, sizeof(b));
  host::Jac<HF> r = host::jadd(a, b);
  memcpy(out, &r, sizeof(r));
}
template <class HF>
static void jac_aff_t(const void* p, void* out) {
  host::Jac<HF> a;
  memcpy(&a, p, sizeof(a));
  host::Aff<HF> r = host::to_aff(a);
  memcpy(out, &r, sizeof(r));
}
}  // extern "C++"

int gm_jac_add(int curve, int g2, const void* p, const void* q, void* out) {
  if (int rc = check_curve(curve)) return rc;
  if (curve == GM_BN254)
    g2 ? jac_add_t<CurveBN254::HG2F>(p, q, out) : jac_add_t<CurveBN254::HG1F>(p, q, out);
  else
    g2 ? jac_add_t<CurveBLS12377::HG2F>(p, q, out) : jac_add_t<CurveBLS12377::HG1F>(p, q, out);
  return GM_OK;
}
int gm_jac_to_affine(int curve, int g2, const void* p, void* out) {
  if (int rc = check_curve(curve)) return rc;
  if (curve == GM_BN254)
    g2 ? jac_aff_t<CurveBN254::HG2F>(p, out) : jac_aff_t<CurveBN254::HG1F>(p, out);
  else
    g2 ? jac_aff_t<CurveBLS12377::HG2F>(p, out) : jac_aff_t<CurveBLS12377::HG1F>(p, out);
  return GM_OK;
}

// ---- synthetic inputs -------------------------------------------------------------------
static const uint64_t GEN_BN_G1[] = GM_BN254_G1_GEN64;
static const uint64_t GEN_BN_G2[] = GM_BN254_G2_GEN64;
static const uint64_t GEN_BLS_G1[] = GM_BLS12377_G1_GEN64;
static const uint64_t GEN_BLS_G2[] = GM_BLS12377_G2_GEN64;

int gm_generator(int curve, int g2, void* out) {
  if (int rc = check_curve(curve)) return rc;
  const uint64_t* src = curve == GM_BN254 ? (g2 ? GEN_BN_G2 : GEN_BN_G1) : (g2 ? GEN_BLS_G2 : GEN_BLS_G1);
  memcpy(out, src, fp_bytes(curve) * (g2 ? 4 : 2));
  return GM_OK;
}

int gm_random_scalars(gm_ctx* ctx, int curve, uint64_t seed, size_t n, void* scalars_dev) {
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  if (curve == GM_BN254)
    hipLaunchKernelGGL(k_random_scalars<Bn254Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                       (uint32_t*)scalars_dev, n, seed);
  else
    hipLaunchKernelGGL(k_random_scalars<Bls377Fr>, dim3(blocks_for(n, 256)), dim3(256), 0,
                       ctx->stream, (uint32_t*)scalars_dev, n, seed);
  GM_HIP(hipGetLastError());
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}

extern "C++" {
template <class C, bool G2>
static int batch_mul_t(gm_ctx* ctx, const void* base, const void* sc, size_t n, void* out) {
  using DF = typename GroupSel<C, G2>::DF;
  GPoint<DF> b;
  memcpy(&b, base, sizeof(b));
  hipLaunchKernelGGL((k_batch_mul_base<typename C::Fr, DF>), dim3(blocks_for(n, 128)), dim3(128), 0,
                     ctx->stream, (const uint32_t*)sc, n, b, (uint32_t*)out);
  GM_HIP(hipGetLastError());
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
}  // extern "C++"

int gm_batch_mul_base(gm_ctx* ctx, int curve, int g2, const void* base, const void* sc, size_t n,
                      void* out) {
  if (int rc = check_curve(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  if (curve == GM_BN254)
    return g2 ? batch_mul_t<CurveBN254, true>(ctx, base, sc, n, out)
              : batch_mul_t<CurveBN254, false>(ctx, base, sc, n, out);
  return g2 ? batch_mul_t<CurveBLS12377, true>(ctx, base, sc, n, out)
            : batch_mul_t<CurveBLS12377, false>(ctx, base, sc, n, out);
}

}  // extern "C"
