// Proving-key I/O and staged prover inputs.
//
//  * gm_g16_pk_upload_dump[_shard]: the five point slices of a gnark
//    `WriteDump` file (backend/groth16/bn254/marshal.go:389-456; ReadDump
//    :460-550 reads them back) streamed from a file descriptor into device
//    buffers.  Each slice is gnark-crypto utils/unsafe.WriteSlice output: a
//    little-endian u64 element count, then the raw G1Affine / G2Affine memory
//    (Montgomery u64 limbs -- this ABI's point layout).  Chunks are pread into
//    two pinned 64 MiB buffers; the H2D copy and the conversion (or window
//    precomputation) of chunk k run on the GPU while chunk k+1 is read, so the
//    Go heap never holds the ~6 GB of points ReadDump would materialise.
//  * gm_g16_pk_save_cache / gm_g16_pk_load_cache: a device-resident key in its
//    device layout (with the GM_PK_PRECOMPUTE window copies, ~77 GB for a
//    BN254 2^24 key) written to / read from a file: the one-time conversion and
//    precomputation are paid once per key, not once per process.
//  * gm_g16_stage_*: a, b, c (and the wires) handed over while the solver
//    (constraint/bn254/solver.go:426-532) still runs, level by level or by
//    ranges, through a pinned ring on the context's copy stream; the prove
//    after Solve then starts from device-resident inputs.
#include <errno.h>
#include <unistd.h>

#include <cstring>
#include <string>

#include "curves.hpp"
#include "groth16.hpp"
#include "msm.hpp"
#include "runtime.hpp"

using namespace gm;

namespace {

constexpr size_t IO_CHUNK = size_t(64) << 20;

int read_at(int fd, void* buf, size_t n, uint64_t off) {
  char* p = static_cast<char*>(buf);
  while (n) {
    const ssize_t r = pread(fd, p, n, (off_t)off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) {
      set_error(r == 0 ? "pk dump: unexpected end of file" : std::string("pk dump: pread: ") + strerror(errno));
      return GM_ERR_INVALID;
    }
    p += r;
    n -= (size_t)r;
    off += (uint64_t)r;
  }
  return GM_OK;
}
int read_seq(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n) {
    const ssize_t r = read(fd, p, n);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) {
      set_error(r == 0 ? "pk cache: unexpected end of file" : std::string("pk cache: read: ") + strerror(errno));
      return GM_ERR_INVALID;
    }
    p += r;
    n -= (size_t)r;
  }
  return GM_OK;
}
int write_seq(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    const ssize_t r = write(fd, p, n);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) {
      set_error(std::string("pk cache: write: ") + strerror(errno));
      return GM_ERR_INVALID;
    }
    p += r;
    n -= (size_t)r;
  }
  return GM_OK;
}

// Two pinned host buffers + two device buffers of IO_CHUNK bytes with an event
// each: slot k % 2 is reused only after the GPU work that read it finished.
struct IoRing {
  void* host[2] = {nullptr, nullptr};
  void* dev[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool used[2] = {false, false};
  int init(bool want_dev) {
    for (int i = 0; i < 2; i++) {
      if (hipHostMalloc(&host[i], IO_CHUNK, hipHostMallocDefault) != hipSuccess) {
        set_error("pk io: hipHostMalloc failed");
        return GM_ERR_OOM;
      }
      if (want_dev && hipMalloc(&dev[i], IO_CHUNK) != hipSuccess) {
        set_error("pk io: hipMalloc failed");
        return GM_ERR_OOM;
      }
      GM_HIP(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    return GM_OK;
  }
  int acquire(int k) {
    if (used[k]) GM_HIP(hipEventSynchronize(ev[k]));
    used[k] = true;
    return GM_OK;
  }
  ~IoRing() {
    for (int i = 0; i < 2; i++) {
      if (ev[i]) {
        hipEventSynchronize(ev[i]);
        hipEventDestroy(ev[i]);
      }
      if (host[i]) hipHostFree(host[i]);
      if (dev[i]) hipFree(dev[i]);
    }
  }
};

// Streams `count` gnark-layout points of pb bytes from fd at `off` into the
// internal array dst (and its window copies when pre != nullptr).
int stream_points(gm_ctx* ctx, IoRing& ring, int curve, bool g2, int fd, uint64_t off, size_t count,
                  const MsmPrecomp* pre, void* dst) {
  const size_t pb = 2 * (g2 ? 2 : 1) * fp_bytes(curve);
  const size_t ipb = internal_point_bytes(curve, g2);
  const size_t per = IO_CHUNK / pb;
  for (size_t i0 = 0, k = 0; i0 < count; i0 += per, k ^= 1) {
    const size_t cnt = std::min(per, count - i0);
    int rc;
    if ((rc = ring.acquire((int)k))) return rc;
    if ((rc = read_at(fd, ring.host[k], cnt * pb, off + i0 * pb))) return rc;
    GM_HIP(hipMemcpyAsync(ring.dev[k], ring.host[k], cnt * pb, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = prepare_points_into(ctx, curve, g2, ring.dev[k], cnt, pre, (char*)dst + i0 * ipb))) return rc;
    GM_HIP(hipEventRecord(ring.ev[k], ctx->stream));
  }
  return GM_OK;
}

void shard_range(size_t n, int rank, int world, size_t* lo, size_t* hi) {
  const size_t q = n / (size_t)world, r = n % (size_t)world;
  *lo = (size_t)rank * q + std::min((size_t)rank, r);
  *hi = *lo + q + ((size_t)rank < r ? 1 : 0);
}

// ---- device-layout cache ---------------------------------------------------
constexpr char CACHE_MAGIC[8] = {'G', 'M', 'P', 'K', 'C', 'A', 'C', 'H'};
constexpr uint32_t CACHE_VERSION = 3;
// Device-layout fingerprint: the internal point form (radix-2^29 Montgomery
// limbs packed in gnark's word layout) and the precomputed-copy rule
// (PRECOMP_LAYOUT, msm.hpp).  A cache written by a build with another layout is
// refused instead of being read as points.
constexpr uint32_t CACHE_LAYOUT = (uint32_t(RADIX) << 24) | (uint32_t(PRECOMP_LAYOUT) << 8) | 1u;

struct CacheHeader {
  char magic[8];
  uint32_t version, curve;
  uint32_t layout, wshare;  // wshare: bit x = array x (A, B, K) wire-indexed (shared wire plan)
  uint64_t n, nb_wires, nb_public, nbA, nbB, nbK, zlo, nbZ, wlo, whi, precomp;
  uint32_t pre_c[4], pre_W[4];
  uint64_t pre_stride[4];
};

// Header invariants of a device-layout cache (a corrupt or foreign header must
// not size allocations or steer device gathers out of bounds).
int check_cache_header(const CacheHeader& h) {
  auto bad = [](const char* what) {
    set_error(std::string("pk cache: inconsistent header (") + what + ")");
    return GM_ERR_INVALID;
  };
  const uint64_t lim = uint64_t(1) << 31;
  if (h.n < 2 || (h.n & (h.n - 1)) || h.n > lim) return bad("domain size");
  if (h.nb_wires == 0 || h.nb_wires > lim || h.nb_public > h.nb_wires) return bad("wire counts");
  if (h.zlo > h.n - 1 || h.nbZ > h.n - 1 - h.zlo) return bad("Z slice");
  if (h.wlo > h.whi || h.whi > h.nb_wires) return bad("wire slice");
  if (h.nbA > h.nb_wires || h.nbB > h.nb_wires || h.nbK > h.nb_wires) return bad("array lengths");
  if (h.precomp > 1) return bad("precompute flag");
  if (h.wshare > 7) return bad("shared-plan flags");
  const uint64_t span = h.whi - h.wlo;
  if (((h.wshare & 1) && h.nbA > span) || ((h.wshare & 2) && h.nbB > span) || ((h.wshare & 4) && h.nbK > span))
    return bad("wire-indexed array longer than its wire span");
  if (h.precomp) {
    const int frbits = h.curve == GM_BN254 ? CurveBN254::FR_BITS : CurveBLS12377::FR_BITS;
    const uint64_t cnt[4] = {(h.wshare & 1) ? span : h.nbA, (h.wshare & 2) ? span : h.nbB, h.nbZ,
                             (h.wshare & 4) ? span : h.nbK};
    for (int i = 0; i < 4; i++) {
      if (h.pre_c[i] < 1 || h.pre_c[i] > 30 || h.pre_W[i] < 1 ||
          (uint64_t)h.pre_c[i] * h.pre_W[i] < (uint64_t)frbits + 1)
        return bad("window geometry");
      if (h.pre_stride[i] < cnt[i] || (uint64_t)h.pre_W[i] * h.pre_stride[i] >= lim) return bad("window copies");
    }
  }
  return GM_OK;
}

size_t array_bytes(const gm_g16_pk* pk, int which) {
  const size_t g1 = internal_point_bytes(pk->curve, false), g2 = internal_point_bytes(pk->curve, true);
  auto copies = [&](const MsmPrecomp& p) { return pk->precomp ? (size_t)p.W : size_t(1); };
  switch (which) {
    case PK_A: return g1 * pk_array_points(pk, PK_A) * copies(pk->preA);
    case PK_B: return g1 * pk_array_points(pk, PK_B) * copies(pk->preB);
    case PK_Z: return g1 * pk->nbZ * copies(pk->preZ);
    case PK_K: return g1 * pk_array_points(pk, PK_K) * copies(pk->preK);
    case PK_B2: return g2 * pk_array_points(pk, PK_B2) * copies(pk->preB);
    case 5: return 4 * pk->nbA;
    case 6: return 4 * pk->nbB;
    default: return 4 * pk->nbK;
  }
}
void** array_ptr(gm_g16_pk* pk, int which) {
  void** p[8] = {&pk->A, &pk->B, &pk->Z, &pk->K, &pk->B2, &pk->idxA, &pk->idxB, &pk->idxK};
  return p[which];
}

}  // namespace

// ---- staged inputs ----------------------------------------------------------
struct gm_g16_stage {
  gm_ctx* ctx = nullptr;
  gm_g16_pk* pk = nullptr;
  size_t nc = 0;
  void* vec[4] = {nullptr, nullptr, nullptr, nullptr};  // a, b, c (n Fr each), wires (nb_wires Fr)
  size_t len[4] = {0, 0, 0, 0};
  static constexpr int SLOTS = 4;
  static constexpr size_t SLOT = size_t(16) << 20;
  void* host[SLOTS] = {};
  void* dev[SLOTS] = {};  // device staging of indexed puts
  hipEvent_t ev[SLOTS] = {};
  bool used[SLOTS] = {};
  int next = 0;
  // Indexed puts are records (u32 element, u32 vector, 32-B value) gathered in
  // the open ring slot: a put of one element (a solver level of one wire, the
  // squaring chain of groth16_test.go:120-156) costs its record copy, not a slot,
  // a copy and a launch.  The slot is flushed when full, when it holds FLUSH_AT
  // records at the end of a put (so the copies still overlap Solve), before a
  // range put and before the prove.
  static constexpr size_t REC_PER = (SLOT - 16) / 40 & ~size_t(3);
  static constexpr size_t FLUSH_AT = size_t(1) << 16;
  int open = -1;
  size_t open_cnt = 0;
  int take(int* k) {
    *k = next;
    next = (next + 1) % SLOTS;
    if (used[*k]) GM_HIP(hipEventSynchronize(ev[*k]));
    used[*k] = true;
    return GM_OK;
  }
  int flush();
  ~gm_g16_stage() {
    for (int i = 0; i < SLOTS; i++) {
      if (ev[i]) {
        hipEventSynchronize(ev[i]);
        hipEventDestroy(ev[i]);
      }
      if (host[i]) hipHostFree(host[i]);
      if (dev[i]) hipFree(dev[i]);
    }
    for (void* v : vec)
      if (v) hipFree(v);
  }
};

namespace {
// env knob that is on unless set to 0 (read per call: tests flip it)
bool getenv_flag_off(const char* name) {
  const char* v = getenv(name);
  return v && atoi(v) == 0;
}

// the stage's four vectors, passed by value to the scatter
struct StageDst {
  uint4* v[4];
  size_t len[4];
};
// dst[rec[j].y][rec[j].x] = val[j] (32-byte Fr)
// (gm_g16_stage_put_indexed checks every index on the host before the copy;
// the bounds test only keeps a bad launch from writing out of bounds)
__global__ void k_scatter_fr(const uint2* __restrict__ rec, const uint4* __restrict__ val, size_t k, StageDst d) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k) return;
  const uint2 r = rec[j];
  if (r.y > 3 || r.x >= d.len[r.y]) return;
  uint4* dst = d.v[r.y];
  dst[2 * (size_t)r.x] = val[2 * j];
  dst[2 * (size_t)r.x + 1] = val[2 * j + 1];
}
}  // namespace

// queue the open slot's records: copy to the slot's device staging, scatter
int gm_g16_stage::flush() {
  if (open < 0) return GM_OK;
  const int s = open;
  const size_t cnt = open_cnt;
  open = -1;
  open_cnt = 0;
  if (cnt == 0) return GM_OK;
  GM_HIP(hipSetDevice(ctx->device));
  StageDst d;
  for (int v = 0; v < 4; v++) {
    d.v[v] = (uint4*)vec[v];
    d.len[v] = len[v];
  }
  char* dv = (char*)dev[s] + 8 * REC_PER;
  GM_HIP(hipMemcpyAsync(dev[s], host[s], 8 * cnt, hipMemcpyHostToDevice, ctx->copy));
  GM_HIP(hipMemcpyAsync(dv, (char*)host[s] + 8 * REC_PER, 32 * cnt, hipMemcpyHostToDevice, ctx->copy));
  hipLaunchKernelGGL(k_scatter_fr, dim3(blocks_for(cnt, 256)), dim3(256), 0, ctx->copy, (const uint2*)dev[s],
                     (const uint4*)dv, cnt, d);
  GM_HIP(hipGetLastError());
  GM_HIP(hipEventRecord(ev[s], ctx->copy));
  return GM_OK;
}

extern "C" {

int gm_g16_pk_upload_dump_shard(gm_ctx* ctx, int curve, const gm_g16_pk_host* meta, int fd, uint64_t offset,
                                unsigned flags, int rank, int world, uint64_t* end_offset, gm_g16_pk** out) {
  if (int rc = check_curve_id(curve)) return rc;
  if (!ctx || !meta || !out || fd < 0 || meta->domain_size < 2) return GM_ERR_INVALID;
  if (flags & ~(unsigned)(GM_PK_PRECOMPUTE | GM_PK_PRECOMPUTE_AUTO)) {
    set_error("pk dump: unknown flags");
    return GM_ERR_INVALID;
  }
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("pk dump: bad rank / world");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  // slice table: (count, first point byte) of each of the five WriteSlice records
  const size_t expect[5] = {meta->nbA, meta->nbB, meta->domain_size - 1, meta->nbK, meta->nbB};
  uint64_t pos[5];
  uint64_t off = offset;
  for (int a = 0; a < 5; a++) {
    uint64_t cnt = 0;
    uint8_t le[8];
    if (int rc = read_at(fd, le, 8, off)) return rc;
    for (int b = 7; b >= 0; b--) cnt = (cnt << 8) | le[b];
    if (cnt != expect[a]) {
      set_error("pk dump: slice " + std::to_string(a) + " holds " + std::to_string(cnt) + " points, expected " +
                std::to_string(expect[a]));
      return GM_ERR_INVALID;
    }
    pos[a] = off + 8;
    off = pos[a] + cnt * 2 * (a == PK_B2 ? 2 : 1) * fp_bytes(curve);
  }
  Ranges rg;
  shard_range(meta->nbA, rank, world, &rg.loA, &rg.hiA);
  shard_range(meta->nbB, rank, world, &rg.loB, &rg.hiB);
  shard_range(meta->nbK, rank, world, &rg.loK, &rg.hiK);
  shard_range(meta->domain_size - 1, rank, world, &rg.loZ, &rg.hiZ);
  rg.rebase = false;
  IoRing ring;
  if (int rc = ring.init(true)) return rc;
  const size_t lo[5] = {rg.loA, rg.loB, rg.loZ, rg.loK, rg.loB};
  PointSource src = [&](int which, size_t count, bool g2, const MsmPrecomp* pre, void* dst) -> int {
    const size_t pb = 2 * (g2 ? 2 : 1) * fp_bytes(curve);
    int rc = stream_points(ctx, ring, curve, g2, fd, pos[which] + lo[which] * pb, count, pre, dst);
    if (rc) return rc;
    GM_HIP(hipStreamSynchronize(ctx->stream));
    return GM_OK;
  };
  int rc = pk_upload_ranges(ctx, curve, meta, flags, rg, out, &src);
  if (rc == GM_OK && end_offset) *end_offset = off;
  return rc;
}

int gm_g16_pk_upload_dump(gm_ctx* ctx, int curve, const gm_g16_pk_host* meta, int fd, uint64_t offset,
                          unsigned flags, uint64_t* end_offset, gm_g16_pk** out) {
  return gm_g16_pk_upload_dump_shard(ctx, curve, meta, fd, offset, flags, 0, 1, end_offset, out);
}

int gm_g16_pk_save_cache(gm_ctx* ctx, const gm_g16_pk* pk, int fd) {
  if (!ctx || !pk || fd < 0) return GM_ERR_INVALID;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  CacheHeader h;
  memset(&h, 0, sizeof(h));
  memcpy(h.magic, CACHE_MAGIC, 8);
  h.version = CACHE_VERSION;
  h.layout = CACHE_LAYOUT;
  h.wshare = (pk->wshare[0] ? 1u : 0u) | (pk->wshare[1] ? 2u : 0u) | (pk->wshare[2] ? 4u : 0u);
  h.curve = (uint32_t)pk->curve;
  h.n = pk->n;
  h.nb_wires = pk->nb_wires;
  h.nb_public = pk->nb_public;
  h.nbA = pk->nbA;
  h.nbB = pk->nbB;
  h.nbK = pk->nbK;
  h.zlo = pk->zlo;
  h.nbZ = pk->nbZ;
  h.wlo = pk->wlo;
  h.whi = pk->whi;
  h.precomp = pk->precomp;
  const MsmPrecomp* pres[4] = {&pk->preA, &pk->preB, &pk->preZ, &pk->preK};
  for (int i = 0; i < 4; i++) {
    h.pre_c[i] = pres[i]->c;
    h.pre_W[i] = pres[i]->W;
    h.pre_stride[i] = pres[i]->stride;
  }
  int rc;
  if ((rc = write_seq(fd, &h, sizeof(h)))) return rc;
  for (const auto* v : {&pk->alpha, &pk->beta, &pk->delta, &pk->beta2, &pk->delta2})
    if ((rc = write_seq(fd, v->data(), v->size()))) return rc;
  IoRing ring;
  if ((rc = ring.init(false))) return rc;
  for (int a = 0; a < 8; a++) {
    const size_t bytes = array_bytes(pk, a);
    const uint64_t b64 = bytes;
    if ((rc = write_seq(fd, &b64, 8))) return rc;
    const char* src = (const char*)*array_ptr(const_cast<gm_g16_pk*>(pk), a);
    for (size_t o = 0; o < bytes; o += IO_CHUNK) {
      const size_t cnt = std::min(IO_CHUNK, bytes - o);
      GM_HIP(hipMemcpy(ring.host[0], src + o, cnt, hipMemcpyDeviceToHost));
      if ((rc = write_seq(fd, ring.host[0], cnt))) return rc;
    }
  }
  return GM_OK;
}

int gm_g16_pk_load_cache(gm_ctx* ctx, int fd, gm_g16_pk** out) {
  if (!ctx || !out || fd < 0) return GM_ERR_INVALID;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  CacheHeader h;
  int rc;
  if ((rc = read_seq(fd, &h, sizeof(h)))) return rc;
  if (memcmp(h.magic, CACHE_MAGIC, 8) || h.version != CACHE_VERSION) {
    set_error("pk cache: not a gnark_mi355x device-layout key (magic / version)");
    return GM_ERR_INVALID;
  }
  if (h.layout != CACHE_LAYOUT) {
    set_error("pk cache: written by a build with another device point layout");
    return GM_ERR_INVALID;
  }
  if ((rc = check_curve_id((int)h.curve))) return rc;
  if ((rc = check_cache_header(h))) return rc;
  auto* pk = new gm_g16_pk();
  auto fail = [&](int code) {
    pk_release(pk);
    return code;
  };
  pk->curve = (int)h.curve;
  pk->n = h.n;
  pk->nb_wires = h.nb_wires;
  pk->nb_public = h.nb_public;
  pk->nbA = h.nbA;
  pk->nbB = h.nbB;
  pk->nbK = h.nbK;
  pk->zlo = h.zlo;
  pk->nbZ = h.nbZ;
  pk->wlo = h.wlo;
  pk->whi = h.whi;
  pk->precomp = h.precomp != 0;
  MsmPrecomp* pres[4] = {&pk->preA, &pk->preB, &pk->preZ, &pk->preK};
  const int frbits = pk->curve == GM_BN254 ? CurveBN254::FR_BITS : CurveBLS12377::FR_BITS;
  for (int i = 0; i < 4; i++) {
    pres[i]->c = h.pre_c[i];
    pres[i]->W = h.pre_W[i];
    pres[i]->narrow = precomp_narrow(h.pre_c[i], h.pre_W[i], frbits);  // layout 2 (CACHE_LAYOUT)
    pres[i]->stride = h.pre_stride[i];
  }
  for (int x = 0; x < 3; x++) pk->wshare[x] = (h.wshare >> x) & 1;
  if (pk->precomp && h.wshare) {
    // the wire plan's window geometry is the one the wire-indexed arrays were
    // built with (their header fields), not a re-derivation by this build's
    // window cost model: a cache stays loadable when the chooser changes.  The
    // shared arrays must agree with each other and span the wire slice.
    const MsmPrecomp* shared[3] = {&pk->preA, &pk->preB, &pk->preK};
    int first = -1;
    for (int x = 0; x < 3; x++)
      if (pk->wshare[x] && first < 0) first = x;
    pk->preW = *shared[first];
    for (int x = 0; x < 3; x++)
      if (pk->wshare[x] && (shared[x]->c != pk->preW.c || shared[x]->W != pk->preW.W ||
                            shared[x]->narrow != pk->preW.narrow || shared[x]->stride != pk->whi - pk->wlo)) {
        set_error("pk cache: wire-indexed arrays with different window geometries");
        return fail(GM_ERR_INVALID);
      }
  }
  const size_t g1b = 2 * fp_bytes(pk->curve), g2b = 4 * fp_bytes(pk->curve);
  for (auto* v : {&pk->alpha, &pk->beta, &pk->delta}) v->resize(g1b);
  for (auto* v : {&pk->beta2, &pk->delta2}) v->resize(g2b);
  for (auto* v : {&pk->alpha, &pk->beta, &pk->delta, &pk->beta2, &pk->delta2})
    if ((rc = read_seq(fd, v->data(), v->size()))) return fail(rc);
  IoRing ring;
  if ((rc = ring.init(false))) return fail(rc);
  for (int a = 0; a < 8; a++) {
    uint64_t b64;
    if ((rc = read_seq(fd, &b64, 8))) return fail(rc);
    const size_t bytes = array_bytes(pk, a);
    if (b64 != bytes) {
      set_error("pk cache: array " + std::to_string(a) + " size mismatch");
      return fail(GM_ERR_INVALID);
    }
    void** dst = array_ptr(pk, a);
    if (hipMalloc(dst, bytes ? bytes : 16) != hipSuccess) {
      set_error("pk cache: hipMalloc failed");
      return fail(GM_ERR_OOM);
    }
    // the compaction maps (arrays 5-7) index the wire slice: k_gather_fr reads
    // wires[idx] unchecked, so every entry is checked here on the host
    const uint32_t wspan = (uint32_t)(pk->whi - pk->wlo);
    for (size_t o = 0, k = 0; o < bytes; o += IO_CHUNK, k ^= 1) {
      const size_t cnt = std::min(IO_CHUNK, bytes - o);
      if ((rc = ring.acquire((int)k))) return fail(rc);
      if ((rc = read_seq(fd, ring.host[k], cnt))) return fail(rc);
      if (a >= 5) {
        const uint32_t* ix = (const uint32_t*)ring.host[k];
        for (size_t j = 0; j < cnt / 4; j++)
          if (ix[j] >= wspan) {
            set_error("pk cache: compaction index outside the wire slice");
            return fail(GM_ERR_INVALID);
          }
      }
      if (hipMemcpyAsync((char*)*dst + o, ring.host[k], cnt, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
          hipEventRecord(ring.ev[k], ctx->stream) != hipSuccess) {
        set_error("pk cache: H2D failed");
        return fail(GM_ERR_DEVICE);
      }
    }
  }
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return fail(GM_ERR_DEVICE);
  pk_prepare_h(ctx, pk);
  *out = pk;
  return GM_OK;
}

// ---- staged inputs ----------------------------------------------------------
}  // extern "C"

// a key's parked stage leaves its context's list (reused or released)
static void spare_unlist(gm_g16_pk* pk) {
  if (!pk->spare_stage) return;
  auto& v = pk->spare_stage->ctx->spare_keys;
  v.erase(std::remove(v.begin(), v.end(), pk), v.end());
}

void gm::stage_spare_release(gm_g16_pk* pk) {
  if (pk->spare_stage) {
    spare_unlist(pk);
    delete pk->spare_stage;
    pk->spare_stage = nullptr;
  }
}

extern "C" {

int gm_g16_stage_begin(gm_ctx* ctx, gm_g16_pk* pk, size_t nb_constraints, gm_g16_stage** out) {
  if (!ctx || !pk || !out) return GM_ERR_INVALID;
  if (nb_constraints > pk->n) {
    set_error("stage: more constraints than the domain size");
    return GM_ERR_INVALID;
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  if (gm_g16_stage* sp = pk->spare_stage; sp && sp->ctx == ctx) {
    // the key's buffers of a previous proof (gm_g16_stage_free parked them)
    spare_unlist(pk);
    pk->spare_stage = nullptr;
    sp->nc = nb_constraints;
    for (int v = 0; v < 3; v++) sp->len[v] = nb_constraints;
    sp->next = 0;
    sp->open = -1;
    sp->open_cnt = 0;
    for (bool& u : sp->used) u = false;
    *out = sp;
    return GM_OK;
  }
  auto* st = new gm_g16_stage();
  st->ctx = ctx;
  st->pk = pk;
  st->nc = nb_constraints;
  const size_t lens[4] = {pk->n, pk->n, pk->n, pk->nb_wires};
  for (int v = 0; v < 4; v++) {
    st->len[v] = v < 3 ? nb_constraints : pk->nb_wires;
    if (hipMalloc(&st->vec[v], 32 * (lens[v] ? lens[v] : 1)) != hipSuccess) {
      delete st;
      set_error("stage: hipMalloc failed");
      return GM_ERR_OOM;
    }
  }
  for (int i = 0; i < gm_g16_stage::SLOTS; i++) {
    if (hipHostMalloc(&st->host[i], gm_g16_stage::SLOT, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&st->dev[i], gm_g16_stage::SLOT) != hipSuccess ||
        hipEventCreateWithFlags(&st->ev[i], hipEventDisableTiming) != hipSuccess) {
      delete st;
      set_error("stage: staging allocation failed");
      return GM_ERR_OOM;
    }
  }
  *out = st;
  return GM_OK;
}

int gm_g16_stage_put_range(gm_g16_stage* st, int which, size_t lo, size_t count, const void* host_src) {
  if (!st || which < 0 || which > 3 || (count && !host_src)) return GM_ERR_INVALID;
  if (lo > st->len[which] || count > st->len[which] - lo) {
    set_error("stage: range outside the vector");
    return GM_ERR_INVALID;
  }
  gm_ctx* ctx = st->ctx;
  gm::CtxLock g(ctx);
  if (int rc = st->flush()) return rc;  // earlier indexed puts land first
  GM_HIP(hipSetDevice(ctx->device));
  const size_t per = gm_g16_stage::SLOT / 32;
  for (size_t o = 0; o < count; o += per) {
    const size_t cnt = std::min(per, count - o);
    int k;
    if (int rc = st->take(&k)) return rc;
    par_memcpy(st->host[k], (const char*)host_src + 32 * o, 32 * cnt, H2D_FILL_THREADS);
    GM_HIP(hipMemcpyAsync((char*)st->vec[which] + 32 * (lo + o), st->host[k], 32 * cnt, hipMemcpyHostToDevice,
                          ctx->copy));
    GM_HIP(hipEventRecord(st->ev[k], ctx->copy));
  }
  return GM_OK;
}

int gm_g16_stage_put_indexed(gm_g16_stage* st, int which, const void* host_base, const uint32_t* idx, size_t k) {
  if (!st || which < 0 || which > 3 || (k && (!host_base || !idx))) return GM_ERR_INVALID;
  if (k == 0) return GM_OK;
  std::lock_guard<std::recursive_mutex> g(st->ctx->mu);  // nothing queued on ctx->stream
  constexpr size_t per = gm_g16_stage::REC_PER;
  const char* base = (const char*)host_base;
  const size_t lim = st->len[which];
  for (size_t o = 0; o < k;) {
    if (st->open < 0) {
      int s;
      if (int rc = st->take(&s)) return rc;
      st->open = s;
    }
    uint2* hr = (uint2*)st->host[st->open];
    char* hv = (char*)st->host[st->open] + 8 * per;
    size_t j = st->open_cnt;
    const size_t end = std::min(k, o + (per - j));
    for (; o < end; o++, j++) {
      const uint32_t i = idx[o];
      if (i >= lim) {
        st->open_cnt = j;
        set_error("stage: index outside the vector");
        return GM_ERR_INVALID;
      }
      hr[j] = make_uint2(i, (uint32_t)which);
      memcpy(hv + 32 * j, base + 32 * (size_t)i, 32);
    }
    st->open_cnt = j;
    if (j == per)
      if (int rc = st->flush()) return rc;
  }
  if (st->open_cnt >= gm_g16_stage::FLUSH_AT) return st->flush();
  return GM_OK;
}

int gm_g16_stage_prove(gm_g16_stage* st, const void* r, const void* s, void* ar_out, void* bs_out, void* krs_out) {
  if (!st) return GM_ERR_INVALID;
  gm_ctx* ctx = st->ctx;
  {
    gm::CtxLock g(ctx);
    if (int rc = st->flush()) return rc;
    GM_HIP(hipSetDevice(ctx->device));
    GM_HIP(hipStreamSynchronize(ctx->copy));
  }
  return gm_g16_prove_device(ctx, st->pk, st->vec[3], st->vec[0], st->vec[1], st->vec[2], st->nc, r, s, ar_out,
                             bs_out, krs_out);
}

int gm_g16_stage_prove_r1cs(gm_g16_stage* st, const gm_r1cs* r1, const void* r, const void* s, void* ar_out,
                            void* bs_out, void* krs_out) {
  if (!st || !r1 || !r || !s || !ar_out || !bs_out || !krs_out) return GM_ERR_INVALID;
  gm_ctx* ctx = st->ctx;
  if (!r1cs_matches_key(st->pk, r1)) {
    set_error("stage_prove_r1cs: constraint system does not match the proving key (constraints <= n, same wires, "
              "whole key)");
    return GM_ERR_INVALID;
  }
  {
    gm::CtxLock g(ctx);
    if (int rc = st->flush()) return rc;
    GM_HIP(hipSetDevice(ctx->device));
    GM_HIP(hipStreamSynchronize(ctx->copy));
  }
  // the stage's a / b / c vectors (n each) receive the R1CS evaluation
  return g16_prove_r1cs_device(ctx, st->pk, r1, st->vec[3], st->vec[0], st->vec[1], st->vec[2], r, s, ar_out,
                               bs_out, krs_out);
}

int gm_g16_stage_free(gm_g16_stage* st) {
  if (!st) return GM_OK;
  gm::CtxLock g(st->ctx);
  st->open = -1;  // records not yet queued are dropped with the stage
  st->open_cnt = 0;
  hipSetDevice(st->ctx->device);
  hipStreamSynchronize(st->ctx->copy);
  // Park the buffers with the key for its next proof (one spare per key): a
  // fresh stage is 4 hipMallocs of up to n Fr plus 4 x 16 MiB of pinned host
  // memory.  The prove that used them has returned, so nothing reads them.
  if (!st->pk->spare_stage && !getenv_flag_off("GM_G16_STAGE_REUSE")) {
    st->pk->spare_stage = st;
    st->ctx->spare_keys.push_back(st->pk);
    return GM_OK;
  }
  delete st;
  return GM_OK;
}

}  // extern "C"
