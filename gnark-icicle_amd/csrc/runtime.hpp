// Runtime plumbing for the C-ABI library: per-device context, stream, error
// reporting, workspace allocation and per-kernel HIP-event profiling.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/gnark_mi355x.h"

namespace gm {

void set_error(const std::string& msg);
std::string last_error();  // this thread's last error message
size_t fp_bytes(int curve);  // bytes of one base-field element (gnark layout)

#define GM_HIP(call)                                                                      \
  do {                                                                                    \
    hipError_t _e = (call);                                                               \
    if (_e != hipSuccess) {                                                               \
      ::gm::set_error(std::string(#call) + ": " + hipGetErrorString(_e) + " @" __FILE__ \
                      ":" + std::to_string(__LINE__));                                    \
      return GM_ERR_DEVICE;                                                               \
    }                                                                                     \
  } while (0)

struct KernelStat {
  double total_ms = 0;
  uint64_t count = 0;
};

// One bump-allocated workspace: chunks of hipMalloc'd memory (see Arena).
struct ArenaState {
  struct Chunk {
    char* base;
    size_t cap;
  };
  std::vector<Chunk> chunks;
  size_t cur_chunk = 0, cur_top = 0;
};

}  // namespace gm

struct gm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t aux = nullptr;   // second stream: work overlapped with `stream` inside one call
  hipStream_t copy = nullptr;  // host->device input copies overlapped with kernels
  // pinned host staging for small device->host readbacks (truly async copies)
  void* pinned = nullptr;
  size_t pinned_cap = 0;
  std::recursive_mutex mu;
  // per-kernel profiling with HIP events on this context's stream
  bool profiling = false;
  struct Pending {
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> event_pool;
  std::map<std::string, gm::KernelStat> stats;
  // Wave stamps of profiled accumulation launches: entry i of this device ring gets
  // the wall clock of the launch's first wave start (atomicMin) and last wave end
  // (atomicMax), i.e. its execution without the time the launch waited for wave
  // slots.  Read back by gm_profile_get / _dump / _reset (stamp_collect).
  // 64 stamp pairs per launch, 256 B apart (one per L2 line: waves stamp the pair of
  // their block index mod 64, so no address takes more than 1/64 of the atomics)
  static constexpr size_t STAMP_CAP = 1024, STAMP_SLOTS = 64, STAMP_STRIDE = 32;
  static constexpr size_t STAMP_WORDS = STAMP_SLOTS * STAMP_STRIDE;  // u64 per launch
  unsigned long long* stamp_dev = nullptr;
  size_t stamp_next = 0;
  std::vector<std::pair<std::string, size_t>> stamp_pending;
  double wall_khz = 0;
  // cached NTT domains: key = curve*64 + logn
  std::map<int, void*> ntt_domains;
  int msm_c_override = 0;
  int msm_glv = -1;   // GLV split of plain MSMs: -1 = default (n <= 2^21), 0 off, 1 on
  // workspace arena (stack-discipline scopes), plus two more for MSMs whose host
  // tail is deferred (pipelined MSMs: gm_msm_async, the Groth16 MSM sequence)
  gm::ArenaState arena;
  // MSM_SLOTS in-flight MSMs (gm_msm_async; the Groth16 sequence uses two)
  static constexpr int MSM_SLOTS = 3;
  gm::ArenaState slots[MSM_SLOTS];
  bool slot_busy[MSM_SLOTS] = {};
  // pinned readback buffers of deferred MSM tails; a buffer stays busy from
  // msm_readback until its MSM's msm_finish (or the tail's destruction), so
  // synchronous MSMs issued while async ones are pending never reuse it
  static constexpr int TAIL_BUFS = 8;
  void* tail_pinned[TAIL_BUFS] = {};
  bool tail_busy[TAIL_BUFS] = {};
  // one stream per slot (gm_msm_async): independent MSMs in flight overlap on
  // the device -- one's sort / reduction (HBM / latency-bound) runs beside
  // another's accumulation (VALU-bound).  Created on first use.
  hipStream_t slot_stream[MSM_SLOTS] = {};
  // Bucket accumulations of in-flight async MSMs run one after another: each one's
  // slot stream waits on `acc_tail`, recorded after the previous accumulation.
  // Only the accumulation is ordered; the sorts and reductions of the other MSMs
  // still run beside it.  `acc_chain` is set while gm_msm_async queues its MSM.
  hipEvent_t acc_tail = nullptr;
  bool acc_chain = false;
  // the Groth16 prove's second MSM stream (GM_G16_MSM_STREAMS=1), created on first use
  hipStream_t g16_stream = nullptr;
  // gm_msm_async handles not yet waited for: gm_destroy drains their device work,
  // releases their slot / readback buffer and orphans them (gm_msm_wait then
  // fails with GM_ERR_INVALID and frees the handle)
  std::vector<gm_msm_pending*> live_msms;
  // "inputs read" events of pending gm_msm_async MSMs (recorded on their slot
  // streams after the digits and the point conversion).  Work queued later on
  // ctx->stream must not overwrite those inputs first: every API call that may
  // queue on ctx->stream takes the context through CtxLock, which makes
  // ctx->stream wait on these events first.  gm_msm_async / gm_msm_wait put
  // nothing on ctx->stream, so back-to-back async MSMs never meet a packet of
  // it in a hardware queue they share.
  std::vector<std::pair<const void*, hipEvent_t>> pending_reads;
  // a / b / c of a host-input prove (gm_g16_prove): their own allocation, outside
  // the workspace arena.  The runtime orders a pageable copy into an allocation
  // after the queued commands that use the same allocation, so copies into an
  // arena chunk shared with MSM scratch waited for the running MSMs (2^24: the
  // copies ran after the B2 MSM, +35 ms, profiles/r04s_g16_host_slow_copies.txt).
  void* in_abc = nullptr;
  size_t in_abc_cap = 0;
  // pinned ring the host-input prove's helper thread copies a / b / c through
  // (HostStagedH): created on first use, kept
  static constexpr int H2D_SLOTS = 4;
  static constexpr size_t H2D_SLOT = size_t(32) << 20;
  void* h2d_pin[H2D_SLOTS] = {};
  hipEvent_t h2d_ev[H2D_SLOTS] = {};
  // keys holding a parked stage of this context (gm_g16_stage_free): gm_trim
  // releases those stages' buffers
  std::vector<gm_g16_pk*> spare_keys;
};

namespace gm {

// Records a kernel launch bracketed by events when profiling is enabled.
// kernel = true: the events are not recorded on the stream; the scope's one
// kernel is launched with hipExtLaunchKernelGGL(..., a, b, ...), which stamps
// them with the kernel's own start and end (its execution, not the time it
// waited in the queue for wave slots another stream's kernels held).
struct ProfScope {
  gm_ctx* ctx;
  const char* name;
  bool kernel;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(gm_ctx* c, const char* n, bool k = false) : ctx(c), name(n), kernel(k) {
    if (!ctx->profiling) return;
    a = take();
    b = take();
    if (!kernel) hipEventRecord(a, ctx->stream);
  }
  ~ProfScope() {
    if (!ctx->profiling) return;
    if (!kernel) hipEventRecord(b, ctx->stream);
    ctx->pending.push_back({name, a, b});
  }
  // device pair for the launch's wave stamps (nullptr when not profiling), its
  // execution time collected as `exec_name`
  unsigned long long* wave_stamp(const char* exec_name);
  hipEvent_t take() {
    if (!ctx->event_pool.empty()) {
      hipEvent_t e = ctx->event_pool.back();
      ctx->event_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
  }
};

// Wave-stamp ring: (re)initialised to {max, 0} pairs; collected into ctx->stats
// after the device is idle.
inline int stamp_reset(gm_ctx* ctx, size_t launches) {
  std::vector<unsigned long long> init(gm_ctx::STAMP_WORDS * launches, 0ull);
  for (size_t i = 0; i < launches * gm_ctx::STAMP_SLOTS; i++) init[i * gm_ctx::STAMP_STRIDE] = ~0ull;
  return hipMemcpy(ctx->stamp_dev, init.data(), init.size() * sizeof(init[0]), hipMemcpyHostToDevice) == hipSuccess
             ? GM_OK
             : GM_ERR_DEVICE;
}
inline void stamp_collect(gm_ctx* ctx) {
  if (ctx->stamp_pending.empty()) return;
  const size_t used = ctx->stamp_next;
  std::vector<unsigned long long> v(gm_ctx::STAMP_WORDS * used);
  if (hipDeviceSynchronize() == hipSuccess &&
      hipMemcpy(v.data(), ctx->stamp_dev, v.size() * sizeof(v[0]), hipMemcpyDeviceToHost) == hipSuccess) {
    for (auto& p : ctx->stamp_pending) {
      unsigned long long t0 = ~0ull, t1 = 0;
      for (size_t k = 0; k < gm_ctx::STAMP_SLOTS; k++) {
        const unsigned long long* q = &v[p.second * gm_ctx::STAMP_WORDS + k * gm_ctx::STAMP_STRIDE];
        t0 = std::min(t0, q[0]);
        t1 = std::max(t1, q[1]);
      }
      if (t1 <= t0 || t0 == ~0ull) continue;  // launch without waves
      auto& s = ctx->stats[p.first];
      s.total_ms += (double)(t1 - t0) / ctx->wall_khz;
      s.count += 1;
    }
  }
  ctx->stamp_pending.clear();
  ctx->stamp_next = 0;
  stamp_reset(ctx, used);
}
// the ring, allocated when profiling is switched on (gm_profile_enable), not
// inside a profiled call; false: no stamps (the event brackets remain)
inline bool stamp_ensure(gm_ctx* ctx) {
  if (ctx->stamp_dev) return true;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess || khz <= 0)
    return false;
  if (hipMalloc(&ctx->stamp_dev, gm_ctx::STAMP_WORDS * gm_ctx::STAMP_CAP * sizeof(unsigned long long)) !=
      hipSuccess) {
    ctx->stamp_dev = nullptr;
    return false;
  }
  ctx->wall_khz = khz;
  if (stamp_reset(ctx, gm_ctx::STAMP_CAP)) {
    hipFree(ctx->stamp_dev);
    ctx->stamp_dev = nullptr;
    return false;
  }
  return true;
}
#ifndef GM_WAVE_STAMPS
#define GM_WAVE_STAMPS 1
#endif
inline unsigned long long* ProfScope::wave_stamp(const char* exec_name) {
  if (!GM_WAVE_STAMPS || !ctx->profiling || !stamp_ensure(ctx)) return nullptr;
  if (ctx->stamp_next == gm_ctx::STAMP_CAP) stamp_collect(ctx);
  const size_t i = ctx->stamp_next++;
  ctx->stamp_pending.push_back({exec_name, i});
  return ctx->stamp_dev + gm_ctx::STAMP_WORDS * i;
}

// Drain finished profiling records (call after stream synchronisation).
inline void prof_collect(gm_ctx* ctx) {
  for (auto& p : ctx->pending) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      auto& s = ctx->stats[p.name];
      s.total_ms += ms;
      s.count += 1;
    }
    ctx->event_pool.push_back(p.a);
    ctx->event_pool.push_back(p.b);
  }
  ctx->pending.clear();
}

// Workspace arena scope.  All scratch of one API call is carved from the
// context's chunk list with a bump pointer and released (LIFO) when the scope
// ends.  Chunks stay allocated for reuse by later calls (no per-call
// hipMalloc / hipFree on the hot path).  Calls on a context are serialised and
// stream-synchronous, so a released range is never still in use by a kernel.
struct Arena {
  gm_ctx* ctx;
  ArenaState* st;
  size_t saved_chunk, saved_top;
  explicit Arena(gm_ctx* c, ArenaState* s = nullptr)
      : ctx(c), st(s ? s : &c->arena), saved_chunk(st->cur_chunk), saved_top(st->cur_top) {}
  ~Arena() {
    st->cur_chunk = saved_chunk;
    st->cur_top = saved_top;
  }
  Arena(const Arena&) = delete;
  Arena& operator=(const Arena&) = delete;
  int alloc(size_t bytes, void** out) {
    bytes = (bytes + 255) & ~size_t(255);
    if (bytes == 0) bytes = 256;
    while (st->cur_chunk < st->chunks.size()) {
      auto& ch = st->chunks[st->cur_chunk];
      if (st->cur_top + bytes <= ch.cap) {
        *out = ch.base + st->cur_top;
        st->cur_top += bytes;
        return GM_OK;
      }
      st->cur_chunk++;
      st->cur_top = 0;
    }
    size_t cap = bytes;
    size_t last = st->chunks.empty() ? 0 : st->chunks.back().cap;
    if (cap < 2 * last) cap = 2 * last;
    if (cap < (size_t(64) << 20)) cap = size_t(64) << 20;
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, cap);
    if (e != hipSuccess) {
      // retry with the exact size
      e = hipMalloc(&p, bytes);
      cap = bytes;
      if (e != hipSuccess) {
        set_error(std::string("workspace hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
        return GM_ERR_OOM;
      }
    }
    st->chunks.push_back({(char*)p, cap});
    st->cur_chunk = st->chunks.size() - 1;
    st->cur_top = bytes;
    *out = p;
    return GM_OK;
  }
};

// ctx->stream waits until every pending async MSM has read its inputs (see
// gm_ctx::pending_reads); a failed wait falls back to a host wait.
inline void flush_pending_reads(gm_ctx* c) {
  if (c->pending_reads.empty()) return;
  hipSetDevice(c->device);
  for (auto& pr : c->pending_reads) {
    if (hipStreamWaitEvent(c->stream, pr.second, 0) != hipSuccess) hipEventSynchronize(pr.second);
    hipEventDestroy(pr.second);
  }
  c->pending_reads.clear();
}
// The context's lock for API calls that may queue work on ctx->stream.
struct CtxLock {
  std::lock_guard<std::recursive_mutex> g;
  explicit CtxLock(gm_ctx* c) : g(c->mu) { flush_pending_reads(c); }
};

// Host-side fill of a pinned staging slot: memcpy split over `nt` threads.  One
// thread copies pageable memory at ~21 GB/s, below the ~57 GB/s DMA behind it
// (a 32 MiB slot: 1.55 ms of memcpy against 0.59 ms of copy,
// profiles/r05i_host_prove_timeline.txt).
inline void par_memcpy(void* dst, const void* src, size_t len, int nt) {
  if (nt <= 1 || len < (size_t(4) << 20)) {
    memcpy(dst, src, len);
    return;
  }
  const size_t part = (len / nt + 4095) & ~size_t(4095);
  std::vector<std::thread> ws;
  for (int i = 1; i < nt && (size_t)i * part < len; i++) {
    const size_t o = (size_t)i * part;
    try {
      ws.emplace_back([=] { memcpy((char*)dst + o, (const char*)src + o, std::min(part, len - o)); });
    } catch (...) {  // no thread to be had: this thread copies the remainder itself
      memcpy((char*)dst + o, (const char*)src + o, len - o);
      break;
    }
  }
  memcpy(dst, src, std::min(part, len));
  for (auto& w : ws) w.join();
}
// threads per pinned-slot fill (profiles/r05l_host_h_incremental_ab.txt)
constexpr int H2D_FILL_THREADS = 4;

// A deferred-tail arena slot of the context (at most MSM_SLOTS MSMs in flight).
// ctx->stream temporarily replaced (all MSM code queues on ctx->stream)
struct StreamSwap {
  gm_ctx* ctx;
  hipStream_t old;
  StreamSwap(gm_ctx* c, hipStream_t s) : ctx(c), old(c->stream) { c->stream = s; }
  ~StreamSwap() { ctx->stream = old; }
  StreamSwap(const StreamSwap&) = delete;
  StreamSwap& operator=(const StreamSwap&) = delete;
};

struct SlotArena {
  gm_ctx* ctx;
  int k = -1;
  Arena* a = nullptr;
  int take() {
    for (int i = 0; i < gm_ctx::MSM_SLOTS; i++)
      if (!ctx->slot_busy[i]) {
        k = i;
        ctx->slot_busy[i] = true;
        a = new Arena(ctx, &ctx->slots[i]);
        return GM_OK;
      }
    set_error("at most " + std::to_string(gm_ctx::MSM_SLOTS) + " MSMs may be in flight per context");
    return GM_ERR_INVALID;
  }
  void release() {
    if (a) {
      delete a;
      a = nullptr;
      ctx->slot_busy[k] = false;
    }
  }
  explicit SlotArena(gm_ctx* c) : ctx(c) {}
  ~SlotArena() { release(); }
  SlotArena(const SlotArena&) = delete;
  SlotArena& operator=(const SlotArena&) = delete;
};

// Pinned readback buffer of a deferred MSM tail: the first free one of the
// context's TAIL_BUFS 512 KiB buffers, marked busy until tail_pinned_release.
inline int tail_pinned_acquire(gm_ctx* ctx, size_t bytes, uint8_t** out, int* idx) {
  constexpr size_t CAP = size_t(512) << 10;
  if (bytes > CAP) {
    set_error("msm: readback larger than the tail buffer");
    return GM_ERR_INVALID;
  }
  for (int i = 0; i < gm_ctx::TAIL_BUFS; i++) {
    if (ctx->tail_busy[i]) continue;
    void*& b = ctx->tail_pinned[i];
    if (!b) {
      hipError_t e = hipHostMalloc(&b, CAP, hipHostMallocDefault);
      if (e != hipSuccess) {
        b = nullptr;
        set_error(std::string("hipHostMalloc: ") + hipGetErrorString(e));
        return GM_ERR_OOM;
      }
    }
    ctx->tail_busy[i] = true;
    *out = static_cast<uint8_t*>(b);
    *idx = i;
    return GM_OK;
  }
  set_error("msm: more than " + std::to_string(gm_ctx::TAIL_BUFS) + " MSM readbacks pending on one context");
  return GM_ERR_INVALID;
}
inline void tail_pinned_release(gm_ctx* ctx, int idx) {
  if (ctx && idx >= 0 && idx < gm_ctx::TAIL_BUFS) ctx->tail_busy[idx] = false;
}

// Pinned host staging of at least `bytes` (grown on demand; freed by gm_destroy).
inline int pinned_buf(gm_ctx* ctx, size_t bytes, void** out) {
  if (ctx->pinned_cap < bytes) {
    if (ctx->pinned) hipHostFree(ctx->pinned);
    ctx->pinned = nullptr;
    ctx->pinned_cap = 0;
    size_t cap = bytes < (size_t(256) << 10) ? (size_t(256) << 10) : bytes;
    hipError_t e = hipHostMalloc(&ctx->pinned, cap, hipHostMallocDefault);
    if (e != hipSuccess) {
      set_error(std::string("hipHostMalloc: ") + hipGetErrorString(e));
      return GM_ERR_OOM;
    }
    ctx->pinned_cap = cap;
  }
  *out = ctx->pinned;
  return GM_OK;
}

// A typed view of one arena allocation.
struct DevBuf {
  void* p = nullptr;
  int alloc(Arena& a, size_t bytes) { return a.alloc(bytes, &p); }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

inline unsigned blocks_for(size_t n, unsigned tpb) { return (unsigned)((n + tpb - 1) / tpb); }

}  // namespace gm
