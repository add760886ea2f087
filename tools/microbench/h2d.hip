// Host->device copy rates on the GPU box (pageable vs pinned vs a pinned
// staging ring fed by T host threads), 512 MiB = one 2^24 Fr vector.
//   hipcc -O3 --offload-arch=gfx950 h2d.hip -o h2d -lpthread && ./h2d
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
  const size_t B = size_t(512) << 20;
  std::vector<char> host(B);
  for (size_t i = 0; i < B; i += 4096) host[i] = (char)i;
  void* dev; CK(hipMalloc(&dev, B));
  hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int rep = 0; rep < 2; rep++) {
    double t = now();
    CK(hipMemcpyAsync(dev, host.data(), B, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st));
    printf("pageable hipMemcpyAsync: %.2f GB/s\n", B / (now() - t) / 1e9);
  }
  void* pin; CK(hipHostMalloc(&pin, B, hipHostMallocDefault));
  memcpy(pin, host.data(), B);
  for (int rep = 0; rep < 2; rep++) {
    double t = now();
    CK(hipMemcpyAsync(dev, pin, B, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st));
    printf("pinned hipMemcpyAsync: %.2f GB/s\n", B / (now() - t) / 1e9);
  }
  for (int T : {1, 2, 4, 8, 16}) {
    double t = now();
    std::vector<std::thread> th;
    for (int k = 0; k < T; k++) th.emplace_back([&, k] { size_t s = B / T * k; memcpy((char*)pin + s, host.data() + s, B / T); });
    for (auto& x : th) x.join();
    printf("memcpy %2d threads: %.2f GB/s\n", T, B / (now() - t) / 1e9);
  }
  // staging ring: T workers, each with 2 pinned slots of C bytes
  for (int T : {2, 4, 8}) for (size_t C : {size_t(4) << 20, size_t(16) << 20}) {
    std::vector<void*> slots(2 * T); std::vector<hipEvent_t> ev(2 * T);
    for (int i = 0; i < 2 * T; i++) { CK(hipHostMalloc(&slots[i], C, hipHostMallocDefault)); CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming)); }
    double t = now();
    std::vector<std::thread> th;
    const size_t nch = (B + C - 1) / C;
    for (int k = 0; k < T; k++) th.emplace_back([&, k] {
      int u = 0;
      for (size_t c = k; c < nch; c += T, u ^= 1) {
        const int s = 2 * k + u;
        hipEventSynchronize(ev[s]);
        const size_t off = c * C, len = std::min(C, B - off);
        memcpy(slots[s], host.data() + off, len);
        hipMemcpyAsync((char*)dev + off, slots[s], len, hipMemcpyHostToDevice, st);
        hipEventRecord(ev[s], st);
      }
    });
    for (auto& x : th) x.join();
    CK(hipStreamSynchronize(st));
    printf("ring T=%d chunk=%zuMB: %.2f GB/s\n", T, C >> 20, B / (now() - t) / 1e9);
    for (int i = 0; i < 2 * T; i++) { hipHostFree(slots[i]); hipEventDestroy(ev[i]); }
  }
  // register the pageable buffer in place
  double t = now();
  CK(hipHostRegister(host.data(), B, hipHostRegisterDefault));
  double t1 = now();
  CK(hipMemcpyAsync(dev, host.data(), B, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st));
  double t2 = now();
  CK(hipHostUnregister(host.data()));
  double t3 = now();
  printf("hipHostRegister %.2f ms, copy %.2f GB/s, unregister %.2f ms\n", (t1 - t) * 1e3, B / (t2 - t1) / 1e9, (t3 - t2) * 1e3);
  return 0;
}
