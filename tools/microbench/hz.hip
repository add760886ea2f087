#include <hip/hip_runtime.h>
#include <cstdint>
__global__ void k(uint32_t* io) {
  int t = threadIdx.x;
  uint32_t a[8], b[8], r[8];
  for (int i = 0; i < 8; i++) { a[i] = io[t*8+i]; b[i] = io[1024+t*8+i]; }
  unsigned c = 0;
  for (int i = 0; i < 8; i++) r[i] = __builtin_addc(a[i], b[i], c, &c);
  for (int i = 0; i < 8; i++) io[t*8+i] = r[i];
}
__global__ void k2(uint64_t* io, uint32_t* x) {
  int t = threadIdx.x;
  uint64_t acc = io[t]; uint32_t a = x[t], b = x[t+64], hi = 0;
  uint64_t p = (uint64_t)a*b;
  acc += p; hi += acc < p;
  uint64_t p2 = (uint64_t)a*a;
  acc += p2; hi += acc < p2;
  io[t] = acc; x[t] = hi;
}
