// Microtest: unaligned LDS b64/b32/b16 access correctness + cost (gfx950).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void check(uint64_t *out, int *bad) {
  __shared__ __attribute__((aligned(16))) uint8_t s[2048];
  const int t = threadIdx.x;
  for (int i = t; i < 2048; i += 64) s[i] = 0;
  __syncthreads();
  // each lane writes 8 bytes at byte offset 11*t + 5 (unaligned), non-overlapping? 11 > 8 yes
  uint64_t v = 0x0102030405060708ull * (uint64_t)(t + 1);
  __builtin_memcpy(s + 11 * t + 5, &v, 8);
  uint32_t w = 0xA1B2C3D4u ^ t;
  __builtin_memcpy(s + 1024 + 7 * t + 1, &w, 4);
  uint16_t h = (uint16_t)(0xBEEF ^ t);
  __builtin_memcpy(s + 1600 + 3 * t + 1, &h, 2);
  __syncthreads();
  uint64_t r;
  __builtin_memcpy(&r, s + 11 * t + 5, 8);
  uint32_t rw;
  __builtin_memcpy(&rw, s + 1024 + 7 * t + 1, 4);
  uint16_t rh;
  __builtin_memcpy(&rh, s + 1600 + 3 * t + 1, 2);
  // byte-level check
  int b = 0;
  for (int i = 0; i < 8; ++i) if (s[11 * t + 5 + i] != (uint8_t)(v >> (8 * i))) b++;
  if (r != v) b += 100;
  if (rw != w) b += 1000;
  if (rh != h) b += 10000;
  out[t] = r;
  if (b) atomicAdd(bad, b);
}

template <int kMode>
__global__ void cost(uint64_t *out, int iters, int seed) {
  __shared__ __attribute__((aligned(16))) uint8_t s[16384];
  const int t = threadIdx.x;
  uint64_t acc = 0;
  int o = (t * 5 + seed) & 1023;  // ~5-byte spacing: scattered like packed strings
  if (kMode == 1) o = t * 8;       // aligned
  uint64_t v = t;
  for (int i = 0; i < iters; ++i) {
    uint8_t *p = s + ((threadIdx.x >> 6) * 2048) + o + (i & 7);
    if (kMode == 1) p = s + ((threadIdx.x >> 6) * 2048) + o;
    __builtin_memcpy(p, &v, 8);
    v += 3;
  }
  __syncthreads();
  uint64_t r;
  __builtin_memcpy(&r, s + t * 8 + 1, 8);
  out[blockIdx.x * blockDim.x + t] = r + acc;
}

__global__ void tickets(uint32_t *ctr, uint32_t *sink, int per) {
  for (int i = 0; i < per; ++i) {
    uint32_t x = atomicAdd(ctr, 1u);
    if (x == 0xffffffffu) sink[0] = x;
  }
}

int main() {
  uint64_t *out; int *bad; uint32_t *ctr;
  hipMalloc(&out, 1 << 26); hipMalloc(&bad, 4); hipMalloc(&ctr, 64);
  hipMemset(bad, 0, 4);
  check<<<1, 64>>>(out, bad);
  int hb = -1; hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("unaligned LDS check: bad=%d\n", hb);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int m = 0; m < 2; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (m == 0) hipLaunchKernelGGL(cost<0>, dim3(2048), dim3(512), 0, 0, out, 4096, rep);
      else hipLaunchKernelGGL(cost<1>, dim3(2048), dim3(512), 0, 0, out, 4096, rep);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      double instr = 2048.0 * 8 * 4096;  // wave-instructions
      if (rep) printf("mode %s: %.3f ms, %.2f cycles per ds_write_b64 per CU (at 2.4GHz)\n",
                      m ? "aligned" : "unaligned", ms, ms * 1e-3 * 2.4e9 * 256 / instr);
    }
  }
  for (int rep = 0; rep < 2; ++rep) {
    hipMemset(ctr, 0, 4);
    hipEventRecord(a);
    tickets<<<8192, 64>>>(ctr, ctr + 8, 64);  // one atomic per wave per iter (lane-folded)
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    if (rep) printf("ticket: %.3f ms for %d wave-atomics -> %.1f per us\n", ms, 8192 * 64, 8192 * 64 / (ms * 1e3));
  }
  return 0;
}
