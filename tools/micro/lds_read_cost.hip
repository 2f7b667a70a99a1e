// Microtest (gfx950): correctness and LDS-pipe cost of the read shapes a
// packed-record walk can use -- three byte reads (tag, c1, c9), one unaligned
// ds_read_b64 (+ a byte), one unaligned ds_read_b128, aligned b32/b64/b128 --
// at scattered per-lane byte positions inside a wave's 4 KiB window, 28 waves
// per CU (the decoder's occupancy).  Prints ns per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint4 __attribute__((aligned(1))) u4a1;
typedef uint2 __attribute__((aligned(1))) u2a1;

__device__ __forceinline__ uint8_t pat(uint32_t i) { return (uint8_t)((i * 2654435761u) >> 13); }

// kLayout 0: positions anywhere in the wave's window (random banks);
// 1: lane l's positions inside its own 56-byte chunk (as the chunk walks)
template <int kMode, int kLayout>
__global__ __attribute__((target("unaligned-access-mode"))) __launch_bounds__(256, 7) void cost(
    uint32_t *out, int iters, uint32_t seed, uint32_t *bad) {
  __shared__ __attribute__((aligned(16))) uint8_t s[4 * 4352];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  uint8_t *win = s + w * 4352;
  for (int i = l; i < 4352; i += 64) win[i] = pat(i);
  __syncthreads();
  uint32_t acc = 0, x = seed * 747796405u + t * 2891336453u;
  for (int i = 0; i < iters; ++i) {
    x = x * 1664525u + 1013904223u;
    uint32_t p = kLayout == 0 ? (x >> 20) % 4096u : l * 56u + (x >> 26) % 56u;
    uint32_t v;
    if (kMode == 0) {  // three byte reads
      v = win[p] | (win[p + 1] << 8) | (win[p + 9] << 16);
    } else if (kMode == 1) {  // unaligned b64 + byte
      const uint2 d = *(const u2a1 *)(win + p);
      v = d.x ^ d.y ^ win[p + 9];
    } else if (kMode == 2) {  // unaligned b128
      const uint4 d = *(const u4a1 *)(win + p);
      v = d.x ^ d.y ^ d.z ^ d.w;
    } else if (kMode == 3) {  // aligned b32
      v = *(const uint32_t *)(win + (p & ~3u));
    } else if (kMode == 4) {  // aligned b128
      const uint4 d = *(const uint4 *)(win + (p & ~15u));
      v = d.x ^ d.y ^ d.z ^ d.w;
    } else if (kMode == 5) {  // unaligned b64 only
      const uint2 d = *(const u2a1 *)(win + p);
      v = d.x ^ d.y;
    } else {  // aligned b64
      const uint2 d = *(const uint2 *)(win + (p & ~7u));
      v = d.x ^ d.y;
    }
    acc += v;
  }
  // correctness of the unaligned forms at every phase
  if (kMode == 1 || kMode == 2 || kMode == 5) {
    for (int ph = 0; ph < 16; ++ph) {
      const uint32_t p = (l * 61u + ph) % 4096u;
      const uint4 d = *(const u4a1 *)(win + p);
      const uint2 e = *(const u2a1 *)(win + p + 1);
      uint32_t want[4], want2[2];
      for (int k = 0; k < 4; ++k)
        want[k] = pat(p + 4 * k) | (pat(p + 4 * k + 1) << 8) | (pat(p + 4 * k + 2) << 16) |
                  ((uint32_t)pat(p + 4 * k + 3) << 24);
      for (int k = 0; k < 2; ++k)
        want2[k] = pat(p + 1 + 4 * k) | (pat(p + 2 + 4 * k) << 8) | (pat(p + 3 + 4 * k) << 16) |
                   ((uint32_t)pat(p + 4 + 4 * k) << 24);
      if (d.x != want[0] || d.y != want[1] || d.z != want[2] || d.w != want[3] || e.x != want2[0] ||
          e.y != want2[1])
        atomicAdd(bad, 1u);
    }
  }
  out[blockIdx.x * 256 + t] = acc;
}

template <int kMode, int kLayout>
static void run(const char *name, uint32_t *out, uint32_t *bad) {
  const int grid = 256 * 7 * 4, iters = 2048;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9f;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL((cost<kMode, kLayout>), dim3(grid), dim3(256), 0, 0, out, iters, (uint32_t)rep, bad);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  const double winst = (double)grid * 4 * iters;  // wave-level read groups
  printf("%-34s layout %d: %8.3f ms  %6.3f ns per read group per CU\n", name, kLayout, best,
         best * 1e6 * 256 / winst);
}

int main() {
  uint32_t *out, *bad;
  hipMalloc(&out, 256 * 7 * 4 * 256 * 4);
  hipMalloc(&bad, 4);
  hipMemset(bad, 0, 4);
  run<0, 0>("3 x u8 (tag, c1, c9)", out, bad);
  run<1, 0>("unaligned b64 + u8", out, bad);
  run<5, 0>("unaligned b64", out, bad);
  run<2, 0>("unaligned b128", out, bad);
  run<3, 0>("aligned b32", out, bad);
  run<6, 0>("aligned b64", out, bad);
  run<4, 0>("aligned b128", out, bad);
  run<0, 1>("3 x u8 (tag, c1, c9)", out, bad);
  run<1, 1>("unaligned b64 + u8", out, bad);
  run<5, 1>("unaligned b64", out, bad);
  run<2, 1>("unaligned b128", out, bad);
  run<3, 1>("aligned b32", out, bad);
  uint32_t hb = 0;
  hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("unaligned read mismatches: %u\n", hb);
  return hb ? 1 : 0;
}
