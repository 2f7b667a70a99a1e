// load_width.hip -- streaming read rate by load width: each wave reads a
// contiguous 64 KiB piece per ticket-free iteration (like e4_size_kernel's
// walk), 8-byte lanes with 8 steps of loads in flight against 16-byte lanes
// with 4 (the same bytes in flight), nontemporal, plus a light per-word ALU
// sink.  hipcc -O3 --offload-arch=gfx950 tools/micro/load_width.hip -o /tmp/lw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int W, int PF>
__global__ __launch_bounds__(256, 8) void rd(const uint8_t *__restrict__ in, uint64_t pieces, uint32_t piece_bytes,
                                              uint32_t *out) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  uint32_t acc = 0;
  for (uint64_t p = wave; p < pieces; p += nw) {
    const uint8_t *src = in + p * piece_bytes;
    const uint32_t steps = piece_bytes / (64 * W);
    if (W == 8) {
      uint64_t v[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) v[j] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(src) + j * 64 + lane);
      for (uint32_t s0 = 0; s0 < steps; s0 += PF) {
        uint64_t vn[PF];
#pragma unroll
        for (int j = 0; j < PF; ++j)
          vn[j] = s0 + PF + j < steps ? __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(src) + (s0 + PF + j) * 64 + lane) : 0;
#pragma unroll
        for (int j = 0; j < PF; ++j) acc += __builtin_popcountll(v[j]);
#pragma unroll
        for (int j = 0; j < PF; ++j) v[j] = vn[j];
      }
    } else {
      typedef unsigned int u4 __attribute__((ext_vector_type(4)));
      u4 v[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) v[j] = __builtin_nontemporal_load(reinterpret_cast<const u4 *>(src) + j * 64 + lane);
      for (uint32_t s0 = 0; s0 < steps; s0 += PF) {
        u4 vn[PF];
#pragma unroll
        for (int j = 0; j < PF; ++j)
          vn[j] = s0 + PF + j < steps ? __builtin_nontemporal_load(reinterpret_cast<const u4 *>(src) + (s0 + PF + j) * 64 + lane) : u4{0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < PF; ++j) acc += __builtin_popcount(v[j].x) + __builtin_popcount(v[j].y) + __builtin_popcount(v[j].z) + __builtin_popcount(v[j].w);
#pragma unroll
        for (int j = 0; j < PF; ++j) v[j] = vn[j];
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t bytes = 16ull << 30;  // 16 GiB
  const uint32_t pb = 65536;
  uint8_t *in;
  uint32_t *out;
  if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(in, 0x5a, bytes);
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](auto k, const char *name) {
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k, dim3(8 * cus), dim3(256), 0, 0, in, bytes / pb, pb, out);
    hipEventRecord(a);
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, dim3(8 * cus), dim3(256), 0, 0, in, bytes / pb, pb, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms / 5, bytes / (ms / 5 * 1e-3) / 1e9);
  };
  run(rd<8, 8>, "8-byte lanes, 8 in flight");
  run(rd<8, 16>, "8-byte lanes, 16 in flight");
  run(rd<16, 4>, "16-byte lanes, 4 in flight");
  run(rd<16, 8>, "16-byte lanes, 8 in flight");
  return 0;
}
