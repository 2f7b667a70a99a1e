// stream_mix.hip -- achievable HBM rate for the codec's read/write mixes:
// each wave streams contiguous 64 KiB input pieces (16-byte lanes, 4 steps of
// loads in flight, nontemporal, as the window loads) and writes R output
// bytes per input byte (16-byte nontemporal stores): R = 0 (read only),
// 0.5 (~config-2 encode: P = 0.47 U), 1 (config 3: P ~ U), 2 (~config-2
// decode: U = 2.1 P), plus write only (store width, temporal hint),
// hipMemset and hipMemcpy device-to-device.
// Rates count read + written bytes (what `roofline.achieved` counts).
//   hipcc -O3 --offload-arch=gfx950 -Wno-unused-value tools/micro/stream_mix.hip -o build/micro/stream_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// RN / RD: output bytes per input byte = RN / RD (RN = 0: read only;
// RD = 0: write only)
template <int RN, int RD>
__global__ __launch_bounds__(256, 8) void mix(const u4 *__restrict__ in, u4 *__restrict__ out, uint64_t pieces,
                                               uint32_t out_flag) {
  constexpr uint32_t kSteps = 65536 / (64 * 16);  // 64 steps of 1 KiB
  constexpr int PF = 4;
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  u4 acc = {0, 0, 0, 0};
  for (uint64_t p = wave; p < pieces; p += nw) {
    const u4 *src = in + p * (kSteps * 64);
    u4 *dst = out + (RD ? p * (kSteps * 64) * RN / RD : p * (kSteps * 64));
    u4 v[PF];
    if (RD) {
#pragma unroll
      for (int j = 0; j < PF; ++j) v[j] = __builtin_nontemporal_load(src + j * 64 + lane);
    }
    for (uint32_t s0 = 0; s0 < kSteps; s0 += PF) {
      u4 vn[PF];
      if (RD) {
#pragma unroll
        for (int j = 0; j < PF; ++j)
          vn[j] = s0 + PF + j < kSteps ? __builtin_nontemporal_load(src + (s0 + PF + j) * 64 + lane) : u4{0, 0, 0, 0};
      }
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const uint32_t s = s0 + j;
        const u4 x = RD ? v[j] : u4{s, (uint32_t)lane, 1u, 2u};
        if (RN == 0) {
          acc ^= x;
        } else if (RD == 0 || RN == RD) {  // write only / 1:1
          __builtin_nontemporal_store(x, dst + s * 64 + lane);
        } else if (2 * RN == RD) {  // 1:0.5 -- even steps' lanes write
          if (!(s & 1)) __builtin_nontemporal_store(x, dst + (s >> 1) * 64 + lane);
          else acc ^= x;
        } else {  // 1:2
          __builtin_nontemporal_store(x, dst + 2 * s * 64 + lane);
          __builtin_nontemporal_store(x ^ u4{1u, 1u, 1u, 1u}, dst + (2 * s + 1) * 64 + lane);
        }
      }
#pragma unroll
      for (int j = 0; j < PF; ++j) v[j] = vn[j];
    }
  }
  if (acc.x == out_flag) out[0] = acc;  // (never: keeps the reads)
}

// write only, store width / temporal hint variants
template <int W, bool NT>
__global__ __launch_bounds__(256, 8) void wr(u4 *__restrict__ out, uint64_t pieces) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  for (uint64_t p = wave; p < pieces; p += nw) {
    if (W == 16) {
      u4 *dst = out + p * 4096;
      for (uint32_t s = 0; s < 64; ++s) {
        const u4 x = {s, (uint32_t)lane, 1u, 2u};
        if (NT) __builtin_nontemporal_store(x, dst + s * 64 + lane);
        else dst[s * 64 + lane] = x;
      }
    } else {
      uint64_t *dst = reinterpret_cast<uint64_t *>(out) + p * 8192;
      for (uint32_t s = 0; s < 128; ++s) {
        const uint64_t x = ((uint64_t)s << 32) | (uint32_t)lane;
        if (NT) __builtin_nontemporal_store(x, dst + s * 64 + lane);
        else dst[s * 64 + lane] = x;
      }
    }
  }
}

int main() {
  const uint64_t in_bytes = 16ull << 30;  // 16 GiB of input pieces
  const uint64_t pieces = in_bytes / 65536;
  u4 *in, *out;
  if (hipMalloc(&in, in_bytes) != hipSuccess || hipMalloc(&out, 2 * in_bytes) != hipSuccess) return 1;
  hipMemset(in, 0x5a, in_bytes);
  hipMemset(out, 0, 2 * in_bytes);
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](auto k, const char *name, double rd, double wr) {
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k, dim3(8 * cus), dim3(256), 0, 0, in, out, pieces, 0xdeadbeefu);
    hipEventRecord(a);
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, dim3(8 * cus), dim3(256), 0, 0, in, out, pieces, 0xdeadbeefu);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double t = ms / 5 * 1e-3, bytes = (rd + wr) * (double)in_bytes;
    printf("%-34s %8.3f ms  %7.1f GB/s (read %.1f + write %.1f GB)\n", name, ms / 5, bytes / t / 1e9,
           rd * in_bytes / 1e9, wr * in_bytes / 1e9);
  };
  auto runw = [&](auto k, const char *name) {
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k, dim3(8 * cus), dim3(256), 0, 0, out, pieces);
    hipEventRecord(a);
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, dim3(8 * cus), dim3(256), 0, 0, out, pieces);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms / 5, (double)in_bytes / (ms / 5 * 1e-3) / 1e9);
  };
  runw(wr<16, true>, "write only, 16 B nontemporal");
  runw(wr<16, false>, "write only, 16 B plain");
  runw(wr<8, true>, "write only, 8 B nontemporal");
  runw(wr<8, false>, "write only, 8 B plain");
  {
    for (int it = 0; it < 2; ++it) hipMemsetAsync(out, it, in_bytes, 0);
    hipEventRecord(a);
    for (int it = 0; it < 5; ++it) hipMemsetAsync(out, it, in_bytes, 0);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-34s %8.3f ms  %7.1f GB/s\n", "hipMemset", ms / 5, (double)in_bytes / (ms / 5 * 1e-3) / 1e9);
  }
  run(mix<0, 1>, "read only", 1.0, 0.0);
  run(mix<1, 2>, "read 1 : write 0.5 (encode, c2)", 1.0, 0.5);
  run(mix<1, 1>, "read 1 : write 1 (copy, c3)", 1.0, 1.0);
  run(mix<2, 1>, "read 1 : write 2 (decode, c2)", 1.0, 2.0);
  {
    for (int it = 0; it < 2; ++it) hipMemcpyAsync(out, in, in_bytes, hipMemcpyDeviceToDevice, 0);
    hipEventRecord(a);
    for (int it = 0; it < 5; ++it) hipMemcpyAsync(out, in, in_bytes, hipMemcpyDeviceToDevice, 0);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-34s %8.3f ms  %7.1f GB/s\n", "hipMemcpy device to device", ms / 5, 2.0 * in_bytes / (ms / 5 * 1e-3) / 1e9);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
