// threshold_probe.cpp -- where the GPU codec starts to pay for one message
// (GpuDispatch.MIN_BYTES).  Per message size: one
// SerializePacked.write (cpk_encode_messages_host) and one SerializePacked.read
// (cpk_read_message_host) through the library's host forms, against the CPU
// restatement of the reference's codec (oracle/packed_oracle.c, one thread:
// the JVM codec is a single-threaded loop of the same shape and is, per the
// reference's own notes, slower -- so this crossover is an upper bound of the
// JVM's).  Messages: one segment of config-2-like words (half zero words,
// the rest a quarter zero bytes).
//
// Test infrastructure (the oracle is the checker and the CPU leg): built and
// run by tests/test_gpu_threshold.py, or by hand:
//   g++ -O2 -std=c++17 -pthread -Iinclude tests/cpp/threshold_probe.cpp oracle/packed_oracle.c
//       -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,$PWD/capnproto-java_amd/lib -o /tmp/probe
//   /tmp/probe [max KiB]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/capnp_packed.h"
extern "C" {
#include "../../oracle/packed_oracle.h"
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double median_time(F f, int reps) {
  std::vector<double> t;
  for (int r = 0; r < reps; ++r) {
    const double a = now();
    f();
    t.push_back(now() - a);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char **argv) {
  const size_t max_kib = argc > 1 ? (size_t)atol(argv[1]) : 16384;
  cpk_ctx ctx = nullptr;
  if (cpk_ctx_create(0, &ctx) != CPK_OK) return 1;
  uint32_t rs = 99;
  auto rnd = [&]() { return rs = rs * 1103515245u + 12345u, rs >> 8; };
  std::printf("# bytes  gpu_write_us  gpu_read_us  cpu_write_us  cpu_read_us  gpu_rt_us  cpu_rt_us\n");
  for (size_t kib = 1; kib <= max_kib; kib *= 2) {
    const size_t W = kib * 128;  // words
    std::vector<uint8_t> seg(8 * W + 8, 0);
    for (size_t w = 0; w < W; ++w)
      if (rnd() % 2)
        for (int b = 0; b < 8; ++b) seg[8 * w + b] = (rnd() % 4) ? (uint8_t)(1 + rnd() % 255) : 0;
    const uint8_t *segp = seg.data();
    const uint32_t sw = (uint32_t)W;
    std::vector<uint8_t> pk(cpko_packed_bound(W + 4) + 64);
    const size_t P = cpko_write_message(&segp, &sw, 1, pk.data());
    // GPU write: one message, table built on the device
    std::vector<uint64_t> swo = {0, W}, mso = {0, 1}, off(3);
    std::vector<uint8_t> out(cpk_packed_bound(W) + 64 + 16);
    std::vector<uint64_t> words(W + 1), info(CPK_MSG_INFO_WORDS);
    std::vector<uint8_t> cpu_out(8 * W + 64);
    const int reps = kib <= 256 ? 200 : 20;
    auto gw = [&]() { cpk_encode_messages_host(ctx, seg.data(), swo.data(), 1, mso.data(), 1, out.data(), out.size(), off.data()); };
    auto gr = [&]() { cpk_read_message_host(ctx, pk.data(), P, 8ull << 20 << 4, words.data(), W, info.data()); };
    auto cw = [&]() { cpko_write_message(&segp, &sw, 1, pk.data()); };
    size_t used;
    uint32_t nseg, sws[4];
    auto cr = [&]() { cpko_read_message(pk.data(), P, &used, &nseg, sws, 4, cpu_out.data(), cpu_out.size(), 8ull << 20 << 4); };
    gw();
    gr();
    if (off[2] != P || memcmp(out.data(), pk.data(), P) != 0 || info[0] != 0 || info[1] != P ||
        memcmp(words.data(), seg.data(), 8 * W) != 0) {
      std::printf("MISMATCH at %zu KiB\n", kib);
      return 2;
    }
    const double a = median_time(gw, reps), b = median_time(gr, reps), c = median_time(cw, reps),
                 d = median_time(cr, reps);
    std::printf("%9zu %13.1f %12.1f %13.1f %12.1f %10.1f %10.1f\n", 8 * W, a * 1e6, b * 1e6, c * 1e6, d * 1e6,
                (a + b) * 1e6, (c + d) * 1e6);
    std::fflush(stdout);
  }
  cpk_ctx_destroy(ctx);
  return 0;
}
