// small_phases.cpp -- in-kernel phase times of the one-launch small-message
// paths (rm_small_kernel / sp_small_kernel) from a CPK_PHASE_STATS variant
// build with s_memrealtime stamps (100 MHz) in g_phase[48..56]; decode_body's
// own core-clock phase sums in g_phase[16..23].  Diagnostic tool only.
//   g++ -O2 -std=c++17 -Iinclude tools/micro/small_phases.cpp oracle/packed_oracle.c -ldl -o build/small_phases
//   build/small_phases build/variants/tdbg.so
#include <dlfcn.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../include/capnp_packed.h"
extern "C" {
#include "../../oracle/packed_oracle.h"
}
typedef int (*create_t)(int, cpk_ctx *);
typedef int (*rd_t)(cpk_ctx, const void *, uint64_t, uint64_t, void *, uint64_t, uint64_t *);
typedef int (*wr_t)(cpk_ctx, const void *, const uint64_t *, uint32_t, const uint64_t *, uint32_t, void *, uint64_t,
                    uint64_t *);
typedef int (*ph_t)(unsigned long long *);
int main(int argc, char **argv) {
  void *h = dlopen(argv[1], RTLD_NOW);
  if (!h) { std::printf("dlopen: %s\n", dlerror()); return 1; }
  auto create = (create_t)dlsym(h, "cpk_ctx_create");
  auto rd = (rd_t)dlsym(h, "cpk_read_message_host");
  auto wr = (wr_t)dlsym(h, "cpk_encode_messages_host");
  auto ph = (ph_t)dlsym(h, "cpk_debug_phase_stats");
  if (!create || !rd || !wr || !ph) { std::printf("missing symbols\n"); return 1; }
  cpk_ctx ctx;
  if (create(0, &ctx)) return 1;
  unsigned long long g[64];
  uint32_t rs = 7;
  auto rnd = [&]() { return rs = rs * 1103515245u + 12345u, rs >> 8; };
  for (size_t kib : {1, 4, 16, 64}) {
    const size_t W = kib * 128;
    std::vector<uint8_t> seg(8 * W + 8, 0);
    for (size_t w = 0; w < W; ++w)
      if (rnd() % 2)
        for (int b = 0; b < 8; ++b) seg[8 * w + b] = (rnd() % 4) ? (uint8_t)(1 + rnd() % 255) : 0;
    const uint8_t *segp = seg.data();
    const uint32_t sw = (uint32_t)W;
    std::vector<uint8_t> pk(cpko_packed_bound(W + 4) + 64);
    const size_t P = cpko_write_message(&segp, &sw, 1, pk.data());
    std::vector<uint64_t> swo = {0, W}, mso = {0, 1}, off(3), words(W + 1), info(CPK_MSG_INFO_WORDS);
    std::vector<uint8_t> out(cpko_packed_bound(W) + 96);
    for (int r = 0; r < 20; ++r) {
      rd(ctx, pk.data(), P, 1ull << 40, words.data(), W, info.data());
      wr(ctx, seg.data(), swo.data(), 1, mso.data(), 1, out.data(), out.size(), off.data());
    }
    ph(g);
    const int N = 200;
    double tr = 0, tw = 0;
    for (int r = 0; r < N; ++r) {
      auto a = std::chrono::steady_clock::now();
      rd(ctx, pk.data(), P, 1ull << 40, words.data(), W, info.data());
      auto b = std::chrono::steady_clock::now();
      wr(ctx, seg.data(), swo.data(), 1, mso.data(), 1, out.data(), out.size(), off.data());
      auto c = std::chrono::steady_clock::now();
      tr += std::chrono::duration<double>(b - a).count();
      tw += std::chrono::duration<double>(c - b).count();
    }
    ph(g);
    const double rn = g[52] ? (double)g[52] : 1, wn = g[56] ? (double)g[56] : 1;
    std::printf("%4zu KiB (packed %zu B): read host %.1f us | kernel: copy %.2f table %.2f decode %.2f final+fence %.2f us"
                " (n=%llu)\n", kib, P, 1e6 * tr / N, g[48] / rn / 100, g[49] / rn / 100, g[50] / rn / 100,
                g[51] / rn / 100, g[52]);
    std::printf("         write host %.1f us | kernel: desc+lut %.2f pieces %.2f tail+fence %.2f us (n=%llu)\n",
                1e6 * tw / N, g[53] / wn / 100, g[54] / wn / 100, g[55] / wn / 100, g[56]);
    unsigned long long tot = 0;
    for (int i = 16; i < 24; ++i) tot += g[i];
    std::printf("         decode_body phases (core clk, all 4 waves):");
    for (int i = 16; i < 24; ++i) std::printf(" %.0f", g[i] / rn);
    std::printf("\n");
  }
  return 0;
}
