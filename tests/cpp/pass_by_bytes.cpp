// pass_by_bytes.cpp -- the benchmark harness's `bytes` mode
// (TestCase.passByBytes, benchmark/.../TestCase.java:80-123) replayed without
// a JVM, to price the `gpu-packed` lines of do_benchmarks.bash
// (integration/capnproto-java.patch: Compression.GPU_PACKED, every message
// on the device).  One iteration, as the reference runs it:
//   request:  SerializePacked.write into an ArrayOutputStream over the
//             request buffer (Packed.writeBuffered, Packed.java:27-31),
//             SerializePacked.read back from an ArrayInputStream;
//   response: the same with the response buffer.
// GPU_PACKED runs both through the C++ mirror of the facade
// (capnproto-java_amd/csrc/host/packed_stream.hpp -> cpk_encode_host_gather /
// cpk_read_message_host, the calls the JNI glue makes); PACKED through the
// C restatement of the reference's codec (oracle/packed_oracle.c, one
// thread; the JVM's loop is the same single-threaded walk, so its time is
// at least this).  Messages: MessageBuilder's segments as the default
// allocator grows them (DefaultAllocator.java:52-77: 8 KiB, then each new
// segment as large as all before it), filled with config-2-like words (half
// zero words, the rest a quarter zero bytes).  The reference's 1 MiB
// scratch buffers (TestCase.java:46-48) would refuse messages over 1 MiB
// (ArrayOutputStream.java:40-42); the replay sizes the buffers to fit.
//
// Test infrastructure (the oracle is the CPU leg and the checker): built and
// run by tests/test_gpu_threshold.py, or by hand:
//   g++ -O2 -std=c++17 -pthread -Iinclude tests/cpp/pass_by_bytes.cpp
//       oracle/packed_oracle.c -Lcapnproto-java_amd/lib -lcapnp_packed_hip
//       -Wl,-rpath,$PWD/capnproto-java_amd/lib -o /tmp/pbb
//   /tmp/pbb [max KiB] [iterations]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../capnproto-java_amd/csrc/host/packed_stream.hpp"
extern "C" {
#include "../../oracle/packed_oracle.h"
}

using Segs = std::vector<std::vector<uint8_t>>;

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// a message of `bytes` words' bytes in the default allocator's segments
static Segs make_message(size_t bytes, uint32_t seed) {
  Segs segs;
  size_t left = bytes / 8 * 8, next = 8192;
  uint32_t rs = seed;
  auto rnd = [&]() { return rs = rs * 1103515245u + 12345u, rs >> 8; };
  while (left) {
    const size_t n = std::min(left, next);
    std::vector<uint8_t> s(n, 0);
    for (size_t w = 0; w < n / 8; ++w)
      if (rnd() % 2)
        for (int b = 0; b < 8; ++b) s[8 * w + b] = (rnd() % 4) ? (uint8_t)(1 + rnd() % 255) : 0;
    segs.push_back(std::move(s));
    left -= n;
    next += n;  // GROW_HEURISTICALLY: the next segment is as large as all so far
  }
  return segs;
}

// PACKED: Serialize.write / Serialize.read over the C restatement
static size_t cpu_write(const Segs &m, std::vector<uint8_t> &buf) {
  std::vector<const uint8_t *> p;
  std::vector<uint32_t> w;
  for (const auto &s : m) {
    p.push_back(s.data());
    w.push_back((uint32_t)(s.size() / 8));
  }
  return cpko_write_message(p.data(), w.data(), (uint32_t)m.size(), buf.data());
}
static bool cpu_read(const std::vector<uint8_t> &buf, size_t len, std::vector<uint8_t> &out,
                     std::vector<uint32_t> &sw) {
  size_t used = 0;
  uint32_t ns = 0;
  return cpko_read_message(buf.data(), len, &used, &ns, sw.data(), (uint32_t)sw.size(), out.data(), out.size(),
                           8ull << 20) == CPKO_OK &&
         used == len;
}

int main(int argc, char **argv) {
  const size_t max_kib = argc > 1 ? (size_t)atol(argv[1]) : 4096;
  const int iters = argc > 2 ? atoi(argv[2]) : 50;
  std::printf("# passByBytes (TestCase.java:80-123): per iteration 2 x SerializePacked.write + 2 x read\n");
  std::printf("# gpu_alloc: the facade returning fresh vectors (packed bytes, then copied into the\n"
              "#   request buffer; one vector per segment read back); gpu_owned: packed in place into the\n"
              "#   caller's ArrayOutputStream, segments read as views of one reused buffer\n"
              "#   (MessageView), split into its write and read calls; cpu: the C codec (one thread)\n");
  std::printf("# msg_bytes  segs  packed_bytes  gpu_alloc_us  gpu_owned_us  (write_us  read_us)  packed_cpu_us"
              "  alloc/cpu  owned/cpu\n");
  for (size_t kib = 1; kib <= max_kib; kib *= 2) {
    // (a context per size: with CPK_HOST_TRACE=1 each prints its phases on destruction)
    capnp_amd::Gpu gpu(0);
    const size_t bytes = kib * 1024;
    const Segs req = make_message(bytes, 7 + (uint32_t)kib), resp = make_message(bytes, 99 + (uint32_t)kib);
    const size_t cap = cpko_packed_bound(bytes / 8 + 520) + 64;
    std::vector<uint8_t> reqbuf(cap), respbuf(cap), dec(bytes + 8);
    std::vector<uint32_t> sw(512);
    // parity once: the GPU's bytes are the C restatement's, and read back
    size_t plen = 0;
    {
      const std::vector<uint8_t> g = capnp_amd::SerializePacked::write(gpu, req);
      plen = cpu_write(req, reqbuf);
      if (g.size() != plen || std::memcmp(g.data(), reqbuf.data(), plen) != 0) {
        std::printf("MISMATCH write %zu\n", bytes);
        return 1;
      }
      capnp_amd::ArrayInputStream in(g.data(), g.size());
      if (capnp_amd::SerializePacked::read(gpu, in) != req) {
        std::printf("MISMATCH read %zu\n", bytes);
        return 1;
      }
    }
    auto gpu_iter = [&]() {
      for (const Segs *m : {&req, &resp}) {
        std::vector<uint8_t> &buf = m == &req ? reqbuf : respbuf;
        capnp_amd::ArrayOutputStream w(buf.data(), buf.size());
        const std::vector<uint8_t> pk = capnp_amd::SerializePacked::write(gpu, *m);
        w.write(pk.data(), pk.size());  // (writer.flush(): the bytes land in the buffer)
        capnp_amd::ArrayInputStream in(buf.data(), w.position());
        const Segs back = capnp_amd::SerializePacked::read(gpu, in);
        if (back.size() != m->size()) std::abort();
      }
    };
    capnp_amd::MessageView view;
    double t_w = 0, t_r = 0;
    auto owned_iter = [&]() {
      for (const Segs *m : {&req, &resp}) {
        std::vector<uint8_t> &buf = m == &req ? reqbuf : respbuf;
        capnp_amd::ArrayOutputStream w(buf.data(), buf.size());
        const double a = now();
        capnp_amd::SerializePacked::write(gpu, *m, w);
        const double b = now();
        capnp_amd::ArrayInputStream in(buf.data(), w.position());
        capnp_amd::SerializePacked::read(gpu, in, view);
        t_w += b - a;
        t_r += now() - b;
        if (view.segmentCount() != m->size()) std::abort();
      }
    };
    // (parity of the in-place forms once: the C codec's bytes, the segments back)
    {
      capnp_amd::ArrayOutputStream w(reqbuf.data(), reqbuf.size());
      const size_t k = capnp_amd::SerializePacked::write(gpu, req, w);
      std::vector<uint8_t> ref(reqbuf.size());
      if (k != plen || cpu_write(req, ref) != plen || std::memcmp(ref.data(), reqbuf.data(), plen) != 0) {
        std::printf("MISMATCH owned write %zu\n", bytes);
        return 1;
      }
      capnp_amd::ArrayInputStream in(reqbuf.data(), k);
      capnp_amd::SerializePacked::read(gpu, in, view);
      for (size_t i = 0; i < req.size(); ++i)
        if (view.segmentBytes(i) != req[i].size() || std::memcmp(view.segment(i), req[i].data(), req[i].size())) {
          std::printf("MISMATCH owned read %zu\n", bytes);
          return 1;
        }
    }
    auto cpu_iter = [&]() {
      for (const Segs *m : {&req, &resp}) {
        std::vector<uint8_t> &buf = m == &req ? reqbuf : respbuf;
        const size_t n = cpu_write(*m, buf);
        if (!cpu_read(buf, n, dec, sw)) std::abort();
      }
    };
    gpu_iter();
    owned_iter();
    cpu_iter();
    t_w = t_r = 0;
    const int it = std::max(3, (int)(iters * 64 / std::max<size_t>(kib, 64)));
    double t0 = now();
    for (int i = 0; i < it; ++i) gpu_iter();
    const double tg = (now() - t0) / it;
    t0 = now();
    for (int i = 0; i < it; ++i) owned_iter();
    const double to = (now() - t0) / it;
    t0 = now();
    for (int i = 0; i < it; ++i) cpu_iter();
    const double tc = (now() - t0) / it;
    std::printf("%10zu  %4zu  %12zu  %12.1f  %12.1f  (%8.1f  %7.1f)  %13.1f  %9.2f  %9.2f\n", bytes, req.size(), plen,
                tg * 1e6, to * 1e6, t_w / it * 1e6, t_r / it * 1e6, tc * 1e6, tg / tc, to / tc);
    std::fflush(stdout);
  }
  return 0;
}
