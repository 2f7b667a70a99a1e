// small_stress.cpp -- back-to-back one-launch small host calls with changing
// contents, each result checked against the oracle.  Modes: r (reads), w
// (writes), rw (alternating), and "2" suffix: a second thread with its own
// context runs writes concurrently.  Diagnostic tool.
//   g++ -O2 -std=c++17 -pthread -Iinclude tools/micro/small_stress.cpp oracle/packed_oracle.c
//       -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,$PWD/capnproto-java_amd/lib -o build/small_stress
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include "../../include/capnp_packed.h"
#include "../../capnproto-java_amd/csrc/host/packed_stream.hpp"
#include <fcntl.h>
using namespace capnp_amd;
extern "C" {
#include "../../oracle/packed_oracle.h"
}
struct Msg {
  std::vector<uint8_t> seg, pk;
  uint32_t W;
};
static std::vector<Msg> make(uint32_t seed, int n) {
  std::vector<Msg> v;
  uint32_t rs = seed;
  auto rnd = [&]() { return rs = rs * 1103515245u + 12345u, rs >> 8; };
  for (int i = 0; i < n; ++i) {
    Msg m;
    m.W = 1 + rnd() % 1200;
    m.seg.assign(8 * m.W, 0);
    for (auto &b : m.seg)
      if (rnd() % 3 == 0) b = (uint8_t)rnd();
    const uint8_t *sp = m.seg.data();
    m.pk.resize(cpko_packed_bound(m.W + 4) + 64);
    m.pk.resize(cpko_write_message(&sp, &m.W, 1, m.pk.data()));
    v.push_back(m);
  }
  return v;
}
static int run(cpk_ctx ctx, const std::vector<Msg> &ms, bool rd, bool wr, int iters, const char *tag) {
  int bad = 0;
  std::vector<uint64_t> words(1300), info(CPK_MSG_INFO_WORDS), off(3);
  std::vector<uint8_t> out(20000);
  const bool verbose = getenv("SS_VERBOSE") != nullptr;
  for (int k = 0; k < iters; ++k) {
    const Msg &m = ms[k % ms.size()];
    if (verbose) std::fprintf(stderr, "%s iter %d (packed %zu)\n", tag, k, m.pk.size());
    if (rd) {
      const int rc = cpk_read_message_host(ctx, m.pk.data(), m.pk.size(), 1ull << 30, words.data(), words.size(),
                                           info.data());
      if (rc || info[1] != m.pk.size() || info[2] != 1 || info[3] != m.W ||
          memcmp(words.data(), m.seg.data(), 8 * m.W)) {
        if (bad < 5)
          std::printf("%s read %d: rc %d consumed %llu/%zu count %llu words %llu/%u\n", tag, k, rc,
                      (unsigned long long)info[1], m.pk.size(), (unsigned long long)info[2],
                      (unsigned long long)info[3], m.W);
        ++bad;
      }
    }
    if (wr) {
      uint64_t swo[2] = {0, m.W}, mso[2] = {0, 1};
      const int rc = cpk_encode_messages_host(ctx, m.seg.data(), swo, 1, mso, 1, out.data(), out.size(), off.data());
      if (rc || off[2] != m.pk.size() || memcmp(out.data(), m.pk.data(), m.pk.size())) {
        if (bad < 5) std::printf("%s write %d: rc %d size %llu/%zu\n", tag, k, rc, (unsigned long long)off[2], m.pk.size());
        ++bad;
      }
    }
  }
  std::printf("%s: %d bad of %d\n", tag, bad, iters);
  return bad;
}
// a stream of messages (1-5 segments of 0-1199 words, every 97th 8192-word
// segments) read back as a channel reader does: a try on what is buffered,
// ETRUNC -> twice the bytes
static int chan(cpk_ctx ctx, int nmsg) {
  uint32_t rs = 12345;
  auto rnd = [&]() { return rs = rs * 1103515245u + 12345u, rs >> 8; };
  std::vector<uint8_t> stream;
  std::vector<std::vector<std::vector<uint8_t>>> msgs;
  for (int m = 0; m < nmsg; ++m) {
    const int nseg = 1 + (int)(rnd() % 5);
    std::vector<std::vector<uint8_t>> segs;
    std::vector<const uint8_t *> ptr;
    std::vector<uint32_t> ws;
    for (int i = 0; i < nseg; ++i) {
      const uint32_t w = (m % 97 == 0) ? 8192 : rnd() % 1200;
      std::vector<uint8_t> sg(8 * w, 0);
      for (auto &b : sg)
        if (rnd() % 3 == 0) b = (uint8_t)rnd();
      segs.push_back(sg);
    }
    for (auto &sg : segs) {
      ptr.push_back(sg.data());
      ws.push_back((uint32_t)(sg.size() / 8));
    }
    uint64_t tw = 0;
    for (auto w : ws) tw += w;
    std::vector<uint8_t> pk(cpko_packed_bound(tw + 300) + 64);
    pk.resize(cpko_write_message(ptr.data(), ws.data(), (uint32_t)nseg, pk.data()));
    stream.insert(stream.end(), pk.begin(), pk.end());
    msgs.push_back(segs);
  }
  for (int g = 0; g < 300; ++g) stream.push_back((uint8_t)(g * 37 + 11));
  std::vector<uint64_t> words(1 << 16), info(CPK_MSG_INFO_WORDS);
  size_t pos = 0;
  int bad = 0, tries = 0;
  for (int m = 0; m < nmsg && bad < 5; ++m) {
    size_t avail = std::min<size_t>(stream.size() - pos, 1000 + (size_t)(rnd() % 3000));
    for (;;) {
      ++tries;
      const int rc = cpk_read_message_host(ctx, stream.data() + pos, avail, 8ull << 20, words.data(), words.size(),
                                           info.data());
      if (rc == CPK_ETRUNC && avail < stream.size() - pos) {
        avail = std::min(stream.size() - pos, 2 * avail);
        continue;
      }
      bool ok = rc == CPK_OK && info[2] == msgs[m].size();
      for (size_t i = 0; ok && i < msgs[m].size(); ++i)
        ok = 8 * (info[5 + i] - info[4 + i]) == msgs[m][i].size() &&
             !memcmp((const uint8_t *)words.data() + 8 * info[4 + i], msgs[m][i].data(), msgs[m][i].size());
      if (!ok) {
        std::printf("chan message %d: rc %d avail %zu count %llu\n", m, rc, avail, (unsigned long long)info[2]);
        ++bad;
      }
      pos += info[1];
      break;
    }
  }
  std::printf("chan: %d bad, %d tries, %zu of %zu bytes consumed\n", bad, tries, pos, stream.size());
  return bad;
}

// the C++ mirror's pipe case: a writer thread (its own context,
// SerializePacked::write = cpk_encode_host_gather) feeds a pipe, the main
// thread reads with readFromUnbuffered; every writer result is also compared
// with the oracle
static int pipe_case(int nmsg, bool check_writer) {
  uint32_t rs = 12345;
  auto rnd = [&]() { return rs = rs * 1103515245u + 12345u, rs >> 8; };
  std::vector<SerializePacked::Message> msgs;
  for (int m = 0; m < nmsg; ++m) {
    SerializePacked::Message msg;
    const int nseg = 1 + (int)(rnd() % 5);
    for (int i = 0; i < nseg; ++i) {
      const uint32_t w = (m % 97 == 0) ? 8192 : rnd() % 1200;
      std::vector<uint8_t> sg(8 * w, 0);
      for (auto &b : sg)
        if (rnd() % 3 == 0) b = (uint8_t)rnd();
      msg.push_back(sg);
    }
    msgs.push_back(msg);
  }
  int fds[2];
  if (pipe(fds)) return 1;
  int wbad = 0, rbad = 0;
  std::thread writer([&]() {
    Gpu wg(0);
    FdChannel out(fds[1]);
    for (int m = 0; m < nmsg; ++m) {
      const std::vector<uint8_t> b = SerializePacked::write(wg, msgs[m]);
      if (check_writer) {
        std::vector<const uint8_t *> ptr;
        std::vector<uint32_t> ws;
        uint64_t tw = 0;
        for (auto &sg : msgs[m]) {
          ptr.push_back(sg.data());
          ws.push_back((uint32_t)(sg.size() / 8));
          tw += sg.size() / 8;
        }
        std::vector<uint8_t> pk(cpko_packed_bound(tw + 300) + 64);
        pk.resize(cpko_write_message(ptr.data(), ws.data(), (uint32_t)ws.size(), pk.data()));
        if (pk != b && wbad++ < 5) std::printf("writer message %d: %zu bytes vs oracle %zu\n", m, b.size(), pk.size());
      }
      out.writeAll(b.data(), b.size());
    }
    close(fds[1]);
  });
  {
    Gpu gpu(0);
    ChannelReader in{FdChannel(fds[0])};
    for (int m = 0; m < nmsg; ++m) {
      try {
        if (SerializePacked::readFromUnbuffered(gpu, in) != msgs[m] && rbad++ < 5)
          std::printf("reader message %d differs\n", m);
      } catch (const std::exception &e) {
        std::printf("reader message %d: %s\n", m, e.what());
        ++rbad;
        break;
      }
    }
    // drain so the writer finishes
    std::vector<uint8_t> sink(1 << 16);
    while (read(fds[0], sink.data(), sink.size()) > 0) {
    }
  }
  writer.join();
  close(fds[0]);
  std::printf("pipe: writer %d bad, reader %d bad of %d\n", wbad, rbad, nmsg);
  return wbad + rbad;
}

int main(int argc, char **argv) {
  const std::string mode = argc > 1 ? argv[1] : "rw";
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  cpk_ctx a = nullptr, b = nullptr;
  if (cpk_ctx_create(0, &a)) return 1;
  const auto ms = make(1, 16), ms2 = make(2, 16);
  const bool rd = mode.find('r') != std::string::npos, wr = mode.find('w') != std::string::npos;
  int bad = 0;
  if (mode == "c") return chan(a, iters) ? 2 : 0;
  if (mode == "p") return pipe_case(iters, true) ? 2 : 0;
  if (mode == "pn") return pipe_case(iters, false) ? 2 : 0;
  if (mode.find('2') != std::string::npos) {
    if (cpk_ctx_create(0, &b)) return 1;
    int bad2 = 0;
    std::thread t([&]() { bad2 = run(b, ms2, false, true, iters, "thread2 writes"); });
    bad = run(a, ms, rd, wr, iters, "main");
    t.join();
    bad += bad2;
  } else {
    bad = run(a, ms, rd, wr, iters, "main");
  }
  return bad ? 2 : 0;
}
