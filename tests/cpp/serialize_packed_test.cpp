// SerializePackedTest (runtime/src/test/java/org/capnproto/SerializePackedTest.java)
// written against the C++ mirror of the reference API (capnproto-java_amd/
// csrc/host/packed_stream.hpp), every byte through the MI355X kernels.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../capnproto-java_amd/csrc/host/packed_stream.hpp"
extern "C" {
#include "../../oracle/packed_oracle.h"  // the checker (test infrastructure only)
}

using namespace capnp_amd;
using Bytes = std::vector<uint8_t>;

static int failures = 0;
#define EXPECT(cond, msg)                                   \
  do {                                                      \
    if (!(cond)) {                                          \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
      ++failures;                                           \
    }                                                       \
  } while (0)

// assertPacksTo, SerializePackedTest.java:63-91
static void assertPacksTo(Gpu &gpu, const Bytes &unpacked, const Bytes &packed) {
  {
    Bytes bytes(packed.size());
    ArrayOutputStream writer(bytes.data(), bytes.size());
    PackedOutputStream pos(gpu, writer);
    pos.write(unpacked.data(), unpacked.size());
    EXPECT(bytes == packed, "packed bytes");
    EXPECT(writer.position() == packed.size(), "packed length");
  }
  {
    ArrayInputStream reader(packed.data(), packed.size());
    PackedInputStream stream(gpu, reader);
    Bytes bytes(unpacked.size());
    size_t n = 0;
    try {
      n = stream.read(bytes.data(), bytes.size());
    } catch (const std::exception &e) {
      EXPECT(false, e.what());
    }
    EXPECT(n == unpacked.size(), "read length");
    EXPECT(bytes == unpacked, "unpacked bytes");
  }
}

// the oracle's Serialize.write through PackedOutputStream (SerializePacked.write)
static Bytes oracleWrite(const std::vector<Bytes> &segs) {
  std::vector<Bytes> padded;
  std::vector<const uint8_t *> ptrs;
  std::vector<uint32_t> words;
  size_t cap = cpko_packed_bound(segs.size() + 2) + 16;
  for (auto &sg : segs) {
    padded.push_back(sg);
    padded.back().resize(sg.size() + 8, 0);
    words.push_back((uint32_t)(sg.size() / 8));
    cap += cpko_packed_bound(sg.size() / 8);
  }
  for (auto &pb : padded) ptrs.push_back(pb.data());
  Bytes out(cap);
  out.resize(cpko_write_message(ptrs.data(), words.data(), (uint32_t)segs.size(), out.data()));
  return out;
}

static Bytes rep(Bytes b, int times) {
  Bytes out;
  for (int i = 0; i < times; ++i) out.insert(out.end(), b.begin(), b.end());
  return out;
}
static Bytes cat(std::initializer_list<Bytes> parts) {
  Bytes out;
  for (auto &p : parts) out.insert(out.end(), p.begin(), p.end());
  return out;
}

int main() {
  Gpu gpu(0);
  // testSimplePacking, SerializePackedTest.java:20-60
  assertPacksTo(gpu, {}, {});
  assertPacksTo(gpu, {0, 0, 0, 0, 0, 0, 0, 0}, {0, 0});
  assertPacksTo(gpu, {0, 0, 12, 0, 0, 34, 0, 0}, {0x24, 12, 34});
  assertPacksTo(gpu, {1, 3, 2, 4, 5, 7, 6, 8}, {0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0});
  assertPacksTo(gpu, {0, 0, 0, 0, 0, 0, 0, 0, 1, 3, 2, 4, 5, 7, 6, 8},
                {0, 0, 0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0});
  assertPacksTo(gpu, {0, 0, 12, 0, 0, 34, 0, 0, 1, 3, 2, 4, 5, 7, 6, 8},
                {0x24, 12, 34, 0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0});
  assertPacksTo(gpu, {1, 3, 2, 4, 5, 7, 6, 8, 8, 6, 7, 4, 5, 2, 3, 1},
                {0xff, 1, 3, 2, 4, 5, 7, 6, 8, 1, 8, 6, 7, 4, 5, 2, 3, 1});
  const Bytes w18 = {1, 2, 3, 4, 5, 6, 7, 8};
  assertPacksTo(gpu, cat({rep(w18, 4), {0, 2, 4, 0, 9, 0, 5, 1}}),
                cat({{0xff}, w18, {3}, rep(w18, 3), {0xd6, 2, 4, 9, 5, 1}}));
  assertPacksTo(gpu, cat({w18, w18, {6, 2, 4, 3, 9, 0, 5, 1}, w18, {0, 2, 4, 0, 9, 0, 5, 1}}),
                cat({{0xff}, w18, {3}, w18, {6, 2, 4, 3, 9, 0, 5, 1}, w18, {0xd6, 2, 4, 9, 5, 1}}));
  assertPacksTo(gpu, cat({{8, 0, 100, 6, 0, 1, 1, 2}, Bytes(24, 0), {0, 0, 1, 0, 2, 0, 3, 1}}),
                {0xed, 8, 100, 6, 1, 1, 2, 0, 2, 0xd4, 1, 2, 3, 1});
  assertPacksTo(gpu, cat({{0, 0, 0, 0, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0}, Bytes(8, 0)}),
                {0x10, 2, 0x40, 1, 0, 0});
  assertPacksTo(gpu, Bytes(8 * 200, 0), {0, 199});
  Bytes packedOnes(10 + 8 * 199, 1);
  packedOnes[0] = 255;
  packedOnes[9] = 199;
  assertPacksTo(gpu, Bytes(8 * 200, 1), packedOnes);

  // read_shouldThrowDecodingExceptionOnEmptyArrayInputStream (:93-98)
  {
    Bytes empty;
    ArrayInputStream in(empty.data(), 0);
    bool threw = false;
    try {
      SerializePacked::read(gpu, in);
    } catch (const DecodeException &) {
      threw = true;
    }
    EXPECT(threw, "empty stream must throw DecodeException");
  }
  // read_shouldThrowDecodingExceptionWhenTryingToReadMoreThanAvailable (:100-105)
  {
    Bytes bytes = {17, 0, 127, 0, 0, 0, 0};
    ArrayInputStream in(bytes.data(), bytes.size());
    bool threw = false;
    try {
      SerializePacked::read(gpu, in);
    } catch (const DecodeException &) {
      threw = true;
    }
    EXPECT(threw, "truncated stream must throw DecodeException");
  }
  // SerializeTest.testSegmentReading (SerializeTest.java:82-141) through packing
  for (int nseg = 1; nseg <= 4; ++nseg) {
    std::vector<Bytes> segs;
    for (int i = 0; i < nseg; ++i) segs.push_back(rep({(uint8_t)i, 0, 0, 0, 0, 0, 0, 0}, i));
    Bytes stream = SerializePacked::write(gpu, segs);
    ArrayInputStream in(stream.data(), stream.size());
    auto got = SerializePacked::read(gpu, in);
    EXPECT(got == segs, "segments round trip");
    EXPECT(in.remaining() == 0, "stream consumed");
  }
  // many messages in one GPU pass each way (cpk_encode_messages_host /
  // cpk_decode_messages_host) == one write()/read() per message
  {
    std::vector<SerializePacked::Message> msgs;
    for (int m = 0; m < 40; ++m) {
      SerializePacked::Message msg;
      for (int i = 0; i <= m % 5; ++i) {
        Bytes sg;
        for (int w = 0; w < (m * 7 + i * 13) % 90; ++w) {
          Bytes word = {(uint8_t)(w * m), 0, (uint8_t)i, 0, 0, 0, (uint8_t)(w & 3 ? 0 : 9), 0};
          sg.insert(sg.end(), word.begin(), word.end());
        }
        msg.push_back(sg);
      }
      msgs.push_back(msg);
    }
    std::vector<uint64_t> moff;
    Bytes all = SerializePacked::writeMessages(gpu, msgs, &moff);
    Bytes one;
    for (auto &m : msgs) {
      Bytes b = SerializePacked::write(gpu, m);
      one.insert(one.end(), b.begin(), b.end());
    }
    EXPECT(all == one, "writeMessages == write per message");
    EXPECT(SerializePacked::readMessages(gpu, all, moff) == msgs, "readMessages round trip");
    bool threw = false;
    try {
      Bytes bad = all;
      bad.resize(moff[3] + 5);  // message 3 truncated
      std::vector<uint64_t> mo(moff.begin(), moff.begin() + 4);
      mo.push_back(bad.size());
      SerializePacked::readMessages(gpu, bad, mo);
    } catch (const DecodeException &) {
      threw = true;
    }
    EXPECT(threw, "truncated message must throw DecodeException");
  }
  // The benchmark harness's "bytes" mode with GPU_PACKED (TestCase.java:
  // 78-120, GpuPacked.java): messages read one at a time from a reused scratch
  // buffer that still holds stale bytes past the current message; each read
  // consumes exactly its message's packed bytes.
  {
    std::vector<std::vector<Bytes>> msgs;
    Bytes scratch;
    for (int m = 0; m < 6; ++m) {
      std::vector<Bytes> segs;
      for (int i = 0; i <= m % 3; ++i) {
        Bytes sg;
        for (int w = 0; w < 3 + 17 * m + 5 * i; ++w) {
          Bytes word = {(uint8_t)(w + m), (uint8_t)(w & 1 ? 0 : 7), 0, (uint8_t)i, 1, 2, 3, (uint8_t)m};
          if (w % 5 == 0) word = Bytes(8, 0);
          sg.insert(sg.end(), word.begin(), word.end());
        }
        segs.push_back(sg);
      }
      Bytes b = SerializePacked::write(gpu, segs);
      scratch.insert(scratch.end(), b.begin(), b.end());
      msgs.push_back(segs);
    }
    const size_t used = scratch.size();
    for (int g = 0; g < 300; ++g) scratch.push_back((uint8_t)(g * 37 + 11));  // stale bytes
    ArrayInputStream in(scratch.data(), scratch.size());
    for (auto &segs : msgs) EXPECT(SerializePacked::read(gpu, in) == segs, "message from scratch");
    EXPECT(in.remaining() == scratch.size() - used, "stale bytes left unread");
  }
  // writeToUnbuffered / readFromUnbuffered through a pipe
  // (SerializePacked.java:84-96, :119-134): 1000 messages of 1-5 segments,
  // 0-64 KiB each, written by one thread (its own context) while another
  // reads them back; then tryReadFromUnbuffered sees the end of the stream.
  {
    std::vector<SerializePacked::Message> msgs;
    uint64_t words = 0;
    uint32_t rs = 12345;
    auto rnd = [&]() { return rs = rs * 1103515245u + 12345u, rs >> 8; };
    for (int m = 0; m < 1000; ++m) {
      SerializePacked::Message msg;
      const int nseg = 1 + (int)(rnd() % 5);
      for (int i = 0; i < nseg; ++i) {
        const uint32_t w = (m % 97 == 0) ? 8192 : rnd() % 1200;
        Bytes sg(8 * w, 0);
        for (uint32_t j = 0; j < 8 * w; ++j)
          if (rnd() % 3 == 0) sg[j] = (uint8_t)rnd();
        words += w;
        msg.push_back(sg);
      }
      msgs.push_back(msg);
    }
    int fds[2];
    EXPECT(pipe(fds) == 0, "pipe");
    const auto t0 = std::chrono::steady_clock::now();
    std::thread writer([&]() {
      Gpu wg(0);
      FdChannel out(fds[1]);
      for (auto &m : msgs) SerializePacked::writeToUnbuffered(wg, out, m);
      close(fds[1]);
    });
    ChannelReader in{FdChannel(fds[0])};
    int same = 0;
    for (auto &m : msgs) {
      try {
        same += SerializePacked::readFromUnbuffered(gpu, in) == m;
      } catch (const std::exception &e) {
        EXPECT(false, e.what());
        break;
      }
    }
    writer.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    EXPECT(same == (int)msgs.size(), "messages through the pipe");
    EXPECT(!SerializePacked::tryReadFromUnbuffered(gpu, in).has_value(), "end of stream");
    close(fds[0]);
    std::printf("pipe: %zu messages, %.1f MiB of words, %.3f s: %.3f GiB/s, %.0f messages/s\n", msgs.size(),
                words * 8 / 1048576.0, dt, words * 8 / dt / (1 << 30), msgs.size() / dt);
    // the wire itself: what writeToUnbuffered puts on the channel is, message
    // by message, the oracle's Serialize.write through PackedOutputStream
    EXPECT(pipe(fds) == 0, "pipe");
    std::thread wire_writer([&]() {
      Gpu wg(0);
      FdChannel out(fds[1]);
      for (int m = 0; m < 300; ++m) SerializePacked::writeToUnbuffered(wg, out, msgs[m]);
      close(fds[1]);
    });
    Bytes wire, expect;
    {
      FdChannel raw(fds[0]);
      std::vector<uint8_t> buf(1 << 16);
      for (size_t k; (k = raw.readSome(buf.data(), buf.size())) > 0;) wire.insert(wire.end(), buf.begin(), buf.begin() + k);
    }
    wire_writer.join();
    close(fds[0]);
    for (int m = 0; m < 300; ++m) {
      Bytes b = oracleWrite(msgs[m]);
      expect.insert(expect.end(), b.begin(), b.end());
    }
    EXPECT(wire == expect, "wire bytes == oracle Serialize.write per message");
    // the same messages packed in one GPU call, then read one by one
    EXPECT(pipe(fds) == 0, "pipe");
    const auto t1 = std::chrono::steady_clock::now();
    std::thread writer2([&]() {
      Gpu wg(0);
      FdChannel out(fds[1]);
      SerializePacked::writeMessagesToUnbuffered(wg, out, msgs);
      close(fds[1]);
    });
    ChannelReader in2{FdChannel(fds[0])};
    same = 0;
    while (auto m = SerializePacked::tryReadFromUnbuffered(gpu, in2)) same += (size_t)same < msgs.size() && *m == msgs[same];
    writer2.join();
    const double dt2 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    EXPECT(same == (int)msgs.size(), "batch-written messages through the pipe");
    close(fds[0]);
    std::printf("pipe (writeMessagesToUnbuffered): %.3f s: %.3f GiB/s\n", dt2, words * 8 / dt2 / (1 << 30));
    // a message cut short by the end of the channel: premature EOF
    EXPECT(pipe(fds) == 0, "pipe");
    {
      Bytes b = SerializePacked::write(gpu, msgs[5]);
      FdChannel out(fds[1]);
      out.writeAll(b.data(), b.size() - 3);
      close(fds[1]);
    }
    ChannelReader in3{FdChannel(fds[0])};
    bool threw = false;
    try {
      SerializePacked::readFromUnbuffered(gpu, in3);
    } catch (const DecodeException &) {
      threw = true;
    }
    EXPECT(threw, "truncated channel must throw DecodeException");
    close(fds[0]);
  }
  // SerializePacked.read of one 64 MiB single-segment message (one library
  // call: cpk_read_message_host) against the oracle's bytes, and the same
  // message read as three PackedInputStream.read calls (first word, table,
  // segment: the round-2 sequence)
  {
    const size_t W = 8u << 20;  // 64 MiB of words
    Bytes seg(8 * W, 0);
    uint32_t rs = 777;
    auto rnd = [&]() { return rs = rs * 1103515245u + 12345u, rs >> 8; };
    for (size_t w = 0; w < W; ++w)
      if (rnd() % 2)
        for (int b = 0; b < 8; ++b) seg[8 * w + b] = (rnd() % 4) ? (uint8_t)(1 + rnd() % 255) : 0;
    const std::vector<Bytes> msg = {seg};
    Bytes pk = oracleWrite(msg);
    EXPECT(SerializePacked::write(gpu, msg) == pk, "64 MiB message: write == oracle");
    const int reps = 5;
    double best1 = 1e9, best3 = 1e9;
    for (int r = 0; r < reps; ++r) {
      ArrayInputStream in(pk.data(), pk.size());
      const auto t0 = std::chrono::steady_clock::now();
      auto got = SerializePacked::read(gpu, in);
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      best1 = dt < best1 ? dt : best1;
      EXPECT(got.size() == 1 && got[0] == seg && in.remaining() == 0, "64 MiB message: read == oracle input");
      ArrayInputStream in3(pk.data(), pk.size());
      PackedInputStream pin(gpu, in3);
      Bytes first(8), out(8 * W);
      const auto t1 = std::chrono::steady_clock::now();
      pin.read(first.data(), 8);  // (count 1: no second table read)
      pin.read(out.data(), out.size());
      const double dt3 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
      best3 = dt3 < best3 ? dt3 : best3;
      EXPECT(out == seg, "64 MiB message: per-read sequence");
    }
    std::printf("read 64 MiB single-segment message (%.1f MiB packed): one call %.2f ms = %.2f GiB/s of words; "
                "per-read calls %.2f ms = %.2f GiB/s\n",
                pk.size() / 1048576.0, best1 * 1e3, 8.0 * W / best1 / (1 << 30), best3 * 1e3,
                8.0 * W / best3 / (1 << 30));
  }
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("serialize_packed_test: all passed\n");
  return 0;
}
