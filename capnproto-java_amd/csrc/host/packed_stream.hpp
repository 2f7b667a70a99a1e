// packed_stream.hpp -- C++ mirror of capnproto-java's packed stream API over
// the MI355X codec's C ABI (include/capnp_packed.h).  Same class names,
// argument meaning and error behaviour as the reference
// (runtime/src/main/java/org/capnproto/):
//   ArrayOutputStream   ArrayOutputStream.java:28-62  (IOException when full)
//   ArrayInputStream    ArrayInputStream.java:27-70   (DecodeException at EOF)
//   PackedOutputStream  PackedOutputStream.java:28-213 (write = one piece)
//   PackedInputStream   PackedInputStream.java:28-148  (read fills the buffer)
//   SerializePacked     SerializePacked.java:35-134 (write / read a message
//                       of segments: table piece + one piece per segment;
//                       writeToUnbuffered / readFromUnbuffered over a channel)
//   FdChannel           java.nio.channels.{Readable,Writable}ByteChannel over a
//                       file descriptor (socket, pipe, file)
//   ChannelReader       BufferedInputStreamWrapper.java:28-108's role for the
//                       GPU path (bytes read ahead of the decoder)
// Every byte is produced by the GPU kernels; there is no CPU codec here.
#pragma once

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include <poll.h>
#include <unistd.h>

#include "../../../include/capnp_packed.h"

namespace capnp_amd {

struct DecodeException : std::runtime_error {  // DecodeException.java:24-27
  explicit DecodeException(const std::string &m) : std::runtime_error(m) {}
};
struct IOException : std::runtime_error {
  explicit IOException(const std::string &m) : std::runtime_error(m) {}
};

inline void check(int st, const char *what) {
  if (st == CPK_OK) return;
  std::string m = std::string(what) + ": " + cpk_status_string(st);
  if (st == CPK_ETRUNC || st == CPK_EOVERRUN || st == CPK_ETRAILING || st == CPK_EINVAL ||
      st == CPK_EFRAME)
    throw DecodeException(m);
  throw IOException(m);
}

class Gpu {  // one device context, shared by the streams below
 public:
  explicit Gpu(int device = 0) { check(cpk_ctx_create(device, &ctx_), "cpk_ctx_create"); }
  ~Gpu() { cpk_ctx_destroy(ctx_); }
  Gpu(const Gpu &) = delete;
  Gpu &operator=(const Gpu &) = delete;
  cpk_ctx get() const { return ctx_; }

 private:
  cpk_ctx ctx_ = nullptr;
};

// ---- in-memory channels (ArrayOutputStream / ArrayInputStream) ----
class ArrayOutputStream {
 public:
  ArrayOutputStream(uint8_t *buf, size_t cap) : buf_(buf), cap_(cap) {}
  size_t write(const uint8_t *src, size_t n) {  // ArrayOutputStream.java:36-45
    if (cap_ - pos_ < n) throw IOException("backing buffer was not large enough");
    std::memcpy(buf_ + pos_, src, n);
    pos_ += n;
    return n;
  }
  size_t position() const { return pos_; }
  // getWriteBuffer (ArrayOutputStream.java:47-49): the free part of the
  // backing buffer, filled in place by a caller that then advances past it
  uint8_t *writeBuffer() { return buf_ + pos_; }
  size_t remaining() const { return cap_ - pos_; }
  void advance(size_t n) {
    if (cap_ - pos_ < n) throw IOException("backing buffer was not large enough");
    pos_ += n;
  }

 private:
  uint8_t *buf_;
  size_t cap_, pos_ = 0;
};

class ArrayInputStream {
 public:
  ArrayInputStream(const uint8_t *buf, size_t len) : buf_(buf), len_(len) {}
  const uint8_t *data() const { return buf_ + pos_; }
  size_t remaining() const { return len_ - pos_; }
  void advance(size_t n) { pos_ += n; }
  void requireData() const {  // getReadBuffer at EOF, ArrayInputStream.java:53-58
    if (remaining() == 0) throw DecodeException("Premature EOF while reading buffer");
  }

 private:
  const uint8_t *buf_;
  size_t len_, pos_ = 0;
};

// ---- unbuffered channels --------------------------------------------------
class FdChannel {  // ReadableByteChannel / WritableByteChannel over a descriptor
 public:
  explicit FdChannel(int fd) : fd_(fd) {}
  int fd() const { return fd_; }
  // WritableByteChannel.write until every byte is out
  void writeAll(const uint8_t *p, size_t n) {
    while (n) {
      const ssize_t k = ::write(fd_, p, n);
      if (k < 0 && errno == EINTR) continue;
      if (k <= 0) throw IOException(std::string("channel write: ") + std::strerror(errno));
      p += k;
      n -= (size_t)k;
    }
  }
  // one ReadableByteChannel.read: blocks for >= 1 byte; 0 at end of stream
  size_t readSome(uint8_t *p, size_t cap) {
    for (;;) {
      const ssize_t k = ::read(fd_, p, cap);
      if (k < 0 && errno == EINTR) continue;
      if (k < 0) throw IOException(std::string("channel read: ") + std::strerror(errno));
      return (size_t)k;
    }
  }
  // bytes (or the end of the stream) ready within timeout_ms
  bool ready(int timeout_ms) {
    pollfd q{fd_, POLLIN, 0};
    for (;;) {
      const int r = ::poll(&q, 1, timeout_ms);
      if (r < 0 && errno == EINTR) continue;
      return r > 0;
    }
  }

 private:
  int fd_;
};

// The bytes read from a channel and not yet decoded (the role of
// BufferedInputStreamWrapper.java:28-108 for the GPU path).  A message's
// packed length is known only once it is decoded, so reads may run ahead of
// the message; what they bring in stays here for the next one (the
// reference's wrapper, made per call, would drop it).
class ChannelReader {
 public:
  explicit ChannelReader(FdChannel ch) : ch_(ch), buf_(1 << 16) {}
  const uint8_t *data() const { return buf_.data() + pos_; }
  size_t available() const { return len_ - pos_; }
  void consume(size_t n) { pos_ += n; }
  FdChannel &channel() { return ch_; }
  // one read of what the channel has (blocking for >= 1 byte); false at EOF
  bool fill() {
    if (pos_ == len_) pos_ = len_ = 0;
    if (len_ + 4096 > buf_.size()) {
      if (pos_ >= buf_.size() / 2) {  // compact
        std::memmove(buf_.data(), buf_.data() + pos_, len_ - pos_);
        len_ -= pos_;
        pos_ = 0;
      } else {
        buf_.resize(2 * buf_.size());
      }
    }
    const size_t k = ch_.readSome(buf_.data() + len_, buf_.size() - len_ - 16);
    len_ += k;
    std::memset(buf_.data() + len_, 0, 16);
    return k > 0;
  }

 private:
  FdChannel ch_;
  std::vector<uint8_t> buf_;
  size_t pos_ = 0, len_ = 0;
};

// One message (Serialize.read over PackedInputStream, Serialize.java:119-178)
// from the front of `avail` packed bytes, in one library call
// (cpk_read_message_host: table and segments on the device).  `words` is a
// reusable output buffer, grown when the segments need more (CPK_ENOMEM
// reports how many words); `info` gets the call's info row.
inline int readMessageBytes(Gpu &gpu, const uint8_t *p, size_t avail, uint64_t limit,
                            std::vector<uint64_t> &words, std::vector<uint64_t> &info) {
  info.assign(CPK_MSG_INFO_WORDS, 0);
  for (;;) {
    const int rc = cpk_read_message_host(gpu.get(), p, avail, limit, words.empty() ? nullptr : words.data(),
                                         words.size(), info.data());
    if (rc == CPK_ENOMEM && (int64_t)info[0] == CPK_ENOMEM && info[3] > words.size()) {
      words.resize(info[3]);
      continue;
    }
    return rc;
  }
}

// A message read into one reusable word buffer, its segments views of it:
// what Serialize.read hands MessageReader -- slices of one ByteBuffer
// holding every segment (Serialize.java:164-177) -- without a vector per
// segment per call.  Reused across reads: its buffers only grow.
struct MessageView {
  std::vector<uint64_t> words, info;
  size_t segmentCount() const { return (size_t)info[2]; }
  const uint8_t *segment(size_t i) const { return (const uint8_t *)(words.data() + info[4 + i]); }
  size_t segmentBytes(size_t i) const { return 8 * (size_t)(info[5 + i] - info[4 + i]); }
};

inline std::vector<std::vector<uint8_t>> segmentsOf(const std::vector<uint64_t> &words,
                                                    const std::vector<uint64_t> &info) {
  std::vector<std::vector<uint8_t>> segs;
  const uint8_t *b = (const uint8_t *)words.data();
  for (uint64_t i = 0; i < info[2]; ++i) segs.emplace_back(b + 8 * info[4 + i], b + 8 * info[5 + i]);
  return segs;
}

// ---- PackedOutputStream: write(piece) == one PackedOutputStream.write ----
class PackedOutputStream {
 public:
  PackedOutputStream(Gpu &gpu, ArrayOutputStream &inner) : gpu_(gpu), inner_(inner) {}
  // PackedOutputStream.java:35-205: len must be word-aligned; returns len
  size_t write(const uint8_t *in, size_t len) {
    if (len % 8) throw std::invalid_argument("PackedOutputStream input must be word-aligned");
    std::vector<uint64_t> swo = {0, len / 8};
    std::vector<uint8_t> out(cpk_batch_packed_capacity(swo.data(), 1));
    std::vector<uint64_t> off(2);
    if (len) {
      check(cpk_encode_host(gpu_.get(), in, swo.data(), 1, out.data(), out.size(), off.data()),
            "cpk_encode_host");
      inner_.write(out.data(), off[1]);
    }
    return len;
  }

 private:
  Gpu &gpu_;
  ArrayOutputStream &inner_;
};

// ---- PackedInputStream: read(buf) fills buf exactly, like the reference ---
class PackedInputStream {
 public:
  PackedInputStream(Gpu &gpu, ArrayInputStream &inner) : gpu_(gpu), inner_(inner) {}
  size_t read(uint8_t *out, size_t len) {  // PackedInputStream.java:35-140
    if (len == 0) return 0;
    if (len % 8) throw DecodeException("PackedInputStream reads must be word-aligned");
    inner_.requireData();
    std::vector<uint64_t> swo = {0, len / 8};
    std::vector<uint64_t> bounds(2);
    int32_t st = 0;
    check(cpk_decode_stream_host(gpu_.get(), inner_.data(), inner_.remaining(), swo.data(), 1,
                                 out, bounds.data(), &st),
          "PackedInputStream.read");
    inner_.advance(bounds[1]);
    return len;
  }

 private:
  Gpu &gpu_;
  ArrayInputStream &inner_;
};

// ---- SerializePacked: a message = [segment table, seg0, ...] pieces -------
struct SerializePacked {
  // Serialize.writeSegmentTable (Serialize.java:256-273) + one write per
  // segment (:283-287), all pieces in ONE batched GPU call; the segments are
  // packed where they lie (cpk_encode_host_gather, no concatenation).
  static std::vector<uint8_t> write(Gpu &gpu, const std::vector<std::vector<uint8_t>> &segs) {
    const size_t n = segs.size();
    const size_t table_ints = (n + 2) & ~size_t(1);
    std::vector<uint8_t> table(4 * table_ints, 0);
    uint32_t v = (uint32_t)n - 1;
    std::memcpy(table.data(), &v, 4);
    std::vector<const void *> pieces = {table.data()};
    std::vector<uint64_t> swo = {0, table.size() / 8};
    for (size_t i = 0; i < n; ++i) {
      if (segs[i].size() % 8) throw std::invalid_argument("segment not word-aligned");
      uint32_t w = (uint32_t)(segs[i].size() / 8);
      std::memcpy(table.data() + 4 * (i + 1), &w, 4);
      pieces.push_back(segs[i].empty() ? nullptr : segs[i].data());
      swo.push_back(swo.back() + w);
    }
    std::vector<uint8_t> out(cpk_batch_packed_capacity(swo.data(), (uint32_t)n + 1));
    std::vector<uint64_t> off(n + 2);
    check(cpk_encode_host_gather(gpu.get(), pieces.data(), swo.data(), (uint32_t)n + 1,
                                 out.data(), out.size(), off.data()),
          "SerializePacked.write");
    out.resize(off[n + 1]);
    return out;
  }

  // SerializePacked.write into the caller's ArrayOutputStream: the packed
  // bytes land in its backing buffer in place (getWriteBuffer,
  // ArrayOutputStream.java:47-49), nothing allocated per call; a message
  // that does not fit is the reference's IOException (:40-42).  Returns the
  // bytes written.
  static size_t write(Gpu &gpu, const std::vector<std::vector<uint8_t>> &segs, ArrayOutputStream &out) {
    const size_t n = segs.size();
    thread_local std::vector<uint8_t> table;
    thread_local std::vector<const void *> pieces;
    thread_local std::vector<uint64_t> swo, off;
    const size_t table_ints = (n + 2) & ~size_t(1);
    table.assign(4 * table_ints, 0);
    const uint32_t v = (uint32_t)n - 1;
    std::memcpy(table.data(), &v, 4);
    pieces.assign(1, table.data());
    swo.assign(1, 0);
    swo.push_back(table.size() / 8);
    for (size_t i = 0; i < n; ++i) {
      if (segs[i].size() % 8) throw std::invalid_argument("segment not word-aligned");
      const uint32_t w = (uint32_t)(segs[i].size() / 8);
      std::memcpy(table.data() + 4 * (i + 1), &w, 4);
      pieces.push_back(segs[i].empty() ? nullptr : segs[i].data());
      swo.push_back(swo.back() + w);
    }
    off.resize(n + 2);
    check(cpk_encode_host_gather(gpu.get(), pieces.data(), swo.data(), (uint32_t)n + 1, out.writeBuffer(),
                                 out.remaining(), off.data()),
          "SerializePacked.write");
    out.advance(off[n + 1]);
    return off[n + 1];
  }

  // SerializePacked.read into a reusable MessageView (its segments views of
  // one word buffer, as Serialize.read slices one ByteBuffer).
  static void read(Gpu &gpu, ArrayInputStream &in, MessageView &msg, uint64_t traversal_limit_words = 8ull << 20) {
    in.requireData();
    check(readMessageBytes(gpu, in.data(), in.remaining(), traversal_limit_words, msg.words, msg.info),
          "SerializePacked.read");
    in.advance(msg.info[1]);
  }

  // Serialize.read (Serialize.java:119-178) over PackedInputStream: the
  // first word, the rest of the table and every segment in ONE library call
  // (cpk_read_message_host); the stream advances past the message only.
  static std::vector<std::vector<uint8_t>> read(Gpu &gpu, ArrayInputStream &in,
                                                uint64_t traversal_limit_words = 8ull << 20) {
    in.requireData();
    thread_local std::vector<uint64_t> words, info;
    check(readMessageBytes(gpu, in.data(), in.remaining(), traversal_limit_words, words, info),
          "SerializePacked.read");
    in.advance(info[1]);
    return segmentsOf(words, info);
  }

  // SerializePacked.writeToUnbuffered (SerializePacked.java:119-134): the
  // message packed on the GPU, then every byte written to the channel.
  static void writeToUnbuffered(Gpu &gpu, FdChannel &out, const std::vector<std::vector<uint8_t>> &segs) {
    const std::vector<uint8_t> b = write(gpu, segs);
    out.writeAll(b.data(), b.size());
  }

  // SerializePacked.readFromUnbuffered (SerializePacked.java:84-96): as read()
  // above, over a channel.  A try on the bytes buffered so far; if they end
  // inside the message (CPK_ETRUNC) more are read -- everything the channel
  // has, then, until twice as many as at the last try are buffered, more as
  // they arrive unless the channel stays idle for a millisecond (so a
  // message of M bytes costs O(log M) tries, and a paused peer never waits on
  // us).  The channel's end inside the message is the reference's "premature
  // EOF" (BufferedInputStreamWrapper.java:98-108).
  static std::vector<std::vector<uint8_t>> readFromUnbuffered(Gpu &gpu, ChannelReader &in,
                                                              uint64_t traversal_limit_words = 8ull << 20) {
    thread_local std::vector<uint64_t> words, info;
    size_t tried = 0;
    for (;;) {
      if (in.available() > tried) {
        const int rc = readMessageBytes(gpu, in.data(), in.available(), traversal_limit_words, words, info);
        if (rc == CPK_OK) {
          in.consume(info[1]);
          return segmentsOf(words, info);
        }
        if (rc != CPK_ETRUNC) check(rc, "readFromUnbuffered");
        tried = in.available();
      }
      if (!in.fill()) throw DecodeException("premature EOF");
      while (in.available() < 2 * tried && in.channel().ready(1))
        if (!in.fill()) break;
    }
  }

  // SerializePacked.tryReadFromUnbuffered (SerializePacked.java:67-79):
  // nothing when the channel ends before a message starts.
  static std::optional<std::vector<std::vector<uint8_t>>> tryReadFromUnbuffered(
      Gpu &gpu, ChannelReader &in, uint64_t traversal_limit_words = 8ull << 20) {
    if (in.available() == 0 && !in.fill()) return std::nullopt;
    return readFromUnbuffered(gpu, in, traversal_limit_words);
  }

  using Message = std::vector<std::vector<uint8_t>>;  // its segments

  // writeToUnbuffered for many messages, packed in one GPU call
  static void writeMessagesToUnbuffered(Gpu &gpu, FdChannel &out, const std::vector<Message> &msgs) {
    const std::vector<uint8_t> b = writeMessages(gpu, msgs);
    out.writeAll(b.data(), b.size());
  }

  // write() for each message, ONE GPU call: the segment tables are built and
  // packed on the device (cpk_encode_messages_host).  Returns the packed
  // bytes, messages back to back; msg_off[m] = message m's first byte.
  static std::vector<uint8_t> writeMessages(Gpu &gpu, const std::vector<Message> &msgs,
                                            std::vector<uint64_t> *msg_off = nullptr) {
    std::vector<uint8_t> words;
    std::vector<uint64_t> swo = {0}, mso = {0};
    uint64_t cap = 16;
    for (auto &m : msgs) {
      for (auto &sg : m) {
        if (sg.size() % 8) throw std::invalid_argument("segment not word-aligned");
        words.insert(words.end(), sg.begin(), sg.end());
        swo.push_back(words.size() / 8);
        cap += cpk_packed_bound(sg.size() / 8);
      }
      mso.push_back(swo.size() - 1);
      cap += 10 * ((m.size() + 2) / 2 + 1);
    }
    const uint32_t nseg = (uint32_t)swo.size() - 1, nm = (uint32_t)msgs.size();
    words.resize(words.size() + 8);
    std::vector<uint8_t> out(cap);
    std::vector<uint64_t> off(nm + nseg + 1);
    check(cpk_encode_messages_host(gpu.get(), words.data(), swo.data(), nseg, mso.data(), nm,
                                   out.data(), out.size(), off.data()),
          "SerializePacked.writeMessages");
    out.resize(off[nm + nseg]);
    if (msg_off) {
      msg_off->clear();
      for (uint32_t m = 0; m < nm; ++m) msg_off->push_back(off[mso[m] + m]);
      msg_off->push_back(off[nm + nseg]);
    }
    return out;
  }

  // read() for each message, ONE GPU pass: message m is
  // packed[msg_off[m], msg_off[m+1]); tables read and validated on the
  // device (cpk_decode_messages_host).  Throws the first bad message's error.
  static std::vector<Message> readMessages(Gpu &gpu, const std::vector<uint8_t> &packed,
                                           const std::vector<uint64_t> &msg_off,
                                           uint64_t traversal_limit_words = 8ull << 20) {
    const uint32_t nm = (uint32_t)msg_off.size() - 1;
    std::vector<uint64_t> mso(nm + 1), tot(2);
    std::vector<int32_t> mst(nm ? nm : 1);
    int rc = cpk_decode_messages_host(gpu.get(), packed.data(), msg_off.data(), nm,
                                      traversal_limit_words, nullptr, 0, nullptr, 0, mso.data(),
                                      mst.data(), tot.data());
    std::vector<uint8_t> out(8 * tot[0] + 8);
    std::vector<uint64_t> swo(tot[1] + 1);
    if (rc == CPK_ENOMEM)
      rc = cpk_decode_messages_host(gpu.get(), packed.data(), msg_off.data(), nm,
                                    traversal_limit_words, out.data(), tot[0], swo.data(),
                                    (uint32_t)tot[1], mso.data(), mst.data(), tot.data());
    check(rc, "SerializePacked.readMessages");
    std::vector<Message> res(nm);
    for (uint32_t m = 0; m < nm; ++m)
      for (uint64_t j = mso[m]; j < mso[m + 1]; ++j)
        res[m].emplace_back(out.begin() + 8 * swo[j], out.begin() + 8 * swo[j + 1]);
    return res;
  }
};

}  // namespace capnp_amd
