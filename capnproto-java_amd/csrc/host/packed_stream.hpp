// packed_stream.hpp -- C++ mirror of capnproto-java's packed stream API over
// the MI355X codec's C ABI (include/capnp_packed.h).  Same class names,
// argument meaning and error behaviour as the reference
// (runtime/src/main/java/org/capnproto/):
//   ArrayOutputStream   ArrayOutputStream.java:28-62  (IOException when full)
//   ArrayInputStream    ArrayInputStream.java:27-70   (DecodeException at EOF)
//   PackedOutputStream  PackedOutputStream.java:28-213 (write = one piece)
//   PackedInputStream   PackedInputStream.java:28-148  (read fills the buffer)
//   SerializePacked     SerializePacked.java:35-134 (write / read a message
//                       of segments: table piece + one piece per segment)
// Every byte is produced by the GPU kernels; there is no CPU codec here.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

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

  // Serialize.read (Serialize.java:119-178) over PackedInputStream.
  static std::vector<std::vector<uint8_t>> read(Gpu &gpu, ArrayInputStream &in,
                                                uint64_t traversal_limit_words = 8ull << 20) {
    PackedInputStream pin(gpu, in);
    uint8_t first[8];
    pin.read(first, 8);
    int32_t raw, s0;
    std::memcpy(&raw, first, 4);
    std::memcpy(&s0, first + 4, 4);
    if (raw < 0 || raw > 511) throw DecodeException("segment count must be between 0 and 512");
    if (s0 < 0) throw DecodeException("segment 0 has more than 2^31 words, which is unsupported");
    const uint32_t count = (uint32_t)raw + 1;
    std::vector<uint64_t> sizes = {(uint64_t)s0};
    uint64_t total = (uint64_t)s0;
    if (count > 1) {
      std::vector<uint8_t> rest(4 * (count & ~1u));
      pin.read(rest.data(), rest.size());
      for (uint32_t i = 0; i + 1 < count; ++i) {
        int32_t s;
        std::memcpy(&s, rest.data() + 4 * i, 4);
        if (s < 0) throw DecodeException("segment has more than 2^31 words");
        sizes.push_back((uint64_t)s);
        total += (uint64_t)s;
      }
    }
    if (total > traversal_limit_words) throw DecodeException("Message size exceeds traversal limit.");
    for (auto s : sizes)  // makeByteBufferForWords (Serialize.java:45-53)
      if (s > (1u << 28) - 1) throw DecodeException("segment has too many words");
    // all segments in one stream-decode call (pieces back to back)
    std::vector<uint64_t> swo = {0};
    for (auto s : sizes) swo.push_back(swo.back() + s);
    std::vector<uint8_t> out(8 * total + 8);
    std::vector<uint64_t> bounds(count + 1);
    std::vector<int32_t> st(count);
    if (total) {
      in.requireData();
      check(cpk_decode_stream_host(gpu.get(), in.data(), in.remaining(), swo.data(), count,
                                   out.data(), bounds.data(), st.data()),
            "SerializePacked.read");
      in.advance(bounds[count]);
    }
    std::vector<std::vector<uint8_t>> segs;
    for (uint32_t i = 0; i < count; ++i)
      segs.emplace_back(out.begin() + 8 * swo[i], out.begin() + 8 * swo[i + 1]);
    return segs;
  }

  using Message = std::vector<std::vector<uint8_t>>;  // its segments

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
