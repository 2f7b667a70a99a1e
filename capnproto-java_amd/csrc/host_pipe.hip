// Host-memory forms of the batch codec (cpk_encode_host / cpk_decode_host):
// the socket/file ByteBuffer path of SerializePacked.java:75-96, :119-134.
// Included from packed_codec.hip.
//
// The batch is cut into chunks of whole pieces (~CPK_HOST_CHUNK_MB of
// unpacked words each) that flow through two staging slots, each a pinned
// host buffer pair and a device buffer pair:
//
//   host threads   copy-in(k) ............ copy-out(k-2)
//   copy stream    H2D(k)
//   codec stream          kernels(k) + its offsets / statuses
//   copy stream 2                   D2H(k-1)
//
// Pageable hipMemcpy moves 9-14 GiB/s host->device on the box; pinned DMA
// runs at 53 GiB/s each way (full duplex) and a threaded memcpy into pinned
// memory at 80-100 GiB/s (tools/host_copy_probe.cpp), so the pipeline is
// bounded by the DMA of the larger side.  Kernels of consecutive chunks run
// in order on one stream (they share the context's workspace).

struct HostSlot {
  void *pin_in = nullptr, *pin_out = nullptr, *d_in = nullptr, *d_out = nullptr;
  uint64_t *pin_meta = nullptr, *d_meta = nullptr;
  hipEvent_t eh = nullptr, ek = nullptr, ed = nullptr;  // H2D done, kernels done, D2H done
  uint64_t cap_in = 0, cap_out = 0, cap_meta = 0;       // bytes, bytes, u64 entries
};

struct HostPipe {
  hipStream_t sh = nullptr, sk = nullptr, sd = nullptr;
  HostSlot slot[2];
  bool ok = false;
};

namespace {

int host_threads() {
  const char *e = getenv("CPK_HOST_THREADS");
  const int t = e ? atoi(e) : 8;
  return t < 1 ? 1 : (t > 64 ? 64 : t);
}

uint64_t host_chunk_bytes() {
  // (CPK_HOST_CHUNK_KB: small chunks for tests)
  if (const char *k = getenv("CPK_HOST_CHUNK_KB")) return (uint64_t)atoll(k) << 10 ?: 1;
  const char *e = getenv("CPK_HOST_CHUNK_MB");
  return (uint64_t)(e ? atoll(e) : 256) << 20 ?: 1;
}

// memcpy over host threads (page-aligned parts)
void par_copy(void *dst, const void *src, uint64_t bytes) {
  const int nt = host_threads();
  if (bytes < (4u << 20) || nt == 1) {
    memcpy(dst, src, bytes);
    return;
  }
  const uint64_t per = ((bytes + nt - 1) / nt + 4095) & ~4095ull;
  std::vector<std::thread> ts;
  for (int i = 1; i < nt; ++i) {
    const uint64_t a = per * i;
    if (a >= bytes) break;
    const uint64_t b = a + per < bytes ? a + per : bytes;
    ts.emplace_back([=] { memcpy((char *)dst + a, (const char *)src + a, b - a); });
  }
  memcpy(dst, src, per < bytes ? per : bytes);
  for (auto &t : ts) t.join();
}

void slot_free_buffers(HostSlot &s) {
  if (s.pin_in) hipHostFree(s.pin_in);
  if (s.pin_out) hipHostFree(s.pin_out);
  if (s.pin_meta) hipHostFree(s.pin_meta);
  if (s.d_in) hipFree(s.d_in);
  if (s.d_out) hipFree(s.d_out);
  if (s.d_meta) hipFree(s.d_meta);
  s.pin_in = s.pin_out = s.d_in = s.d_out = nullptr;
  s.pin_meta = s.d_meta = nullptr;
  s.cap_in = s.cap_out = s.cap_meta = 0;
}

void pipe_free_buffers(HostPipe *p) {
  for (HostSlot &s : p->slot) slot_free_buffers(s);
}

void pipe_destroy(HostPipe *p) {
  if (!p) return;
  if (p->sh) hipStreamSynchronize(p->sh);
  if (p->sk) hipStreamSynchronize(p->sk);
  if (p->sd) hipStreamSynchronize(p->sd);
  pipe_free_buffers(p);
  for (HostSlot &s : p->slot) {
    if (s.eh) hipEventDestroy(s.eh);
    if (s.ek) hipEventDestroy(s.ek);
    if (s.ed) hipEventDestroy(s.ed);
  }
  if (p->sh) hipStreamDestroy(p->sh);
  if (p->sk) hipStreamDestroy(p->sk);
  if (p->sd) hipStreamDestroy(p->sd);
  delete p;
}

// the context's pipe with staging of at least the given sizes (grow-only)
// One large transfer through a pinned slot, pipelined in chunks of
// kPipeChunk: the threaded host copy of chunk k+1 overlaps the DMA of chunk k
// (single-slot host forms: one message or stream of unknown length).
constexpr uint64_t kPipeChunk = 16ull << 20;
// host src -> pinned -> device: every chunk's H2D is enqueued on s as soon as
// its bytes are in the pinned buffer (which is not reused before s drains)
int h2d_pipelined(void *dev, void *pin, const void *src, uint64_t bytes, hipStream_t s) {
  for (uint64_t a = 0; a < bytes; a += kPipeChunk) {
    const uint64_t n = bytes - a < kPipeChunk ? bytes - a : kPipeChunk;
    par_copy((char *)pin + a, (const char *)src + a, n);
    if (hipMemcpyAsync((char *)dev + a, (const char *)pin + a, n, hipMemcpyHostToDevice, s) != hipSuccess)
      return CPK_EDEVICE;
  }
  return CPK_OK;
}
// device -> pinned -> host dst: two chunks' D2H in flight on s, each copied
// on to dst once its event fires (e0 / e1: two free events of the slot)
int d2h_pipelined(void *dst, void *pin, const void *dev, uint64_t bytes, hipStream_t s, hipEvent_t e0,
                  hipEvent_t e1) {
  const uint64_t nc = (bytes + kPipeChunk - 1) / kPipeChunk;
  hipEvent_t ev[2] = {e0, e1};
  auto issue = [&](uint64_t k) {
    const uint64_t a = k * kPipeChunk, n = bytes - a < kPipeChunk ? bytes - a : kPipeChunk;
    return hipMemcpyAsync((char *)pin + a, (const char *)dev + a, n, hipMemcpyDeviceToHost, s) == hipSuccess &&
           hipEventRecord(ev[k & 1], s) == hipSuccess;
  };
  for (uint64_t k = 0; k < nc && k < 2; ++k)
    if (!issue(k)) return CPK_EDEVICE;
  for (uint64_t k = 0; k < nc; ++k) {
    if (hipEventSynchronize(ev[k & 1]) != hipSuccess) return CPK_EDEVICE;
    const uint64_t a = k * kPipeChunk, n = bytes - a < kPipeChunk ? bytes - a : kPipeChunk;
    if (k + 2 < nc && !issue(k + 2)) return CPK_EDEVICE;  // (its event: chunk k's, now consumed)
    par_copy((char *)dst + a, (const char *)pin + a, n);
  }
  return CPK_OK;
}

// (nslots: the slots the caller stages through -- the single-slot forms, one
// message or stream of unknown length, grow slot 0 alone, so a large one
// does not also pin and allocate the same again in slot 1)
int pipe_get(cpk_ctx ctx, uint64_t in_bytes, uint64_t out_bytes, uint64_t meta, HostPipe **out, int nslots = 2) {
  HostPipe *p = ctx->pipe;
  if (!p) {
    p = new HostPipe();
    ctx->pipe = p;
    bool ok = hipStreamCreateWithFlags(&p->sh, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&p->sk, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&p->sd, hipStreamNonBlocking) == hipSuccess;
    for (HostSlot &s : p->slot)
      ok = ok && hipEventCreateWithFlags(&s.eh, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&s.ek, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&s.ed, hipEventDisableTiming) == hipSuccess;
    p->ok = ok;
  }
  if (!p->ok) return CPK_EDEVICE;
  in_bytes = (in_bytes + 64 + 4095) & ~4095ull;  // (+ the decoder's zero read slack)
  out_bytes = (out_bytes + 64 + 4095) & ~4095ull;
  for (int i = 0; i < nslots; ++i) {
    HostSlot &s = p->slot[i];
    if (in_bytes <= s.cap_in && out_bytes <= s.cap_out && meta <= s.cap_meta) continue;
    const uint64_t ci = in_bytes > s.cap_in ? in_bytes : s.cap_in;
    const uint64_t co = out_bytes > s.cap_out ? out_bytes : s.cap_out;
    const uint64_t cm = meta > s.cap_meta ? meta : s.cap_meta;
    slot_free_buffers(s);
    if (hipHostMalloc(&s.pin_in, ci, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.pin_out, co, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&s.pin_meta, cm * 8, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&s.d_in, ci) != hipSuccess || hipMalloc(&s.d_out, co) != hipSuccess ||
        hipMalloc((void **)&s.d_meta, cm * 8) != hipSuccess) {
      pipe_free_buffers(p);
      return CPK_ENOMEM;
    }
    s.cap_in = ci;
    s.cap_out = co;
    s.cap_meta = cm;
  }
  *out = p;
  return CPK_OK;
}

// Small batches (<= cpk::kSpSmallWords words, pieces and tables): ONE
// kernel launch (cpk::sp_small_kernel, one workgroup) reads the words from
// the pinned slot and writes the packed bytes and offsets into pinned memory
// in place, then one sync -- no DMA, no second kernel, no second sync.
// lay(pin_words, desc) puts the pieces' words into the slot and their
// (first word, words) pairs, in output order, into desc.
// (CPK_HOST_CHUNK_KB, the tests' small chunks, keeps batches on the pipeline)
bool small_ok(uint64_t words, uint64_t np) {
  return words <= cpk::kSpSmallWords && np <= cpk::kSpSmallPieces && !getenv("CPK_NO_SMALL") &&
         !getenv("CPK_HOST_CHUNK_KB");
}

template <class Lay>
int small_encode(cpk_ctx ctx, uint64_t np, uint64_t words, Lay lay, void *h_out, uint64_t h_out_cap,
                 uint64_t *h_out_off, uint64_t off_base) {
  HostPipe *p = nullptr;
  const uint64_t ocap = 9 * words + np + 16;
  // meta: desc [2 np] | out_off [np + 1] | completion flag
  int rc = pipe_get(ctx, 8 * words + 64, ocap + 64, 3 * np + 2, &p, 1);
  if (rc) return rc;
  HostSlot &s = p->slot[0];
  uint64_t *desc = s.pin_meta, *off = desc + 2 * np;
  TrClock tc(ctx);
  lay((uint64_t *)s.pin_in, desc);
  tc.mark(kTrWIn);
  const uint64_t seq = small_arm(ctx, off + np + 1);
  cpk::SpSmallArgs da = {};
  if (np <= cpk::kSpArgPieces) memcpy(da.d, desc, 16 * np);
  hipLaunchKernelGGL(cpk::sp_small_kernel, dim3(1), dim3(cpk::kSpThreads), cpk::kSpSmallLds, p->sk,
                     (const uint64_t *)s.pin_in, (const uint64_t *)desc, (uint32_t)np, (uint8_t *)s.pin_out, off,
                     ocap, ctx->tickets + cpk::kTkErr, off + np + 1, seq, da);
  if (hipGetLastError() != hipSuccess) return CPK_EDEVICE;
  tc.mark(kTrWLaunch);
  if (small_wait(ctx, p->sk, off + np + 1, seq)) return CPK_EDEVICE;
  tc.mark(kTrWWait);
  const uint64_t P = off[np];
  if (P > ocap) return CPK_EDEVICE;
  if (P > h_out_cap) return CPK_ENOMEM;
  memcpy(h_out, s.pin_out, P);
  for (uint64_t j = 0; j <= np; ++j) h_out_off[j] = off_base + off[j];
  tc.mark(kTrWOut);
  return CPK_OK;
}

struct HostChunk {
  uint32_t i0, i1;       // pieces [i0, i1)
  uint64_t in0, in_len;  // input bytes (encode: words * 8; decode: packed range)
  uint64_t out_cap;      // output bytes the chunk may produce
  uint64_t maxw;         // largest piece, words
};

// chunks of whole pieces, each about `target` bytes of unpacked words (a
// piece larger than that is a chunk of its own); decode also bounds the
// packed bytes of a chunk
std::vector<HostChunk> host_chunks(const uint64_t *swo, const uint64_t *in_off, uint32_t n,
                                   uint64_t target) {
  std::vector<HostChunk> cs;
  uint32_t i = 0;
  while (i < n) {
    HostChunk c{i, i, 0, 0, 0, 0};
    uint64_t words = 0, pk = 0, cap = 0;
    while (c.i1 < n) {
      const uint64_t w = swo[c.i1 + 1] - swo[c.i1];
      const uint64_t p = in_off ? in_off[c.i1 + 1] - in_off[c.i1] : 0;
      if (c.i1 > c.i0 && ((words + w) * 8 > target || pk + p > target)) break;
      words += w;
      pk += p;
      cap += cpk_packed_bound(w);
      c.maxw = w > c.maxw ? w : c.maxw;
      ++c.i1;
    }
    if (in_off) {
      c.in0 = in_off[c.i0];
      c.in_len = pk;
      c.out_cap = words * 8;
    } else {
      c.in0 = swo[c.i0] * 8;
      c.in_len = words * 8;
      c.out_cap = cap + 16;
    }
    cs.push_back(c);
    i = c.i1;
  }
  return cs;
}

// wait for everything the pipe has in flight (error paths)
void pipe_drain(HostPipe *p) {
  hipStreamSynchronize(p->sh);
  hipStreamSynchronize(p->sk);
  hipStreamSynchronize(p->sd);
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {

// piece j of the chunk is 8 * (swo[j+1] - swo[j]) bytes at pieces[j]; they go
// back to back into `dst` (pinned staging), split over host threads by bytes
void gather_copy(uint8_t *dst, const void *const *pieces, const uint64_t *swo, uint32_t i0,
                 uint32_t i1) {
  const uint64_t bytes = 8 * (swo[i1] - swo[i0]);
  const int T = host_threads();
  auto run = [=](uint32_t a, uint32_t b) {
    for (uint32_t j = a; j < b; ++j)
      if (swo[j + 1] > swo[j])
        memcpy(dst + 8 * (swo[j] - swo[i0]), pieces[j], 8 * (swo[j + 1] - swo[j]));
  };
  if (T <= 1 || bytes < (4u << 20)) {
    run(i0, i1);
    return;
  }
  std::vector<std::thread> ts;
  uint32_t a = i0;
  for (int t = 1; t <= T && a < i1; ++t) {
    const uint64_t goal = swo[i0] + (swo[i1] - swo[i0]) * t / T;
    uint32_t b = a;
    while (b < i1 && (swo[b] < goal || b == a)) ++b;
    if (t == T) b = i1;
    ts.emplace_back(run, a, b);
    a = b;
  }
  for (auto &t : ts) t.join();
}

// cpk_encode_host / cpk_encode_host_gather: `copy_in` fills a chunk's pinned
// input slot
template <class CopyIn>
int encode_host_impl(cpk_ctx ctx, CopyIn copy_in, const uint64_t *h_swo, uint32_t n, void *h_out,
                     uint64_t h_out_cap, uint64_t *h_out_off, const uint8_t *contig = nullptr) {
  if (n == 0) {
    h_out_off[0] = 0;
    return CPK_OK;
  }
  for (uint32_t i = 0; i < n; ++i)
    if (h_swo[i + 1] < h_swo[i]) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  if (small_ok(h_swo[n] - h_swo[0], n)) {
    // (in0: the words' absolute byte offset in the caller's buffer, as
    // host_chunks sets it; the gather form copies piece by piece)
    const HostChunk all{0, n, 8 * h_swo[0], 8 * (h_swo[n] - h_swo[0]), 0, 0};
    return small_encode(
        ctx, n, h_swo[n] - h_swo[0],
        [&](uint64_t *pin, uint64_t *desc) {
          copy_in((uint8_t *)pin, all);
          for (uint32_t i = 0; i < n; ++i) {
            desc[2 * i] = h_swo[i] - h_swo[0];
            desc[2 * i + 1] = h_swo[i + 1] - h_swo[i];
          }
        },
        h_out, h_out_cap, h_out_off, 0);
  }
  const std::vector<HostChunk> cs = host_chunks(h_swo, nullptr, n, host_chunk_bytes());
  uint64_t mi = 0, mo = 0, mm = 0;
  for (const HostChunk &c : cs) {
    mi = c.in_len > mi ? c.in_len : mi;
    mo = c.out_cap > mo ? c.out_cap : mo;
    mm = c.i1 - c.i0 > mm ? c.i1 - c.i0 : mm;
  }
  HostPipe *p = nullptr;
  int rc = pipe_get(ctx, mi, mo, 2 * (mm + 1), &p);
  if (rc) return rc;
  uint8_t *dst = (uint8_t *)h_out;
  uint64_t base = 0;          // output bytes so far
  const size_t K = cs.size();
  TrClock tc(ctx);
  // one large chunk (e.g. a single big piece): nothing to overlap it with,
  // so its own transfers are pipelined in 16 MiB chunks instead
  const bool one = K == 1 && cs[0].in_len >= 2 * kPipeChunk;
  for (size_t k = 0; k <= K + 1 && rc == CPK_OK; ++k) {
    if (k < K) {  // copy-in, H2D, kernels of chunk k
      const HostChunk &c = cs[k];
      HostSlot &s = p->slot[k & 1];
      const uint32_t nk = c.i1 - c.i0;
      for (uint32_t j = 0; j <= nk; ++j) s.pin_meta[j] = h_swo[c.i0 + j] - h_swo[c.i0];
      if (one && contig) {
        if (h2d_pipelined(s.d_in, s.pin_in, contig + c.in0, c.in_len, p->sh)) {
          rc = CPK_EDEVICE;
          break;
        }
      } else {
        copy_in((uint8_t *)s.pin_in, c);
        if (c.in_len && hipMemcpyAsync(s.d_in, s.pin_in, c.in_len, hipMemcpyHostToDevice, p->sh)) {
          rc = CPK_EDEVICE;
          break;
        }
      }
      tc.mark(kTrWIn);
      if (hipMemcpyAsync(s.d_meta, s.pin_meta, (nk + 1) * 8ull, hipMemcpyHostToDevice, p->sh) ||
          hipEventRecord(s.eh, p->sh) || hipStreamWaitEvent(p->sk, s.eh, 0) ||
          (k >= 2 && hipStreamWaitEvent(p->sk, s.ed, 0))) {  // (d_out free: chunk k-2's D2H)
        rc = CPK_EDEVICE;
        break;
      }
      rc = cpk_encode_batch(ctx, s.d_in, s.d_meta, nk, c.maxw ? c.maxw : 1, s.d_out,
                            s.d_meta + nk + 1, p->sk);
      if (rc) break;
      if (hipMemcpyAsync(s.pin_meta + nk + 1, s.d_meta + nk + 1, (nk + 1) * 8ull,
                         hipMemcpyDeviceToHost, p->sk) ||
          hipEventRecord(s.ek, p->sk)) {
        rc = CPK_EDEVICE;
        break;
      }
      tc.mark(kTrWLaunch);
    }
    if (k >= 1 && k - 1 < K) {  // chunk k-1: offsets, then its D2H
      const HostChunk &c = cs[k - 1];
      HostSlot &s = p->slot[(k - 1) & 1];
      const uint32_t nk = c.i1 - c.i0;
      if (hipEventSynchronize(s.ek)) {
        rc = CPK_EDEVICE;
        break;
      }
      tc.mark(kTrWWait);
      const uint64_t *off = s.pin_meta + nk + 1;
      const uint64_t P = off[nk];
      if (P > c.out_cap) {  // (cannot happen: a piece over its hint)
        rc = CPK_EDEVICE;
        break;
      }
      if (base + P > h_out_cap) {
        rc = CPK_ENOMEM;
        break;
      }
      for (uint32_t j = 0; j <= nk; ++j) h_out_off[c.i0 + j] = base + off[j];
      if (one && P >= 2 * kPipeChunk) {
        // (the one chunk's copy-out under its own D2H; the events of the
        // other slot are free)
        if (d2h_pipelined(dst + base, s.pin_out, s.d_out, P, p->sd, p->slot[1].eh, p->slot[1].ed)) {
          rc = CPK_EDEVICE;
          break;
        }
        base += P;
        break;
      }
      if ((P && hipMemcpyAsync(s.pin_out, s.d_out, P, hipMemcpyDeviceToHost, p->sd)) ||
          hipEventRecord(s.ed, p->sd)) {
        rc = CPK_EDEVICE;
        break;
      }
      base += P;
    }
    if (k >= 2) {  // chunk k-2: copy-out
      const HostChunk &c = cs[k - 2];
      HostSlot &s = p->slot[k & 1];
      if (hipEventSynchronize(s.ed)) {
        rc = CPK_EDEVICE;
        break;
      }
      tc.mark(kTrWWait);
      const uint64_t o0 = h_out_off[c.i0], o1 = h_out_off[c.i1];
      par_copy(dst + o0, s.pin_out, o1 - o0);
      tc.mark(kTrWOut);
    }
  }
  if (rc) {
    pipe_drain(p);
    return rc;
  }
  // (a piece over its hint cannot occur: each chunk's hint is its largest piece)
  rc = cpk_ctx_take_error(ctx, p->sk);
  tc.mark(kTrWWait);
  return rc;
}

}  // namespace

extern "C" {

int cpk_encode_host(cpk_ctx ctx, const void *h_in, const uint64_t *h_swo, uint32_t n,
                    void *h_out, uint64_t h_out_cap, uint64_t *h_out_off) {
  if (!ctx || !h_swo || !h_out_off || (n && ((!h_in && h_swo[n] > h_swo[0]) || !h_out)))
    return CPK_EINVAL;
  const uint8_t *src = (const uint8_t *)h_in;
  return encode_host_impl(
      ctx, [&](uint8_t *pin, const HostChunk &c) { par_copy(pin, src + c.in0, c.in_len); }, h_swo,
      n, h_out, h_out_cap, h_out_off, src);
}

int cpk_encode_host_gather(cpk_ctx ctx, const void *const *h_pieces, const uint64_t *h_swo,
                           uint32_t n, void *h_out, uint64_t h_out_cap, uint64_t *h_out_off) {
  if (!ctx || !h_swo || !h_out_off || (n && (!h_pieces || !h_out))) return CPK_EINVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (h_swo[i + 1] > h_swo[i] && !h_pieces[i]) return CPK_EINVAL;
  return encode_host_impl(
      ctx,
      [&](uint8_t *pin, const HostChunk &c) { gather_copy(pin, h_pieces, h_swo, c.i0, c.i1); },
      h_swo, n, h_out, h_out_cap, h_out_off);
}

int cpk_decode_host(cpk_ctx ctx, const void *h_packed, const uint64_t *h_in_off,
                    const uint64_t *h_swo, uint32_t n, void *h_out, int32_t *h_status) {
  if (!ctx || !h_in_off || !h_swo || !h_status) return CPK_EINVAL;
  if (n == 0) return CPK_OK;
  for (uint32_t i = 0; i < n; ++i)
    if (h_swo[i + 1] < h_swo[i] || h_in_off[i + 1] < h_in_off[i]) return CPK_EINVAL;
  if ((!h_packed && h_in_off[n] > h_in_off[0]) || (!h_out && h_swo[n] > h_swo[0])) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  if (n <= 32 && h_swo[n] - h_swo[0] >= ((uint64_t)n << 20)) {
    // A few large pieces (>= 8 MiB of words each on average): the batch
    // decoder gives a piece one wave (one 64 MiB piece: 104 ms), so decode
    // them as one stream, 256-byte blocks in parallel (cpk_decode_stream),
    // and keep that when every piece ended exactly where its packed range
    // does -- then each read() consumed exactly its bytes, as the batch
    // decode requires; otherwise (an error, or a piece ending elsewhere) the
    // batch decoder below gives each piece its own status.  It stages the
    // whole stream through slot 0 alone (pinned + device buffers of the
    // packed bytes and the words, grown once and kept by the context: the
    // same memory a batch chunk of these pieces would take in one slot).
    std::vector<uint64_t> sin(n + 1);
    std::vector<int32_t> sst(n);
    const uint8_t *sp = (const uint8_t *)h_packed + (h_packed ? h_in_off[0] : 0);
    if (cpk_decode_stream_host(ctx, sp, h_in_off[n] - h_in_off[0], h_swo, n, h_out, sin.data(), sst.data()) ==
        CPK_OK) {
      bool same = true;
      for (uint32_t i = 0; i <= n && same; ++i) same = sin[i] == h_in_off[i] - h_in_off[0];
      if (same) {
        for (uint32_t i = 0; i < n; ++i) h_status[i] = CPK_OK;
        return CPK_OK;
      }
    }
  }
  const std::vector<HostChunk> cs = host_chunks(h_swo, h_in_off, n, host_chunk_bytes());
  uint64_t mi = 0, mo = 0, mm = 0;
  for (const HostChunk &c : cs) {
    mi = c.in_len > mi ? c.in_len : mi;
    mo = c.out_cap > mo ? c.out_cap : mo;
    mm = c.i1 - c.i0 > mm ? c.i1 - c.i0 : mm;
  }
  HostPipe *p = nullptr;
  // meta: swo | in_off | status (int32, n/2 + 1 entries)
  int rc = pipe_get(ctx, mi, mo, 2 * (mm + 1) + mm / 2 + 1, &p);
  if (rc) return rc;
  const uint8_t *src = (const uint8_t *)h_packed;
  uint8_t *dst = (uint8_t *)h_out;
  const size_t K = cs.size();
  // one large chunk (a single big piece): its own transfers pipelined in
  // 16 MiB chunks (encode_host_impl likewise)
  const bool one = K == 1 && cs[0].out_cap >= 2 * kPipeChunk;
  for (size_t k = 0; k <= K + 1 && rc == CPK_OK; ++k) {
    if (k < K) {  // copy-in, H2D, decode of chunk k
      const HostChunk &c = cs[k];
      HostSlot &s = p->slot[k & 1];
      const uint32_t nk = c.i1 - c.i0;
      memset((uint8_t *)s.pin_in + c.in_len, 0, 32);  // (the decoder reads whole 16-byte lines)
      for (uint32_t j = 0; j <= nk; ++j) {
        s.pin_meta[j] = h_swo[c.i0 + j] - h_swo[c.i0];
        s.pin_meta[nk + 1 + j] = h_in_off[c.i0 + j] - h_in_off[c.i0];
      }
      int32_t *st = (int32_t *)(s.d_meta + 2 * (nk + 1));
      if (one) {
        if (h2d_pipelined(s.d_in, s.pin_in, src + c.in0, c.in_len, p->sh) ||
            hipMemcpyAsync((uint8_t *)s.d_in + c.in_len, (uint8_t *)s.pin_in + c.in_len, 32, hipMemcpyHostToDevice,
                           p->sh)) {
          rc = CPK_EDEVICE;
          break;
        }
      } else {
        par_copy(s.pin_in, src + c.in0, c.in_len);
        if (hipMemcpyAsync(s.d_in, s.pin_in, c.in_len + 32, hipMemcpyHostToDevice, p->sh)) {
          rc = CPK_EDEVICE;
          break;
        }
      }
      if (hipMemcpyAsync(s.d_meta, s.pin_meta, 2 * (nk + 1) * 8ull, hipMemcpyHostToDevice, p->sh) ||
          hipEventRecord(s.eh, p->sh) || hipStreamWaitEvent(p->sk, s.eh, 0) ||
          (k >= 2 && hipStreamWaitEvent(p->sk, s.ed, 0))) {
        rc = CPK_EDEVICE;
        break;
      }
      rc = decode_batch_impl(ctx, s.d_in, s.d_meta + nk + 1, s.d_meta, nk, s.d_out, st, p->sk, false);
      if (rc) break;
      if (hipMemcpyAsync(s.pin_meta + 2 * (nk + 1), st, nk * 4ull, hipMemcpyDeviceToHost, p->sk) ||
          hipEventRecord(s.ek, p->sk)) {
        rc = CPK_EDEVICE;
        break;
      }
    }
    if (k >= 1 && k - 1 < K) {  // chunk k-1: statuses, then its D2H
      const HostChunk &c = cs[k - 1];
      HostSlot &s = p->slot[(k - 1) & 1];
      const uint32_t nk = c.i1 - c.i0;
      if (hipEventSynchronize(s.ek)) {
        rc = CPK_EDEVICE;
        break;
      }
      memcpy(h_status + c.i0, s.pin_meta + 2 * (nk + 1), nk * 4ull);
      if (one) {
        // (its copy-out under its own D2H; the other slot's events are free)
        if (d2h_pipelined(dst + 8 * h_swo[c.i0], s.pin_out, s.d_out, c.out_cap, p->sd, p->slot[1].eh,
                          p->slot[1].ed))
          rc = CPK_EDEVICE;
        break;
      }
      if ((c.out_cap && hipMemcpyAsync(s.pin_out, s.d_out, c.out_cap, hipMemcpyDeviceToHost, p->sd)) ||
          hipEventRecord(s.ed, p->sd)) {
        rc = CPK_EDEVICE;
        break;
      }
    }
    if (k >= 2) {  // chunk k-2: copy-out
      const HostChunk &c = cs[k - 2];
      HostSlot &s = p->slot[k & 1];
      if (hipEventSynchronize(s.ed)) {
        rc = CPK_EDEVICE;
        break;
      }
      par_copy(dst + 8 * h_swo[c.i0], s.pin_out, c.out_cap);
    }
  }
  if (rc) {
    pipe_drain(p);
    return rc;
  }
  for (uint32_t i = 0; i < n; ++i)
    if (h_status[i] != CPK_OK) return h_status[i];
  return CPK_OK;
}

}  // extern "C"

// ---- message batches from host memory (SerializePacked.write / read for
// many messages, the JNI facade's encodeMessages / decodeMessages): chunks of
// whole messages through the same two pinned slots as the piece forms
namespace {

struct MsgChunk {
  uint32_t m0, m1;    // messages [m0, m1)
  uint64_t s0, s1;    // their segments (encode) / none (decode)
  uint64_t in0, in_len;  // input bytes: segment words (encode) / packed (decode)
  uint64_t out_cap;   // encode: packed bytes the chunk may produce
  uint64_t maxw;      // encode: largest segment, words
};

// encode: chunks of about `target` bytes of segment words
std::vector<MsgChunk> enc_msg_chunks(const uint64_t *swo, const uint64_t *mso, uint32_t nm, uint64_t target) {
  std::vector<MsgChunk> cs;
  uint32_t m = 0;
  while (m < nm) {
    MsgChunk c{m, m, mso[m], mso[m], 0, 0, 16, 1};
    while (c.m1 < nm) {
      const uint64_t a = mso[c.m1], b = mso[c.m1 + 1];
      const uint64_t bytes = 8 * (swo[b] - swo[a]);
      if (c.m1 > c.m0 && c.in_len + bytes > target) break;
      c.in_len += bytes;
      for (uint64_t i = a; i < b; ++i) {
        const uint64_t w = swo[i + 1] - swo[i];
        c.out_cap += cpk_packed_bound(w);
        c.maxw = w > c.maxw ? w : c.maxw;
      }
      c.out_cap += 10 * ((b - a + 2) / 2 + 1);
      ++c.m1;
    }
    c.s1 = mso[c.m1];
    c.in0 = 8 * (swo[c.s0] - swo[0]);
    cs.push_back(c);
    m = c.m1;
  }
  return cs;
}

// cpk_encode_messages_host(_gather): `fill(pin, c)` puts chunk c's segment
// words, back to back, into the pinned input slot
template <class Fill>
int encode_messages_host_impl(cpk_ctx ctx, Fill fill, const uint64_t *h_swo, uint32_t nseg,
                              const uint64_t *h_msg_seg_off, uint32_t nm, void *h_out,
                              uint64_t h_out_cap, uint64_t *h_out_off, const uint8_t *contig = nullptr) {
  if (!ctx || !h_swo || !h_msg_seg_off || !h_out_off) return CPK_EINVAL;
  if (h_msg_seg_off[0] != 0 || h_msg_seg_off[nm] != nseg) return CPK_EINVAL;
  for (uint32_t m = 0; m < nm; ++m)
    if (h_msg_seg_off[m + 1] < h_msg_seg_off[m]) return CPK_EINVAL;
  for (uint32_t i = 0; i < nseg; ++i)
    if (h_swo[i + 1] < h_swo[i]) return CPK_EINVAL;
  if (nm == 0) {
    h_out_off[0] = 0;
    return CPK_OK;
  }
  DeviceGuard g(ctx->device);
  {
    // a small batch: tables (Serialize.java:256-267, laid out after the
    // segments) and segments, in message order, through one kernel
    const uint64_t sw = h_swo[nseg] - h_swo[0];
    uint64_t tw = 0;
    for (uint32_t m = 0; m < nm; ++m) tw += ((h_msg_seg_off[m + 1] - h_msg_seg_off[m] + 2) & ~1ull) / 2;
    const uint64_t np = (uint64_t)nm + nseg;
    if (small_ok(sw + tw, np))
      return small_encode(
          ctx, np, sw + tw,
          [&](uint64_t *pin, uint64_t *desc) {
            if (sw) fill((uint8_t *)pin, MsgChunk{0, nm, 0, nseg, 0, 8 * sw, 0, 0});
            uint64_t t = sw, q = 0;
            for (uint32_t m = 0; m < nm; ++m) {
              const uint64_t a = h_msg_seg_off[m], b = h_msg_seg_off[m + 1];
              const uint32_t count = (uint32_t)(b - a);
              const uint64_t ntw = ((uint64_t)count + 2) / 2;
              for (uint64_t k = 0; k < ntw; ++k) {
                uint32_t v[2];
                for (int h = 0; h < 2; ++h) {
                  const uint64_t j = 2 * k + h;
                  v[h] = j == 0 ? count - 1 : (j <= count ? (uint32_t)(h_swo[a + j] - h_swo[a + j - 1]) : 0u);
                }
                pin[t + k] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
              }
              desc[2 * q] = t;
              desc[2 * q + 1] = ntw;
              ++q;
              t += ntw;
              for (uint64_t i = a; i < b; ++i, ++q) {
                desc[2 * q] = h_swo[i] - h_swo[0];
                desc[2 * q + 1] = h_swo[i + 1] - h_swo[i];
              }
            }
          },
          h_out, h_out_cap, h_out_off, 0);
  }
  const std::vector<MsgChunk> cs = enc_msg_chunks(h_swo, h_msg_seg_off, nm, host_chunk_bytes());
  uint64_t mi = 0, mo = 0, mm = 0;
  for (const MsgChunk &c : cs) {
    const uint64_t ns = c.s1 - c.s0, nmk = c.m1 - c.m0;
    mi = c.in_len > mi ? c.in_len : mi;
    mo = c.out_cap > mo ? c.out_cap : mo;
    // meta: swo [ns + 1] | msg_seg_off [nm + 1] | out_off [nm + ns + 1]
    const uint64_t need = (ns + 1) + (nmk + 1) + (nmk + ns + 1);
    mm = need > mm ? need : mm;
  }
  HostPipe *p = nullptr;
  int rc = pipe_get(ctx, mi, mo, mm, &p);
  if (rc) return rc;
  uint8_t *dst = (uint8_t *)h_out;
  uint64_t base = 0;
  const size_t K = cs.size();
  // one large chunk (e.g. one big message): its own transfers pipelined in
  // 16 MiB sub-chunks (encode_host_impl likewise)
  const bool one = K == 1 && cs[0].in_len >= 2 * kPipeChunk;
  for (size_t k = 0; k <= K + 1 && rc == CPK_OK; ++k) {
    if (k < K) {  // copy-in, H2D, kernels of chunk k
      const MsgChunk &c = cs[k];
      HostSlot &s = p->slot[k & 1];
      const uint32_t ns = (uint32_t)(c.s1 - c.s0), nmk = c.m1 - c.m0;
      uint64_t *m = s.pin_meta;
      for (uint32_t j = 0; j <= ns; ++j) m[j] = h_swo[c.s0 + j] - h_swo[c.s0];
      for (uint32_t j = 0; j <= nmk; ++j) m[ns + 1 + j] = h_msg_seg_off[c.m0 + j] - c.s0;
      uint64_t *dm = s.d_meta, *doff = dm + (ns + 1) + (nmk + 1);
      if (one && contig) {
        if (h2d_pipelined(s.d_in, s.pin_in, contig + c.in0, c.in_len, p->sh)) {
          rc = CPK_EDEVICE;
          break;
        }
      } else {
        fill((uint8_t *)s.pin_in, c);
        if (c.in_len && hipMemcpyAsync(s.d_in, s.pin_in, c.in_len, hipMemcpyHostToDevice, p->sh)) {
          rc = CPK_EDEVICE;
          break;
        }
      }
      if (hipMemcpyAsync(dm, m, ((ns + 1) + (nmk + 1)) * 8ull, hipMemcpyHostToDevice, p->sh) ||
          hipEventRecord(s.eh, p->sh) || hipStreamWaitEvent(p->sk, s.eh, 0) ||
          (k >= 2 && hipStreamWaitEvent(p->sk, s.ed, 0))) {
        rc = CPK_EDEVICE;
        break;
      }
      rc = cpk_encode_messages(ctx, s.d_in, dm, ns, dm + ns + 1, nmk, c.maxw, s.d_out, doff, p->sk);
      if (rc) break;
      if (hipMemcpyAsync(m + (ns + 1) + (nmk + 1), doff, ((uint64_t)nmk + ns + 1) * 8, hipMemcpyDeviceToHost,
                         p->sk) ||
          hipEventRecord(s.ek, p->sk)) {
        rc = CPK_EDEVICE;
        break;
      }
    }
    if (k >= 1 && k - 1 < K) {  // chunk k-1: offsets, then its D2H
      const MsgChunk &c = cs[k - 1];
      HostSlot &s = p->slot[(k - 1) & 1];
      const uint32_t ns = (uint32_t)(c.s1 - c.s0), nmk = c.m1 - c.m0;
      if (hipEventSynchronize(s.ek)) {
        rc = CPK_EDEVICE;
        break;
      }
      const uint64_t *off = s.pin_meta + (ns + 1) + (nmk + 1);
      const uint64_t np = (uint64_t)nmk + ns, P = off[np];
      if (P > c.out_cap) {
        rc = CPK_EDEVICE;
        break;
      }
      if (base + P > h_out_cap) {
        rc = CPK_ENOMEM;
        break;
      }
      // pieces in message order: chunk k-1's start at piece c.m0 + c.s0
      for (uint64_t j = 0; j <= np; ++j) h_out_off[c.m0 + c.s0 + j] = base + off[j];
      if (one && P >= 2 * kPipeChunk) {
        // (the one chunk's copy-out under its own D2H; the other slot's events are free)
        if (d2h_pipelined(dst + base, s.pin_out, s.d_out, P, p->sd, p->slot[1].eh, p->slot[1].ed)) {
          rc = CPK_EDEVICE;
          break;
        }
        base += P;
        break;
      }
      if ((P && hipMemcpyAsync(s.pin_out, s.d_out, P, hipMemcpyDeviceToHost, p->sd)) ||
          hipEventRecord(s.ed, p->sd)) {
        rc = CPK_EDEVICE;
        break;
      }
      base += P;
    }
    if (k >= 2) {  // chunk k-2: copy-out
      const MsgChunk &c = cs[k - 2];
      HostSlot &s = p->slot[k & 1];
      if (hipEventSynchronize(s.ed)) {
        rc = CPK_EDEVICE;
        break;
      }
      const uint64_t np = (uint64_t)(c.m1 - c.m0) + (c.s1 - c.s0);
      const uint64_t o0 = h_out_off[c.m0 + c.s0], o1 = h_out_off[c.m0 + c.s0 + np];
      par_copy(dst + o0, s.pin_out, o1 - o0);
    }
  }
  if (rc) {
    pipe_drain(p);
    return rc;
  }
  return cpk_ctx_take_error(ctx, p->sk);
}

}  // namespace

extern "C" {

int cpk_encode_messages_host(cpk_ctx ctx, const void *h_in, const uint64_t *h_swo, uint32_t nseg,
                             const uint64_t *h_msg_seg_off, uint32_t nm, void *h_out,
                             uint64_t h_out_cap, uint64_t *h_out_off) {
  if (!h_swo || (nseg && h_swo[nseg] > h_swo[0] && !h_in) || (nm && !h_out)) return CPK_EINVAL;
  const uint8_t *src = (const uint8_t *)h_in + 8 * h_swo[0];
  return encode_messages_host_impl(
      ctx, [&](uint8_t *pin, const MsgChunk &c) { par_copy(pin, src + c.in0, c.in_len); }, h_swo, nseg,
      h_msg_seg_off, nm, h_out, h_out_cap, h_out_off, src);
}

int cpk_encode_messages_host_gather(cpk_ctx ctx, const void *const *h_segs, const uint64_t *h_swo,
                                    uint32_t nseg, const uint64_t *h_msg_seg_off, uint32_t nm,
                                    void *h_out, uint64_t h_out_cap, uint64_t *h_out_off) {
  if (!h_swo || (nseg && !h_segs) || (nm && !h_out)) return CPK_EINVAL;
  for (uint32_t i = 0; i < nseg; ++i)
    if (h_swo[i + 1] > h_swo[i] && !h_segs[i]) return CPK_EINVAL;
  return encode_messages_host_impl(
      ctx,
      [&](uint8_t *pin, const MsgChunk &c) {
        gather_copy(pin, h_segs, h_swo, (uint32_t)c.s0, (uint32_t)c.s1);
      },
      h_swo, nseg, h_msg_seg_off, nm, h_out, h_out_cap, h_out_off);
}

// Decode: chunks of whole messages by packed bytes.  A chunk's table pass
// gives its words and segments; the chunk is then decoded straight into the
// caller's arrays at the running totals.  When the caller's capacities are
// too small (or zero: the sizing call) the remaining chunks only run their
// table passes, and the totals are returned with CPK_ENOMEM.
int cpk_decode_messages_host(cpk_ctx ctx, const void *h_packed, const uint64_t *h_msg_off, uint32_t nm,
                             uint64_t traversal_limit_words, void *h_out, uint64_t out_cap_words,
                             uint64_t *h_seg_word_off, uint32_t seg_cap, uint64_t *h_msg_seg_off,
                             int32_t *h_msg_status, uint64_t *h_totals) {
  if (!ctx || !h_msg_off || !h_msg_seg_off || !h_msg_status || !h_totals) return CPK_EINVAL;
  h_totals[0] = h_totals[1] = 0;
  if (nm == 0) {
    h_msg_seg_off[0] = 0;
    return CPK_OK;
  }
  for (uint32_t m = 0; m < nm; ++m)
    if (h_msg_off[m + 1] < h_msg_off[m]) return CPK_EINVAL;
  if (!h_packed && h_msg_off[nm] > h_msg_off[0]) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  // chunks of whole messages, about `target` packed bytes each
  const uint64_t target = host_chunk_bytes() / 2;
  std::vector<MsgChunk> cs;
  for (uint32_t m = 0; m < nm;) {
    MsgChunk c{m, m, 0, 0, h_msg_off[m], 0, 0, 0};
    while (c.m1 < nm && (c.m1 == c.m0 || h_msg_off[c.m1 + 1] - c.in0 <= target)) ++c.m1;
    c.in_len = h_msg_off[c.m1] - c.in0;
    cs.push_back(c);
    m = c.m1;
  }
  uint64_t mi = 0, mmsg = 0;
  for (const MsgChunk &c : cs) {
    mi = c.in_len > mi ? c.in_len : mi;
    mmsg = (uint64_t)(c.m1 - c.m0) > mmsg ? c.m1 - c.m0 : mmsg;
  }
  // meta: msg_off [n + 1] | msg_seg_off [n + 1] | msg_status [n] (as u32 pairs)
  //       | seg_word_off [S + 1] | seg_in_off [S + 1] | seg_status [S]
  auto meta_need = [](uint64_t nmk, uint64_t S) { return 2 * (nmk + 1) + (nmk + 1) / 2 + 2 * (S + 1) + S / 2 + 1; };
  HostPipe *p = nullptr;
  int rc = pipe_get(ctx, mi, 64, meta_need(mmsg, 0), &p);
  if (rc) return rc;
  const uint8_t *src = (const uint8_t *)h_packed;
  uint64_t W = 0, S = 0;  // running totals
  bool sizing = false;     // capacities exceeded: table passes only
  int first_bad = CPK_OK;
  for (size_t k = 0; k < cs.size() && rc == CPK_OK; ++k) {
    const MsgChunk &c = cs[k];
    const uint32_t nmk = c.m1 - c.m0;
    for (int attempt = 0; attempt < 2; ++attempt) {
      HostSlot &s = p->slot[k & 1];
      par_copy(s.pin_in, src + c.in0, c.in_len);
      memset((uint8_t *)s.pin_in + c.in_len, 0, 64);  // (the decoder reads whole 16-byte lines)
      uint64_t *m = s.pin_meta, *dm = s.d_meta;
      for (uint32_t j = 0; j <= nmk; ++j) m[j] = h_msg_off[c.m0 + j] - c.in0;
      uint64_t *d_ms = dm + (nmk + 1);
      int32_t *d_mst = (int32_t *)(d_ms + (nmk + 1));
      uint64_t *d_sw = dm + 2 * (nmk + 1) + (nmk + 1) / 2;
      uint64_t tot[2] = {0, 0};
      if (hipMemcpyAsync(s.d_in, s.pin_in, c.in_len + 64, hipMemcpyHostToDevice, p->sk) ||
          hipMemcpyAsync(dm, m, (nmk + 1) * 8ull, hipMemcpyHostToDevice, p->sk)) {
        rc = CPK_EDEVICE;
        break;
      }
      // the table pass (synchronises the stream for the chunk's totals)
      rc = cpk_decode_messages(ctx, s.d_in, dm, nmk, traversal_limit_words, nullptr, 0, nullptr, nullptr, nullptr,
                               0, d_ms, d_mst, tot, p->sk);
      if (rc == CPK_ENOMEM) rc = CPK_OK;
      if (rc) break;
      if (!sizing && (W + tot[0] > out_cap_words || S + tot[1] > seg_cap || (tot[1] && (!h_out || !h_seg_word_off))))
        sizing = true;
      if (sizing) {
        W += tot[0];
        S += tot[1];
        break;
      }
      // room in the slot for the chunk's words and segments?
      if (tot[0] * 8 + 64 > s.cap_out || meta_need(nmk, tot[1]) > s.cap_meta) {
        if (attempt) {
          rc = CPK_EDEVICE;
          break;
        }
        pipe_drain(p);
        rc = pipe_get(ctx, mi, tot[0] * 8, meta_need(mmsg, tot[1]), &p);
        if (rc) break;  // (no pinned slots left: report it, stage nothing)
        continue;       // (buffers replaced: stage the chunk again)
      }
      uint64_t *d_si = d_sw + (tot[1] + 1);
      int32_t *d_ss = (int32_t *)(d_si + (tot[1] + 1));
      rc = cpk_decode_messages(ctx, s.d_in, dm, nmk, traversal_limit_words, s.d_out, tot[0], d_sw, d_si, d_ss,
                               (uint32_t)tot[1], d_ms, d_mst, tot, p->sk);
      if (rc) break;
      uint64_t *hm = m + (nmk + 1);  // msg_seg_off | msg_status | seg_word_off
      if (hipMemcpyAsync(hm, d_ms, ((nmk + 1) + (nmk + 1) / 2 + (tot[1] + 1)) * 8ull, hipMemcpyDeviceToHost,
                         p->sk) ||
          (tot[0] && hipMemcpyAsync(s.pin_out, s.d_out, tot[0] * 8, hipMemcpyDeviceToHost, p->sk)) ||
          hipStreamSynchronize(p->sk)) {
        rc = CPK_EDEVICE;
        break;
      }
      const uint64_t *ms = hm;
      const int32_t *mst = (const int32_t *)(hm + (nmk + 1));
      const uint64_t *sw = hm + (nmk + 1) + (nmk + 1) / 2;
      for (uint32_t j = 0; j < nmk; ++j) {
        h_msg_seg_off[c.m0 + j] = S + ms[j];
        h_msg_status[c.m0 + j] = mst[j];
        if (mst[j] != CPK_OK && first_bad == CPK_OK) first_bad = mst[j];
      }
      // (a chunk of broken messages has no segments: the sizing call, with no
      //  segment array, still gets its statuses)
      if (h_seg_word_off)
        for (uint64_t j = 0; j <= tot[1]; ++j) h_seg_word_off[S + j] = W + sw[j];
      if (tot[0]) par_copy((uint8_t *)h_out + 8 * W, s.pin_out, tot[0] * 8);
      W += tot[0];
      S += tot[1];
      break;
    }
  }
  if (rc) {
    pipe_drain(p);
    return rc;
  }
  h_msg_seg_off[nm] = S;
  h_totals[0] = W;
  h_totals[1] = S;
  if (sizing) return CPK_ENOMEM;
  return first_bad;
}

}  // extern "C"
