// Fused encoder: the two passes of encode_v4.hip in one launch, each wave a
// few pieces ahead of its own emit.  Included from packed_codec.hip
// (namespace cpk, after encode_sp.hip: the look-back words are sp_word's).
//
// A wave takes a piece from one ordered counter (pieces in stream order),
// sizes it (e4_size_piece: the step rows into bvbuf, the packed size) and
// publishes the size at once for the decoupled look-back over pieces.  It
// keeps up to `depth` sized pieces pending; the oldest is emitted
// (e4_emit_piece) as soon as the look-back finds its offset without waiting,
// or, when the queue is full or the counter is spent, after waiting for it.
// Sizing never waits on anything, so every piece a look-back waits for is
// sized by a running wave: no residency assumption.  The emit re-reads the
// piece's words a few pieces after the size sweep read them -- from L2 or the
// Infinity Cache when the pieces in flight fit there -- instead of one whole
// batch later ("Fused encoder"; PackedOutputStream.java:
// 35-205 per piece, Serialize.java:256-288 for the offsets).

#ifndef CPK_E4F_WPE
#define CPK_E4F_WPE 6  // waves per SIMD the registers are sized for (8 spills)
#endif
constexpr int kE4fMaxDepth = 64;  // pending pieces per wave: one lane each

__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}

// The look-back of sp_lookback (encode_sp.hip) over pieces, which returns
// false instead of waiting when `block` is false and a predecessor has not
// published its size yet.  On success: excl = the exclusive prefix, the
// inclusive one published.
__device__ bool e4f_lookback(uint64_t *status, uint32_t p, uint64_t agg, uint32_t ep, uint32_t *err, int lane,
                             bool block, uint64_t &excl) {
  excl = 0;
  if (p == 0) return true;  // (piece 0 published its size as inclusive)
  int64_t top = (int64_t)p - 1;
  uint32_t spins = 0;
  for (;;) {
    uint64_t v[4];
    int fi = 4;  // first inclusive among this lane's four (nearest first)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t idx = top - 4 * lane - i;
      v[i] = idx >= 0 ? ld_status(&status[idx]) : sp_word(ep, 2u, 0);
    }
#pragma unroll
    for (int i = 3; i >= 0; --i)
      if (sp_flag(v[i], ep) == 2) fi = i;
    const uint64_t has = __ballot(fi < 4);
    const int fln = has ? __builtin_ctzll(has) : 64;
    const int firstPos = fln < 64 ? 4 * fln + __builtin_amdgcn_readlane(fi, fln) : 256;
    bool z = false;
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (4 * lane + i <= firstPos) {
        z = z || sp_flag(v[i], ep) == 0;
        sum += v[i] & kSpValMask;
      }
    }
    if (__ballot(z)) {
      if (!block) return false;
      if (++spins > (1u << 22)) {  // cannot happen: every predecessor is sized by a running wave
        if (lane == 0) atomicOr(err, kErrWait);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    excl += sum;
    if (firstPos < 256) break;
    top -= 256;
  }
  excl = rfl64(excl);
  if (lane == 0) st_status(&status[p], sp_word(ep, 2u, excl + agg));
  return true;
}

// out_off[0..n] and the packed bytes of pieces [swo[p], swo[p+1]) in stream
// order; ticket: a zeroed counter; status: look-back words of epoch ep.
__global__ __launch_bounds__(kE4Threads, CPK_E4F_WPE) void e4_fused_kernel(
    const uint64_t *__restrict__ in, const uint64_t *__restrict__ swo, uint32_t n, uint8_t *__restrict__ out,
    uint64_t *__restrict__ out_off, uint64_t *status, uint32_t ep, uint32_t *ticket, uint64_t *__restrict__ bvbuf,
    uint64_t stride, const uint32_t *skip, uint64_t hint, uint64_t ocap, uint32_t *err, uint32_t depth) {
  if (skip && __builtin_amdgcn_readfirstlane(*skip)) return;  // (the single pass took the batch)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint64_t *lut = reinterpret_cast<const uint64_t *>(smem + kE4oLut);
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  uint32_t *ring = reinterpret_cast<uint32_t *>(smem + kE4oRing + w * kE4RingBytes);
  fill_luts(reinterpret_cast<uint64_t *>(smem + kE4oLut), false);
  for (uint32_t i = lane; i < kE4RingLines; i += 64)
    reinterpret_cast<uint4 *>(ring)[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  // the wave's pending pieces, a queue over the lanes: lane j holds entry j
  // (ticket, packed size); h = oldest, c = count
  uint32_t qt = 0;
  uint64_t qs = 0;
  uint32_t h = 0, c = 0;
  bool more = true;
  for (;;) {
    while (c) {
      const uint32_t p = (uint32_t)__builtin_amdgcn_readlane((int)qt, (int)h);
      const uint64_t sz = rl64(qs, (int)h);
      uint64_t excl;
      if (!e4f_lookback(status, p, sz, ep, err, lane, !more || c == depth, excl)) break;
      if (lane == 0) {
        out_off[p] = excl;
        if (p + 1 == n) out_off[n] = excl + sz;
      }
      // (a piece whose bytes would pass the caller's capacity: not written,
      // reported; ArrayOutputStream.java:40-42)
      if (excl + sz > ocap) {
        if (lane == 0) atomicOr(err, kErrCap);
      } else if (sz) {
        e4_emit_piece<true>(in, swo, p, excl, out, bvbuf, stride, lut, ring, lane);
      }
      h = h + 1 == depth ? 0u : h + 1;
      --c;
    }
    if (!more) {
      if (!c) break;
      continue;
    }
    const uint32_t t = take_ordered(ticket);
    if (t >= n) {
      more = false;
      continue;
    }
    const uint64_t sz = rl64(e4_size_piece<false>(in, swo, t, hint, err, bvbuf, stride, lane), 63);
    // the size, published before the piece waits for anything
    if (lane == 0) st_status(&status[t], sp_word(ep, t == 0 ? 2u : 1u, sz));
    uint32_t j = h + c;
    if (j >= depth) j -= depth;
    qt = (uint32_t)lane == j ? t : qt;
    qs = (uint32_t)lane == j ? sz : qs;
    ++c;
  }
}
