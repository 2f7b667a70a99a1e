// encode_sp3.hip -- one workgroup encoding a small batch in order: the
// one-launch kernel behind the host path for small messages
// (cpk_encode_messages_host / cpk_encode_host, host_pipe.hip).  Included from
// packed_codec.hip after encode_sp.hip (namespace cpk); reuses the single
// pass's per-unit algebra (A1 tags / ballots, A2 roles, B strings),
// PackedOutputStream.java:35-205 restated per 8192-word chunk, with the
// chunk's packed bytes staged whole in LDS and the output offset running.
//
// (Round 4 also ran a pipelined batch encoder on these pieces -- each
// workgroup with the next unit's words in flight and a whole-unit LDS stage,
// its look-back one iteration late: 2 workgroups per CU, config 2 encode
// +7 % against the per-unit kernel with 11 KiB rings, docs/tuning_log.md.)

constexpr uint32_t kSp3Stage = 9 * 64 * kSpCS + 32;  // a unit's packed bytes (<= 9 per word) + put spill
constexpr uint32_t kSp3oLut = 0;
constexpr uint32_t kSp3oMsk = 2048;
constexpr uint32_t kSp3oScr = kSp3oMsk + kSpCS * 24;
constexpr uint32_t kSp3oStage = kSp3oScr + 32 * 8;
constexpr uint32_t kSp3Lds = kSp3oStage + kSp3Stage;  // 79,136 B
static_assert(kSp3oStage % 16 == 0, "LDS alignment");

// One unit as a wave sees it: the piece, the chunk and this wave's steps.
struct Sp3Unit {
  const uint64_t *pw;  // the piece's first word
  uint32_t W;          // piece words (0: an unsupported piece, sized 0)
  uint32_t p, c;       // piece, chunk
  bool lastc;          // the piece's last chunk
  bool bad;            // unsupported (reported once)
  bool over;           // more words than the caller's hint (reported once)
  int cs;              // steps in the chunk
  int sa, cnt;         // this wave's steps [sa, sa + cnt) of the chunk
  uint32_t wfirst;     // the wave's first word (piece-relative)
  uint32_t wrem;       // piece words from wfirst on (0: no steps)
};

// The wave's words of a chunk, every load issued (none waited for): step j
// of lane l reads word min(64 j + l, last) -- a partial step or wave reads
// its last word again, a wave without steps a valid dummy word.
__device__ __forceinline__ void sp3_load(uint64_t (&V)[kSpWS], const Sp3Unit &u, const uint64_t *dummy, int lane) {
  const uint64_t *src = u.cnt ? u.pw + u.wfirst : dummy;
  const uint32_t last = u.cnt ? u.wrem - 1 : 0u;
#pragma unroll
  for (int j = 0; j < kSpWS; ++j) V[j] = ld_stream(src + min(64u * j + (uint32_t)lane, last));
}

// The four steps past the chunk (the zero run / D/L stretch continuing from
// its end, for the last wave's head counts): issued with the unit's own
// words, used only by the chunk's last wave when the piece continues.
__device__ __forceinline__ bool sp3_la_need(const Sp3Unit &u) {
  return u.cnt && u.sa + u.cnt == u.cs && u.wfirst + 64u * u.cnt < u.W;
}
__device__ __forceinline__ void sp3_la_load(uint64_t (&LA)[4], const Sp3Unit &u, const uint64_t *dummy, int lane) {
  const bool need = sp3_la_need(u);
  const uint32_t wend = u.wfirst + 64u * u.cnt;
  const uint64_t *src = need ? u.pw + wend : dummy;
  const uint32_t last = need ? u.W - wend - 1 : 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) LA[j] = ld_stream(src + min(64u * j + (uint32_t)lane, last));
}
__device__ __forceinline__ void sp3_lookahead(const uint64_t (&LA)[4], uint32_t avail, int lane, uint32_t &laz,
                                              uint32_t &ladl) {
  uint32_t rz = 0, rd = 0;
  bool oz = true, od = true;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool valid = (uint32_t)lane < (avail > 64u * j ? avail - 64u * j : 0u);
    const uint32_t m = valid ? e4_tag(LA[j]) : 0u;
    const uint64_t Z = __ballot(valid && m == 0), DL = __ballot(__builtin_popcount(m) >= 7);
    if (oz) {
      if (Z == ~0ull) rz += 64;
      else { rz += (uint32_t)__builtin_ctzll(~Z); oz = false; }
    }
    if (od) {
      if (DL == ~0ull) rd += 64;
      else { rd += (uint32_t)__builtin_ctzll(~DL); od = false; }
    }
  }
  laz = rz;
  ladl = rd;
}

// A1 on words already in registers: per word the nonzero-byte tag
// (PackedOutputStream.java:64-117), per step the Z / DL / D ballots stashed
// lane-per-step; returns this lane's nonzero bytes
template <bool kFull>
__device__ __forceinline__ uint32_t sp3_a1(SpRegs &R, const uint64_t (&V)[kSpWS], uint32_t wrem, int cnt,
                                           int lane) {
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < kSpWS; ++j) {
    if (kFull || j < cnt) {
      const bool valid = kFull || (uint32_t)lane < wrem - 64u * j;
      const uint32_t m = valid ? e4_tag(V[j]) : 0u;
      if (j & 3) R.mp[j >> 2] |= m << (8 * (j & 3));
      else R.mp[j >> 2] = m;
      const uint32_t pc = (uint32_t)__builtin_popcount(m);
      acc += pc;
      const uint64_t Z = __ballot(valid && m == 0), DL = __ballot(pc >= 7), D = __ballot(m == 0xffu);
      R.zl = sp_wl(R.zl, (uint32_t)Z, j);
      R.zh = sp_wl(R.zh, (uint32_t)(Z >> 32), j);
      R.dll = sp_wl(R.dll, (uint32_t)DL, j);
      R.dlh = sp_wl(R.dlh, (uint32_t)(DL >> 32), j);
      R.dl_ = sp_wl(R.dl_, (uint32_t)D, j);
      R.dh_ = sp_wl(R.dh_, (uint32_t)(D >> 32), j);
    }
    CPK_SP_STEP_FENCE();
  }
  return acc;
}

// A of one unit (all waves; two barriers, three when the chunk continues a
// piece): masks to LDS, the state entering the chunk (fresh, or what the
// piece's previous chunk published: pst is a first probe of it, issued
// with the loads), roles, the chunk's packed bytes (returned; wbefore /
// wmine: bytes of the waves before this one / of this one).  The state the
// chunk leaves goes to `next` when the piece continues.
__device__ __forceinline__ uint64_t sp3_chunk(SpRegs &R, const uint64_t (&V)[kSpWS], const uint64_t (&LA)[4],
                                              const Sp3Unit &u, uint64_t *msk, uint64_t *scr, uint64_t pst,
                                              uint64_t *prev, uint64_t *next, uint32_t ep, uint32_t *err, int w,
                                              int lane, uint32_t &Xlast, uint64_t &wbefore) {
  const int cs = u.cs, sa = u.sa, cnt = u.cnt;
  const uint32_t wrem = u.wrem, W = u.W;
  uint32_t acc = 0;
  if (cnt) {
    if (cnt == kSpWS && wrem >= 64u * kSpWS) acc = sp3_a1<true>(R, V, wrem, cnt, lane);
    else acc = sp3_a1<false>(R, V, wrem, cnt, lane);
    sp_put_masks(R, msk, sa, cnt, lane);
  }
  __syncthreads();  // the chunk's masks in LDS
  SpSt cst = {0u, 0u, 0u};
  // the state leaving the chunk depends on the entering one only when a zero
  // run or D/L stretch covers the whole chunk: otherwise it is published now
  bool early = false;
  if (next && cnt && sa + cnt == cs) {
    bool dep = false;
    const SpSt ex = sp_state_at(msk, cs, cst, dep);
    if (!dep) {
      early = true;
      if (lane == 0) st_status(next, sp_word(ep, 2u, sp_pack_state(ex)));
    }
  }
  if (prev) {
    if (threadIdx.x == 0) {
      uint32_t spins = 0;
      uint64_t v = pst;
      while (sp_flag(v, ep) != 2u) {
        if (++spins > (1u << 24)) {  // cannot happen: the predecessor chunk is held by a running workgroup
          atomicOr(err, 4u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = ld_status(prev);
      }
      scr[12] = v & kSpValMask;
    }
    __syncthreads();
    cst = sp_unpack_state(sp_ld(&scr[12]));
  }
  SpSt st = cst;
  uint32_t bytes = 0;
  const bool last = cnt && sa + cnt == cs;  // this wave holds the chunk's last step
  Xlast = 0;
  if (cnt) {
    bool dep_ = false;
    st = sp_state_at(msk, sa, cst, dep_);
    uint32_t nz0 = 0, ndl0 = 0;
    {
      uint32_t laz = 0, ladl = 0;
      const uint32_t wend = u.wfirst + 64u * cnt;
      if (last && wend < W) sp3_lookahead(LA, W - wend, lane, laz, ladl);
      if (sa + cnt < cs) {
        nz0 = (uint32_t)sp_ld(&msk[3 * (sa + cnt)]) & 1u;
        ndl0 = (uint32_t)sp_ld(&msk[3 * (sa + cnt) + 1]) & 1u;
      } else {
        nz0 = laz ? 1u : 0u;
        ndl0 = ladl ? 1u : 0u;
      }
      const uint64_t Zl = sp_rl(R.zl, R.zh, cnt - 1), DLl = sp_rl(R.dll, R.dlh, cnt - 1);
      const int cls = (Zl >> 63) ? 0 : ((DLl >> 63) ? 1 : -1);
      if (cls >= 0) {
        const uint32_t r = sp_cont(msk, sa + cnt, cs, cls, cls ? ladl : laz);
        Xlast = r ? r - 1 : 0;
      }
    }
    uint32_t rb = 0;
    if (!sp_a2p(R, cnt, wrem, st, nz0, ndl0, lane, rb)) rb = sp_a2_seq(R, cnt, wrem, st, nz0, ndl0);
    sp_xs(R, cnt, Xlast, lane);
    bytes = rb + (uint32_t)__builtin_amdgcn_readlane(wave_incl_add((int)acc), 63);
  }
  if (last && next && !early) {
    bool dep_ = false;
    st = sp_state_at(msk, cs, cst, dep_);
    if (lane == 0) st_status(next, sp_word(ep, 2u, sp_pack_state(st)));
  }
  if (lane == 0) scr[16 + w] = bytes;
  __syncthreads();  // wave bytes in LDS
  uint64_t tot = 0;
  wbefore = 0;
#pragma unroll
  for (int q = 0; q < kSpWaves; ++q) {
    const uint64_t b = sp_ld(&scr[16 + q]);
    if (q < w) wbefore += b;
    tot += b;
  }
  return tot;
}

// B: the wave's strings OR-ed into the unit's LDS stage at unit-relative
// bytes from `base` on (the whole unit fits: no offset needed).  Each
// word's string: tag + v_perm-compacted nonzero bytes + the count after a
// 0x00 / 0xFF head, or the 8 bytes of a literal-run member
// (PackedOutputStream.java:64-193).
__device__ __forceinline__ void sp3_b(SpRegs &R, const uint64_t (&V)[kSpWS], int cnt, const uint64_t *lut,
                                      uint32_t *stage, uint32_t base, int lane) {
  uint32_t rel = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
  const uint32_t l64 = 64u - (uint32_t)lane;
  auto strings = [&](const int j, uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &nb)
      __attribute__((always_inline)) {
    const uint64_t Mem = sp_rl(R.oml, R.omh, j);
    const uint64_t HC = sp_rl(R.ohl, R.ohh, j);
    const uint32_t m = (R.mp[j >> 2] >> (8 * (j & 3))) & 0xffu;
    const uint32_t lo = (uint32_t)V[j], hi = (uint32_t)(V[j] >> 32);
    const uint64_t sel = lut[m];
    const uint32_t c0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
    const uint32_t c1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
    const bool zw = m == 0;
    uint32_t cz = 0, cd = 0;
    if (HC) {
      // a head's count: words to its run's end, at most 255 (:119-131, :143-164)
      const uint32_t X = (uint32_t)__builtin_amdgcn_readlane((int)R.ox, j);
      const uint64_t E = sp_rl(R.oel, R.oeh, j);
      const uint64_t e = E >> lane;
      const uint32_t z_lo = sp_ffbl((uint32_t)e);
      const uint32_t z_hi = sp_ffbl((uint32_t)(e >> 32)) | 32u;
      const uint32_t tt = min(min(z_lo, z_hi), min(l64 + X, 255u));
      const uint32_t cn = sp_sel(0u, tt, HC);
      cz = zw ? cn : 0u;
      cd = cn - cz;
    }
    const uint32_t c0p = c0 | cz;
    s0 = m | (c0p << 8);
    s1 = __builtin_amdgcn_alignbyte(c1, c0p, 3);
    s2 = __builtin_amdgcn_alignbyte(cd, c1, 3);
    s0 = sp_sel(s0, lo, Mem);
    s1 = sp_sel(s1, hi, Mem);
    s2 = sp_sel(s2, 0u, Mem);
    nb = (uint32_t)__builtin_popcount(m) + sp_sel(1u, 2u, HC);
    nb = sp_sel(nb, 8u, Mem);
    nb = sp_sel(zw ? 0u : nb, nb, HC);
  };
  auto put = [&](uint32_t p, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t nb) __attribute__((always_inline)) {
    const uint32_t b = p & 3;
    const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, b, 0u);
    const uint32_t d0 = __builtin_amdgcn_perm(s0, 0u, sel), d1 = __builtin_amdgcn_perm(s1, s0, sel);
    const uint32_t d2 = __builtin_amdgcn_perm(s2, s1, sel), d3 = __builtin_amdgcn_perm(0u, s2, sel);
    uint32_t *rp = stage + (p >> 2);
    if (nb) {  // (zero-length strings would all hit one address)
      atomicOr(rp, d0);
      atomicOr(rp + 1, d1);
      atomicOr(rp + 2, d2);
      atomicOr(rp + 3, d3);
    }
  };
#pragma unroll
  for (int j = 0; j < kSpWS; j += 2) {
    if (j < cnt) {
      uint32_t a0, a1, a2, na, b0 = 0, b1 = 0, b2 = 0, nb2 = 0;
      strings(j, a0, a1, a2, na);
      if (j + 1 < cnt) strings(j + 1, b0, b1, b2, nb2);
      const uint32_t pk = na | (nb2 << 16);
      const uint32_t incl = (uint32_t)wave_incl_add((int)pk);
      const uint32_t stot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      if (stot) {
        const uint32_t ta = stot & 0xffffu;
        put(rel + (incl & 0xffffu) - na, a0, a1, a2, na);
        put(rel + ta + (incl >> 16) - nb2, b0, b1, b2, nb2);
        rel += ta + (stot >> 16);
      }
    }
    CPK_SP_STEP_FENCE();
  }
}

// global line (g0 >> 4) + t from stage lines t - 1 and t (k = g0 & 15)
__device__ __forceinline__ uint4 sp3_gline(const uint4 *sl, uint32_t t, uint32_t k) {
  const uint4 b = sl[t];
  if (k == 0) return b;
  const uint4 a = t ? sl[t - 1] : make_uint4(0u, 0u, 0u, 0u);
  const uint32_t q = 16u - k, s = q & 3;
  uint4 r;
  switch (q >> 2) {
    case 0:
      r = make_uint4(__builtin_amdgcn_alignbyte(a.y, a.x, s), __builtin_amdgcn_alignbyte(a.z, a.y, s),
                     __builtin_amdgcn_alignbyte(a.w, a.z, s), __builtin_amdgcn_alignbyte(b.x, a.w, s));
      break;
    case 1:
      r = make_uint4(__builtin_amdgcn_alignbyte(a.z, a.y, s), __builtin_amdgcn_alignbyte(a.w, a.z, s),
                     __builtin_amdgcn_alignbyte(b.x, a.w, s), __builtin_amdgcn_alignbyte(b.y, b.x, s));
      break;
    case 2:
      r = make_uint4(__builtin_amdgcn_alignbyte(a.w, a.z, s), __builtin_amdgcn_alignbyte(b.x, a.w, s),
                     __builtin_amdgcn_alignbyte(b.y, b.x, s), __builtin_amdgcn_alignbyte(b.z, b.y, s));
      break;
    default:
      r = make_uint4(__builtin_amdgcn_alignbyte(b.x, a.w, s), __builtin_amdgcn_alignbyte(b.y, b.x, s),
                     __builtin_amdgcn_alignbyte(b.z, b.y, s), __builtin_amdgcn_alignbyte(b.w, b.z, s));
      break;
  }
  return r;
}

// A staged unit's ct packed bytes to out[g0, g0 + ct) (all threads): whole
// 16-byte lines as nontemporal stores, the first and last line's own bytes
// (shared with the neighbours) as byte stores; then the stage cleared for
// the next unit's ORs.  Stores past ocap are dropped (a corrupted offset
// cannot fault the device).  Two barriers.
__device__ __forceinline__ void sp3_flush(uint8_t *out, uint32_t *stage, uint64_t g0, uint64_t ct, uint64_t ocap) {
  const uint4 *sl = reinterpret_cast<const uint4 *>(stage);
  const uint32_t k = (uint32_t)(g0 & 15);
  const uint64_t L0 = g0 >> 4;
  const uint32_t nl = (uint32_t)((k + ct + 15) >> 4);
  const uint32_t endb = (uint32_t)((k + ct) & 15);
  for (uint32_t t = threadIdx.x; t < nl; t += kSpThreads) {
    const uint4 v = sp3_gline(sl, t, k);
    const uint32_t j0 = t == 0 ? k : 0u, j1 = (t + 1 == nl && endb) ? endb : 16u;
    const uint64_t a = (L0 + t) * 16;
    if (j0 == 0 && j1 == 16) {
      if (a + 16 <= ocap) st_stream(v, out + a);
    } else {
      for (uint32_t j = j0; j < j1; ++j) {
        const uint32_t d = (j & 8) ? ((j & 4) ? v.w : v.z) : ((j & 4) ? v.y : v.x);
        if (a + j < ocap) out[a + j] = (uint8_t)(d >> (8 * (j & 3)));
      }
    }
  }
  __syncthreads();  // (every line read before any is cleared)
  uint4 *cl = reinterpret_cast<uint4 *>(stage);
  const uint32_t used = (uint32_t)((ct + 15) >> 4) + 1;
  for (uint32_t i = threadIdx.x; i < used; i += kSpThreads) cl[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
}

// ------------------------------------------------------------ one workgroup
// A small batch of pieces encoded by ONE workgroup in order, the output
// offset running (no tickets, no look-back, no status words): the
// one-launch form behind the host path for small messages
// (cpk_encode_messages_host / cpk_encode_host below kSpSmallWords).  The
// words and the output may be pinned host memory, read and written in
// place.  Piece p is desc[2p + 1] words from word desc[2p] of `in` (pieces
// need not be contiguous: a message's table may follow the segments).  The
// run state a chunk leaves for the piece's next chunk passes through two LDS
// words.  out_off[0..n] written.
// (32768 segment words and the tables: a 256 KiB message with its table
// stays here -- 4 chunks, ~90 us, against ~135 us through the DMA pipeline)
constexpr uint64_t kSpSmallWords = 32768 + 1024;
constexpr uint32_t kSpSmallPieces = 512;   // piece descriptors staged in LDS (8 KiB)
// pieces of at most this many words (a message's segment table, tiny
// segments) are packed byte-serially by one thread from LDS: ~5 us of the
// chunk machinery (loads, three barriers, the flush) saved per piece
constexpr uint32_t kSpSerialWords = 16;
constexpr uint32_t kSpSmallLds = kSp3Lds + 16 * kSpSmallPieces + 8 * kSpSerialWords;

__device__ __forceinline__ Sp3Unit sp3_unit_at(const uint64_t *pw, uint32_t W, uint32_t p, uint32_t c, int w) {
  Sp3Unit u;
  u.pw = pw;
  u.W = W;
  u.p = p;
  u.c = c;
  u.bad = u.over = false;
  const uint32_t ns = (W + 63) >> 6;
  const uint32_t nch = max((ns + kSpCS - 1) / kSpCS, 1u);
  u.lastc = c + 1 >= nch;
  const uint32_t cs0 = c * kSpCS;
  u.cs = ns > cs0 ? (int)min((uint32_t)kSpCS, ns - cs0) : 0;
  const int per = min(kSpWS, ((u.cs + kSpWaves - 1) / kSpWaves + 1) & ~1);
  u.sa = w * per;
  u.cnt = max(0, min(per, u.cs - u.sa));
  u.wfirst = (cs0 + (uint32_t)u.sa) * 64;
  u.wrem = u.cnt ? W - u.wfirst : 0;
  return u;
}

// the descriptors of a batch of at most kSpArgPieces pieces, passed by value
// (no dependent round trip to pinned memory before the first word loads)
constexpr uint32_t kSpArgPieces = 8;
struct SpSmallArgs {
  uint64_t d[2 * kSpArgPieces];
};
__global__ __launch_bounds__(kSpThreads, 1) void sp_small_kernel(const uint64_t *__restrict__ in,
                                                                 const uint64_t *__restrict__ desc, uint32_t n,
                                                                 uint8_t *__restrict__ out,
                                                                 uint64_t *__restrict__ out_off, uint64_t ocap,
                                                                 uint32_t *err, uint64_t *flag, uint64_t seq,
                                                                 SpSmallArgs da) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem + kSp3oLut);
  uint64_t *msk = reinterpret_cast<uint64_t *>(smem + kSp3oMsk);
  uint64_t *scr = reinterpret_cast<uint64_t *>(smem + kSp3oScr);
  uint32_t *stage = reinterpret_cast<uint32_t *>(smem + kSp3oStage);
  uint64_t *ldesc = reinterpret_cast<uint64_t *>(smem + kSp3Lds);
  uint64_t *sbuf = reinterpret_cast<uint64_t *>(smem + kSp3Lds + 16 * kSpSmallPieces);
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  if (flag) small_begin();
  // the descriptors in LDS at once (they may be host memory: one round
  // trip, not two dependent ones per piece)
  if (n <= kSpArgPieces) {
    if (threadIdx.x < 2 * n) ldesc[threadIdx.x] = da.d[threadIdx.x];
  } else {
    for (uint32_t i = threadIdx.x; i < 2 * n; i += kSpThreads) ldesc[i] = desc[i];
  }
  fill_luts(lut, false);
  for (uint32_t i = threadIdx.x; i < kSp3Stage / 16; i += kSpThreads)
    reinterpret_cast<uint4 *>(stage)[i] = make_uint4(0u, 0u, 0u, 0u);
  // scr[13]: this launch's chunk-state timeouts (LDS; the context's error
  // word may hold an earlier call's, so the result cannot be judged by it)
  uint32_t *lerr = reinterpret_cast<uint32_t *>(&scr[13]);
  if (threadIdx.x == 0) scr[24] = scr[25] = scr[13] = 0;
  SpRegs R;
  R.zl = R.zh = R.dll = R.dlh = R.dl_ = R.dh_ = 0;
  R.oml = R.omh = R.ohl = R.ohh = R.oel = R.oeh = 0;
  __syncthreads();
  uint64_t g = 0;
  for (uint32_t p = 0; p < n; ++p) {
    const uint64_t w0 = sp_ld(&ldesc[2 * p]);
    const uint32_t W = (uint32_t)sp_ld(&ldesc[2 * p + 1]);
    const uint32_t nch = max((((W + 63) >> 6) + kSpCS - 1) / kSpCS, 1u);
    if (threadIdx.x == 0) out_off[p] = g;
    if (W <= kSpSerialWords) {
      // PackedOutputStream.write (:35-205) byte-serially, as the tables'
      // kernel packs them (serial_pack), the words read in one round trip
      if (threadIdx.x < W) sbuf[threadIdx.x] = in[w0 + threadIdx.x];
      __syncthreads();
      if (threadIdx.x == 0) {
        uint64_t o = g;
        serial_pack(W, [&](uint32_t i) { return sbuf[i]; }, [&](uint32_t b) {
          if (o < ocap) out[o] = (uint8_t)b;
          ++o;
        });
        scr[28] = o - g;
      }
      __syncthreads();
      g += sp_ld(&scr[28]);
      continue;
    }
    for (uint32_t c = 0; c < nch; ++c) {
      const Sp3Unit u = sp3_unit_at(in + w0, W, p, c, w);
      uint64_t V[kSpWS], LA[4];
      sp3_load(V, u, desc, lane);
      sp3_la_load(LA, u, desc, lane);
      uint64_t *prev = c ? &scr[24 + ((c - 1) & 1)] : nullptr;
      uint64_t *next = u.lastc ? nullptr : &scr[24 + (c & 1)];
      const uint64_t pst = (prev && threadIdx.x == 0) ? ld_status(prev) : 0;
      uint32_t Xlast = 0;
      uint64_t wbefore = 0;
      const uint64_t ct = sp3_chunk(R, V, LA, u, msk, scr, pst, prev, next, 1u, lerr, w, lane, Xlast, wbefore);
      if (u.cnt) sp3_b(R, V, u.cnt, lut, stage, (uint32_t)wbefore, lane);
      __syncthreads();
      sp3_flush(out, stage, g, ct, ocap);
      g += ct;
    }
  }
  // a timed-out chunk hand-off: the total reads past any capacity and the
  // host reports CPK_EDEVICE (small_encode), the context's word notes it too
  __syncthreads();
  if (threadIdx.x == 0) {
    const bool bad = *reinterpret_cast<volatile uint32_t *>(lerr) != 0;
    if (bad) atomicOr(err, 4u);
    out_off[n] = bad ? ~0ull : g;
  }
  if (flag) small_done(flag, seq);
}
