// encode_v3.hip -- included by packed_codec.hip inside namespace cpk.
//
// Workgroup-per-tile encoder.  The batch's words [swo[0], swo[n]) are cut
// into fixed tiles of kE3TileWords consecutive words regardless of where the
// pieces start: a piece start is a run boundary inside a tile
// (PackedOutputStream.java:36-43 re-initialises all run state per write()).
// A 256-thread workgroup encodes one tile in three phases:
//   1. each wave loads its 16 steps of 64 words (lane = word), computes every
//      word's nonzero-byte tag and keeps words and tags in registers; the tags
//      also go to LDS (one byte per word) for the other waves, and the last
//      wave classifies up to 4 steps past the tile to find where the run
//      crossing its end stops (the counts need it);
//   2. each wave derives the run state entering its first word from the tags
//      before it -- or, when the tile's first run continues the previous
//      tile's, from that tile's published exit state -- then walks its steps
//      with wave-uniform carries and gives every word its role
//      (PackedOutputStream.java:119-193 restated per word):
//      run boundaries, 0x00 heads every 256 words of a zero run, 0xFF heads
//      and literal-run members by a carry-propagate add over the D and D/L
//      masks (a D/L stretch longer than 256 words walks the head chain), and
//      the packed size of every word;
//   3. after a decoupled look-back over the tile totals has given the tile's
//      output offset, each wave builds every word's packed string (tag +
//      v_perm-compacted bytes + count), ORs it into a 2 KiB LDS ring at its
//      output position and streams complete 16-byte lines to memory.
// Tiles are dealt round-robin to a persistent grid that fits on the device
// at once, so every tile a workgroup waits on is being worked on.
// tools/e3_model.py is this algorithm at mask level on the CPU.

constexpr int kE3Waves = 4;
constexpr int kE3Threads = 64 * kE3Waves;
constexpr int kE3Steps = 16;                             // 64-word steps per wave
constexpr int kE3WaveWords = 64 * kE3Steps;              // 1024
constexpr int kE3TileWords = kE3Waves * kE3WaveWords;    // 4096
constexpr int kE3La = 4;                                 // look-ahead steps
constexpr int kE3Rows = kE3Waves * kE3Steps + kE3La;     // 68 step rows
constexpr uint32_t kE3RingBytes = 2048;                  // output ring per wave
constexpr uint32_t kE3RingLines = kE3RingBytes / 16;
constexpr uint32_t kE3RingDw = kE3RingBytes / 4;
// LDS byte offsets.  The per-tile state (tags, step rows, wave totals) is
// double-buffered: a workgroup builds tile i's state while it finishes tile
// i-1 (look-back + strings), so the look-back never stalls the pipeline.
// Phase 3 re-reads the tile's words from memory (L2 / Infinity Cache).
constexpr uint32_t kE3oLut = 0;                                    // u64[256]
constexpr uint32_t kE3oRing = kE3oLut + 2048;                      // u32[waves][512]
constexpr uint32_t kE3oBuf = kE3oRing + kE3Waves * kE3RingBytes;   // 2 x per-tile state
constexpr uint32_t kE3bTag = 0;                                    // u8[rows][64]
constexpr uint32_t kE3bPs = kE3bTag + kE3Rows * 64;                // u64[rows] piece starts
constexpr uint32_t kE3bB = kE3bPs + kE3Rows * 8;                   // u64[rows] run boundaries
constexpr uint32_t kE3bRole = kE3bB + kE3Rows * 8;                 // u8[rows][64] word roles
constexpr uint32_t kE3bScr = kE3bRole + kE3Rows * 64;  // int[32]: wave totals, offset, partial sums
constexpr uint32_t kE3BufBytes = kE3bScr + 128;
constexpr uint32_t kE3Lds = kE3oBuf + 2 * kE3BufBytes;
constexpr uint32_t kE3oPs = kE3oBuf + kE3bPs;  // (alignment check below)
static_assert(kE3oPs % 8 == 0 && kE3oRing % 16 == 0, "LDS alignment");

#ifndef CPK_E3_WPE
#define CPK_E3_WPE 4
#endif

// Look-back words: [63:48] launch epoch, [47:46] flag (1 aggregate,
// 2 inclusive prefix), [45:0] value.  A word from another launch reads as
// "not published", so the arrays need no clearing between launches.
constexpr uint64_t kE3ValMask = (1ull << 46) - 1;
__device__ __forceinline__ uint64_t e3_word(uint32_t ep, uint32_t flag, uint64_t v) {
  return ((uint64_t)ep << 48) | ((uint64_t)flag << 46) | (v & kE3ValMask);
}
__device__ __forceinline__ uint32_t e3_flag(uint64_t w, uint32_t ep) {
  return (uint32_t)(w >> 48) == ep ? (uint32_t)(w >> 46) & 3u : 0u;
}

__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// bit `lane` of a wave-uniform mask: one v_cndmask on the SGPR pair
__device__ __forceinline__ uint32_t lanebit(uint64_t mask) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(r) : "s"(mask));
  return r;
}

// Run state at a word position: the run the word would continue.
//   g   0 zero run, 1 D/L stretch (words with <= 1 zero byte), 2 none
//   len words of the run before the position (zero runs: only len mod 256
//       matters, the 0x00 heads are every 256 words from the run start)
//   hd  D/L stretch: words since its last 0xFF head, capped at 256; 0 = no
//       head yet (PackedOutputStream.java:143-161: a head's run takes the
//       next <= 255 words of the stretch)
struct E3St {
  int g, len, hd;
};
// tile exit states: [63:48] epoch, [46] valid, [33:32] g, [31:20] hd, [19:0] len
__device__ __forceinline__ uint64_t e3_st_pack(uint32_t ep, E3St s) {
  const uint32_t len = s.g == 0 ? (uint32_t)(s.len & 255) : (uint32_t)min(s.len, (1 << 20) - 1);
  return ((uint64_t)ep << 48) | (1ull << 46) | ((uint64_t)(s.g & 3) << 32) |
         ((uint64_t)(s.hd & 0xfff) << 20) | len;
}
__device__ __forceinline__ E3St e3_st_unpack(uint64_t w) {
  E3St s;
  s.g = (int)(w >> 32) & 3;
  s.hd = (int)(w >> 20) & 0xfff;
  s.len = (int)(w & 0xfffff);
  return s;
}

// nonzero-byte tag of a word (PackedOutputStream.java:64-117): bit i set iff
// byte i != 0.  SWAR: bit 7 of every byte of t = byte != 0, gathered by shifts.
__device__ __forceinline__ uint32_t e3_tag(uint64_t v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  const uint32_t tl = ((lo & 0x7f7f7f7fu) + 0x7f7f7f7fu) | lo;
  const uint32_t th = ((hi & 0x7f7f7f7fu) + 0x7f7f7f7fu) | hi;
  const uint32_t y = ((tl >> 7) & 0x01010101u) | ((th >> 3) & 0x10101010u);
  return (y | (y >> 7) | (y >> 14) | (y >> 21)) & 0xffu;
}
// 0 = Z (all-zero word), 1 = D/L (<= 1 zero byte), 2 = M
__device__ __forceinline__ int e3_grp(uint32_t m) {
  return m == 0 ? 0 : (__builtin_popcount(m) >= 7 ? 1 : 2);
}

// state entering tile t from tile t-1's published exit state (one wave)
__device__ E3St e3_tile_entry(const uint64_t *tstate, uint32_t t, uint32_t ep, uint32_t *err,
                              int lane) {
  uint32_t spins = 0;
  for (;;) {
    const uint64_t v = uni64(ld_status(const_cast<uint64_t *>(&tstate[t - 1])));
    if ((uint32_t)(v >> 48) == ep) return e3_st_unpack(v);
    if (++spins > (1u << 16)) {  // cannot happen with a co-resident grid (~0.1 s)
      if (lane == 0) atomicOr(err, 4u);
      E3St s = {2, 0, 0};
      return s;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// first D word (tag 0xff) at tile position >= x and < lim, else lim
__device__ int e3_first_d(const uint8_t *tagrow, int x, int lim, int lane) {
  for (int r = x >> 6; r * 64 < lim; ++r) {
    const int p = r * 64 + lane;
    const uint64_t b = __ballot(p >= x && p < lim && tagrow[p] == 0xffu);
    if (b) return r * 64 + __builtin_ctzll(b);
  }
  return lim;
}

// State entering tile position wp (> 0, a multiple of 64): the run holding
// word wp - 1, from the tag rows; a run reaching back to the tile's first
// word continues from the previous tile's exit state.  All 64 lanes.
__device__ E3St e3_state_at(const uint8_t *tagrow, const uint64_t *psrow, int wp,
                            const uint64_t *tstate, uint32_t t, uint32_t ep, uint32_t *err,
                            int lane) {
  E3St s = {2, 0, 0};
  const int g = e3_grp((uint32_t)uni((int)tagrow[wp - 1]));
  if (g == 2) return s;
  // run start: after the last word of another group, or at the last piece start
  int rs = -1;
  for (int r = (wp - 1) >> 6; r >= 0; --r) {
    const uint64_t other = __ballot(e3_grp(tagrow[r * 64 + lane]) != g);
    const uint64_t ps = uni64(psrow[r]);
    int c = -1;
    if (other) c = r * 64 + 64 - __builtin_clzll(other);
    if (ps) c = max(c, r * 64 + 63 - __builtin_clzll(ps));
    if (c >= 0) {
      rs = c;
      break;
    }
  }
  bool before = false;
  if (rs < 0) {  // reaches the tile's first word, which is no piece start
    rs = 0;
    if (t > 0) {
      const E3St tin = e3_tile_entry(tstate, t, ep, err, lane);
      if (tin.g == g) {
        before = true;
        s = tin;
      }
    }
  }
  if (g == 0) {
    s.g = 0;
    s.len = (before ? s.len : 0) + (wp - rs);
    s.hd = 0;
    return s;
  }
  // D/L stretch: its 0xFF head chain from rs (PackedOutputStream.java:143-161):
  // the first D is a head, then the first D at least 256 words after a head
  const int len0 = before ? s.len : 0;
  bool hasH = before && s.hd > 0;
  int h = hasH ? -s.hd : 0;
  for (;;) {
    const int from = hasH ? max(h + 256, rs) : rs;
    if (from >= wp) break;
    const int d = e3_first_d(tagrow, from, wp, lane);
    if (d >= wp) break;
    h = d;
    hasH = true;
  }
  s.g = 1;
  s.len = len0 + (wp - rs);
  s.hd = hasH ? min(wp - h, 256) : 0;
  return s;
}

#ifndef CPK_E3_LBW
#define CPK_E3_LBW 512
#endif
constexpr int kE3LbW = CPK_E3_LBW;  // predecessors read per look-back poll

// Decoupled look-back over the tile totals (one wave, all lanes): publishes
// the aggregate, returns the exclusive prefix, publishes the inclusive one.
__device__ uint64_t e3_lookback(uint64_t *status, uint32_t t, uint64_t agg, uint32_t ep,
                                uint32_t *err, int lane) {
  if (lane == 0) st_status(&status[t], e3_word(ep, t == 0 ? 2u : 1u, agg));
  if (t == 0) return 0;
  uint64_t excl = 0;
  int64_t top = (int64_t)t - 1;
  uint32_t spins = 0;
  for (;;) {
    // one poll reads the kE3LbW nearest predecessors, all loads in flight
    // at once: with the pipelined grid the nearest inclusive prefix is about
    // one grid's worth of tiles back
    constexpr int kPer = kE3LbW / 64;
    uint64_t v[kPer];
    int fi = kPer;  // first inclusive among this lane's (nearest first)
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int64_t idx = top - kPer * lane - i;
      v[i] = idx >= 0 ? ld_status(&status[idx]) : e3_word(ep, 2u, 0);
    }
#pragma unroll
    for (int i = kPer - 1; i >= 0; --i)
      if (e3_flag(v[i], ep) == 2) fi = i;
    const uint64_t has = __ballot(fi < kPer);
    const int fln = has ? __builtin_ctzll(has) : 64;
    const int firstPos = fln < 64 ? kPer * fln + __builtin_amdgcn_readlane(fi, fln) : kE3LbW;
    bool z = false;
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      if (kPer * lane + i <= firstPos) {
        z = z || e3_flag(v[i], ep) == 0;
        sum += v[i] & kE3ValMask;
      }
    }
    if (__ballot(z)) {
      if (++spins > (1u << 16)) {  // cannot happen with a co-resident grid (~0.1 s)
        if (lane == 0) atomicOr(err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    excl += sum;
    if (firstPos < kE3LbW) break;
    top -= kE3LbW;
  }
  if (lane == 0) st_status(&status[t], e3_word(ep, 2u, excl + agg));
  return excl;
}

// bytes [j0, j1) of global line L from the ring, then clears the ring line
__device__ __forceinline__ void e3_store_bytes(uint8_t *out, uint32_t *ring, uint64_t L, int j0,
                                               int j1, int lane) {
  uint4 *rl = reinterpret_cast<uint4 *>(ring) + (L & (kE3RingLines - 1));
  const uint4 val = *rl;
  if (lane >= j0 && lane < j1) {
    const uint32_t d = (lane & 8) ? ((lane & 4) ? val.w : val.z) : ((lane & 4) ? val.y : val.x);
    out[L * 16 + lane] = (uint8_t)(d >> (8 * (lane & 3)));
  }
  wave_lds_order();
  if (lane == 0) *rl = make_uint4(0u, 0u, 0u, 0u);
}

// stores the complete lines [fl, upto) of the ring; bytes below `lo` belong
// to the previous wave / tile (only the wave's first line can hold them)
__device__ __forceinline__ void e3_flush(uint8_t *out, uint32_t *ring, uint64_t &fl, uint64_t upto,
                                         uint64_t lo, int lane) {
  if (fl >= upto) return;
  if (fl * 16 < lo) {
    e3_store_bytes(out, ring, fl, (int)(lo - fl * 16), 16, lane);
    ++fl;
  }
  for (uint64_t L0 = fl; L0 < upto; L0 += 64) {
    const uint64_t L = L0 + lane;
    if (L < upto) {
      uint4 *rl = reinterpret_cast<uint4 *>(ring) + (L & (kE3RingLines - 1));
      const uint4 val = *rl;
      *rl = make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4 *>(out + L * 16) = val;
    }
  }
  fl = upto;
}

// tfirst[t] = first piece i with swo[i] >= swo[0] + t * kE3TileWords
// (n + 1 if none), t in [0, nt + 1], nt = min(tiles of the batch, ntb).
// Also checks the size hint; an empty batch gets all-zero piece offsets.
__global__ void e3_plan_kernel(const uint64_t *__restrict__ swo, uint32_t n, uint32_t ntb,
                               uint32_t *tfirst, uint64_t *out_off, uint64_t hint, uint32_t *err) {
  const uint64_t base = swo[0], N = swo[n];
  uint64_t nt = (N - base + kE3TileWords - 1) / kE3TileWords;
  if (nt > ntb) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, 1u);
    nt = ntb;
  }
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i <= (uint64_t)n + 1;
       i += (uint64_t)gridDim.x * blockDim.x) {
    if (N == base) {
      if (i <= n) out_off[i] = 0;
      if (i <= 1) tfirst[i] = 0;
      continue;
    }
    uint64_t lo = 0, hi = 0;
    if (i > 0) {
      const uint64_t prev = swo[i - 1];
      lo = (prev - base) / kE3TileWords + 1;
      hi = i <= n ? (swo[i] - base) / kE3TileWords : nt + 1;
      if (i <= n && hint && swo[i] - prev > hint) atomicOr(err, 1u);
    }
    if (hi > nt + 1) hi = nt + 1;
    for (uint64_t t = lo; t <= hi; ++t) tfirst[t] = (uint32_t)i;
  }
}

constexpr int kE3MaxPer = 5;  // tile sizes each thread sums: grids up to 1280 workgroups

// Phases 0-2 of tile t into state buffer `bf` (all waves; ends with the
// wave totals in bf's scratch and the tile's exit run state published).
__device__ __forceinline__ void e3_front(const uint64_t *__restrict__ in,
                                         const uint64_t *__restrict__ swo,
                                         const uint32_t *__restrict__ tfirst, uint8_t *bf,
                                         uint64_t *tstate, uint32_t ep, uint32_t *err, uint32_t t,
                                         uint32_t nt, uint64_t base, uint64_t N, int w, int wb,
                                         int lane) {
  uint8_t *tagrow = bf + kE3bTag;
  uint64_t *psrow = reinterpret_cast<uint64_t *>(bf + kE3bPs);
  uint64_t *brow = reinterpret_cast<uint64_t *>(bf + kE3bB);
  uint8_t *rolerow = bf + kE3bRole;
  int *scr = reinterpret_cast<int *>(bf + kE3bScr);
  const int tid = w * 64 + lane;
  const uint64_t T0 = base + (uint64_t)t * kE3TileWords;
  const uint64_t rem = N - T0;
  const int TW = rem < (uint64_t)kE3TileWords ? (int)rem : kE3TileWords;    // words of the tile
  const int pN = rem < (uint64_t)(kE3Rows * 64) ? (int)rem : kE3Rows * 64;  // batch end
  // ---- phase 1a: the loads go out first --------------------------------------
  const uint64_t *src = in + T0;
  uint64_t v[kE3Steps];
#pragma unroll
  for (int s = 0; s < kE3Steps; ++s) {
    const int k = wb + 64 * s + lane;
    const uint64_t x = src[min(k, TW - 1)];
    v[s] = k < TW ? x : 0ull;
  }
  // ---- phase 0: piece-start rows, boundary rows (buffer free since the
  // previous iteration's barrier) ----------------------------------------------
  if (tid < kE3Rows) {
    psrow[tid] = 0;
    brow[tid] = 0;
  }
  __syncthreads();
  {
    const uint32_t p0 = tfirst[t], p2 = tfirst[min(t + 2, nt + 1)];
    for (uint32_t i = p0 + tid; i < p2; i += kE3Threads) {
      const uint64_t k = swo[i] - T0;
      if (k < (uint64_t)pN)
        atomicOr(reinterpret_cast<unsigned long long *>(&psrow[k >> 6]), 1ull << (k & 63));
    }
    if (tid == 0 && pN < kE3Rows * 64)  // the end of the batch ends every run
      atomicOr(reinterpret_cast<unsigned long long *>(&brow[pN >> 6]), 1ull << (pN & 63));
  }
  // ---- phase 1b: tags ----------------------------------------------------------
  uint32_t mlast = 0;  // tag of the wave's last word
#pragma unroll
  for (int s = 0; s < kE3Steps; ++s) {
    const uint32_t m = e3_tag(v[s]);
    tagrow[wb + 64 * s + lane] = (uint8_t)m;
    mlast = m;
  }
  __syncthreads();  // B1: tags and piece starts of the whole tile
  if (w == kE3Waves - 1 && TW == kE3TileWords && pN > kE3TileWords) {
    // look-ahead: boundaries of up to kE3La steps past the tile, until the
    // run crossing the tile end stops (counts are capped at 255 words)
    int gprev = e3_grp((uint32_t)__builtin_amdgcn_readlane((int)mlast, 63));
    for (int r = 0; r < kE3La; ++r) {
      const int k = kE3TileWords + 64 * r + lane;
      const bool ok = k < pN;
      const uint64_t x = in[T0 + (uint64_t)min(k, pN - 1)];
      const int g = ok ? e3_grp(e3_tag(x)) : 3;
      const int gp = wave_shr1(g, gprev);
      const uint64_t ps = uni64(psrow[kE3Waves * kE3Steps + r]);
      const uint64_t b = __ballot(ok && (g != gp || g == 2)) | ps | __ballot(k == pN);
      if (lane == 0) brow[kE3Waves * kE3Steps + r] = b;
      gprev = __builtin_amdgcn_readlane(g, 63);
      if (b) break;
    }
  }
  // ---- phase 2: roles and sizes ------------------------------------------------
  int wtot = 0;
  if (wb < TW) {
    E3St st = {2, 0, 0};
    if (w == 0) {
      if (!(uni64(psrow[0]) & 1) && t > 0) st = e3_tile_entry(tstate, t, ep, err, lane);
    } else {
      st = e3_state_at(tagrow, psrow, wb, tstate, t, ep, err, lane);
    }
    const uint64_t lem = lane == 63 ? ~0ull : ((2ull << lane) - 1);  // lanes <= this one
    uint32_t acc = 0;  // this lane's packed bytes over the steps
#pragma unroll 1
    for (int s = 0; s < kE3Steps; ++s) {
      const int kb = wb + 64 * s;
      const int k = kb + lane;
      const bool valid = k < TW;
      const uint32_t m = tagrow[k];
      const uint32_t pop = (uint32_t)__builtin_popcount(m);
      const uint64_t PS = uni64(psrow[kb >> 6]);
      // run boundaries (piece starts, group changes, every M word), per lane
      const int g = !valid ? 3 : (m == 0 ? 0 : (pop >= 7 ? 1 : 2));
      const int gp = wave_shr1(g, st.g);
      const bool isB = valid && (lanebit(PS) || g != gp || g == 2);
      const uint64_t B = __ballot(isB), D = __ballot(m == 0xffu), DL = __ballot(g == 1);
      // this lane's run start (step-relative; the carried run started st.len
      // words before the step) and the last D before it
      const uint64_t bl = B & lem;
      const int rs = bl ? 63 - __builtin_clzll(bl) : -st.len;
      const uint64_t dl = D & (lem >> 1);
      const int lastD = dl ? 63 - __builtin_clzll(dl) : (st.hd > 0 ? -st.hd : -(1 << 30));
      // 0x00 heads every 256 words of a zero run from its start (:119-131);
      // literal-run members: a D earlier in the same D/L stretch (:133-161,
      // exact for stretches of <= 256 words; longer ones below)
      uint32_t zh = (g == 0 && ((lane - rs) & 255) == 0) ? 1u : 0u;
      uint32_t memb = (g == 1 && lastD >= rs) ? 1u : 0u;
      uint32_t dh = (m == 0xffu && !memb) ? 1u : 0u;
      const uint64_t BV = B | __ballot(!valid);  // (past the batch's end no run continues)
      const int f = BV ? __builtin_ctzll(BV) : 64;  // words [0, f) continue the carried run
      int h1 = -1;
      if (st.g == 1 && st.len + f > 256) {
        // the carried stretch is longer than 256 words: members lie within
        // 255 words of a head, the next head is the first D 256 or more
        // words after the last (:143-161)
        const uint64_t rng = f >= 64 ? ~0ull : ((1ull << f) - 1);
        uint64_t mc = 0;
        if (st.hd > 0 && st.hd <= 255) {
          const int me = 255 - st.hd;
          mc = me >= 63 ? ~0ull : ((2ull << me) - 1);
        }
        const int js = st.hd > 0 ? max(0, 256 - st.hd) : 0;
        const uint64_t dc = js >= 64 ? 0ull : (D & rng & (~0ull << js));
        if (dc) {
          h1 = __builtin_ctzll(dc);
          mc |= h1 == 63 ? 0ull : (~0ull << (h1 + 1));
        }
        if ((rng >> lane) & 1) {
          memb = ((mc & DL) >> lane) & 1;
          dh = (h1 == lane) ? 1u : 0u;
        }
      }
      const uint32_t isH = zh | dh;
      // packed bytes: M words 1 + popcount, D/L 8 (+2 for a 0xFF head), 0x00 heads 2
      const uint32_t nb = !valid ? 0u : (g == 2 ? 1 + pop : (g == 1 ? 8 + 2 * dh : 2 * zh));
      acc += nb;
      rolerow[k] = (uint8_t)(nb | (memb << 4) | (isH << 5));
      const uint64_t bend = __ballot(k == pN);
      if (lane == 0) brow[kb >> 6] = B | bend;
      // the run state entering the next step
      if (B) {
        const int lb = 63 - __builtin_clzll(B);
        const int g63 = __builtin_amdgcn_readlane(g, 63);
        st.g = g63 == 0 ? 0 : (g63 == 1 ? 1 : 2);
        st.len = 64 - lb;
        st.hd = 0;
        if (st.g == 1) {
          const uint64_t dd = D & (~0ull << lb);
          st.hd = dd ? 64 - __builtin_ctzll(dd) : 0;
        }
      } else if (st.g != 2) {
        st.len += 64;
        if (st.g == 1) {
          if (h1 >= 0) st.hd = 64 - h1;
          else if (st.hd > 0) st.hd = min(st.hd + 64, 256);
          else st.hd = D ? 64 - __builtin_ctzll(D) : 0;
        }
      }
    }
    wtot = wave_incl_add((int)acc);
    wtot = __builtin_amdgcn_readlane(wtot, 63);
    // the tile's exit state, for the next tile's first run
    if (w == kE3Waves - 1 && lane == 0) st_status(&tstate[t], e3_st_pack(ep, st));
  }
  if (lane == 0) scr[w] = wtot;
}

// Look-back of tile t from state buffer `bf` (wave 0): the tile's output
// offset into the buffer's scratch.
__device__ __forceinline__ void e3_tile_offset(const uint64_t *__restrict__ swo, uint32_t n,
                                               uint64_t *__restrict__ out_off, uint8_t *bf,
                                               uint64_t *status, uint32_t ep, uint32_t *err,
                                               uint32_t t, uint64_t base, uint64_t N, int w,
                                               int lane) {
  int *scr = reinterpret_cast<int *>(bf + kE3bScr);
  const uint64_t T0 = base + (uint64_t)t * kE3TileWords;
  const uint64_t rem = N - T0;
  const int TW = rem < (uint64_t)kE3TileWords ? (int)rem : kE3TileWords;
  if (w == 0) {
    uint64_t tot = 0;
    for (int q = 0; q < kE3Waves; ++q) tot += (uint32_t)scr[q];
    const uint64_t excl = e3_lookback(status, t, tot, ep, err, lane);
    if (lane == 0) {
      *reinterpret_cast<uint64_t *>(&scr[8]) = excl;
      if (T0 + (uint64_t)TW == N)  // pieces starting at the end of the batch (and swo[n])
        for (int64_t j = n; j >= 0 && swo[j] == N; --j) out_off[j] = excl + tot;
    }
  }
}

// Phase 3 of tile t after its look-back (all waves).
__device__ __forceinline__ void e3_strings(const uint64_t *__restrict__ in,
                                           const uint64_t *__restrict__ swo, uint32_t n,
                                           const uint32_t *__restrict__ tfirst,
                                           uint8_t *__restrict__ out,
                                           uint64_t *__restrict__ out_off, const uint64_t *lut,
                                           uint32_t *ring, uint8_t *bf, uint32_t t, uint64_t base,
                                           uint64_t N, int w, int wb, int lane,
                                           const uint64_t (&v)[kE3Steps]) {
  uint64_t *psrow = reinterpret_cast<uint64_t *>(bf + kE3bPs);
  uint64_t *brow = reinterpret_cast<uint64_t *>(bf + kE3bB);
  const uint8_t *rolerow = bf + kE3bRole;
  int *scr = reinterpret_cast<int *>(bf + kE3bScr);
  const uint64_t gtm = lane == 63 ? 0ull : (~0ull << (lane + 1));  // lanes above this one
  const uint64_t T0 = base + (uint64_t)t * kE3TileWords;
  const uint64_t rem = N - T0;
  const int TW = rem < (uint64_t)kE3TileWords ? (int)rem : kE3TileWords;
  if (wb < TW) {
    uint64_t obase = *reinterpret_cast<const uint64_t *>(&scr[8]);
    for (int q = 0; q < w; ++q) obase += (uint32_t)scr[q];
    uint64_t rpos = obase;     // output offset of the next string
    uint64_t fl = obase >> 4;  // first line not stored yet
    int nbrRow = -1, nbr = 0;  // first boundary in the rows after nbrRow
    const uint32_t pfirst = tfirst[t], plast = tfirst[t + 1];
#pragma unroll
      for (int s = 0; s < kE3Steps; ++s) {
        const int kb = wb + 64 * s;
        const int k = kb + lane;
        const uint64_t word = v[s];
        const uint32_t m = e3_tag(word);
        const uint32_t role = rolerow[k];
        const uint32_t nb = role & 15u, isMb = (role >> 4) & 1u, isH = (role >> 5) & 1u;
        const int incl = wave_incl_add((int)nb);
        const uint32_t o = (uint32_t)incl - nb;
        const uint32_t stot = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
        uint32_t cnt = 0;
        if (__ballot(isH)) {
          // a head's count: words to the run's end, at most 255 (:123-131, :143-164)
          const int row = kb >> 6;
          if (nbrRow != row) {
            nbrRow = row;
            nbr = kE3Rows * 64;
            for (int r = row + 1; r < kE3Rows; ++r) {
              const uint64_t br = uni64(brow[r]);
              if (br) {
                nbr = r * 64 + __builtin_ctzll(br);
                break;
              }
            }
          }
          const uint64_t bb = uni64(brow[row]) & gtm;
          const int re = bb ? kb + __builtin_ctzll(bb) : nbr;
          cnt = isH ? (uint32_t)min(255, re - k - 1) : 0u;
        }
        const uint32_t lo = (uint32_t)word, hi = (uint32_t)(word >> 32);
        const uint64_t sel = lut[m];
        const uint32_t c0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
        const uint32_t c1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
        const uint32_t c0p = m == 0 ? cnt : c0;
        uint32_t s0 = m | (c0p << 8);
        uint32_t s1 = __builtin_amdgcn_alignbyte(c1, c0p, 3);
        uint32_t s2 = __builtin_amdgcn_alignbyte(m == 0xffu ? cnt : 0u, c1, 3);
        if (isMb) {  // literal-run member: the word verbatim (:163-171)
          s0 = lo;
          s1 = hi;
          s2 = 0;
        }
        // OR the string into the ring at its output offset
        const uint32_t p = (uint32_t)rpos + o;
        const uint32_t sh = (p & 3) * 8;
        const uint64_t a01 = (((uint64_t)s1 << 32) | s0) << sh;
        const uint64_t a12 = (((uint64_t)s2 << 32) | s1) << sh;
        const uint32_t w3 = (uint32_t)(((uint64_t)s2 << sh) >> 32);
        const uint32_t d0 = (p >> 2) & (kE3RingDw - 1);
        const uint32_t end = (p & 3) + nb;
        if (nb) atomicOr(&ring[d0], (uint32_t)a01);
        if (end > 4) {
          uint32_t *dp = &ring[(d0 + 1) & (kE3RingDw - 1)];
          if (end >= 8) *dp = (uint32_t)(a01 >> 32);
          else atomicOr(dp, (uint32_t)(a01 >> 32));
        }
        if (end > 8) {
          uint32_t *dp = &ring[(d0 + 2) & (kE3RingDw - 1)];
          if (end >= 12) *dp = (uint32_t)(a12 >> 32);
          else atomicOr(dp, (uint32_t)(a12 >> 32));
        }
        if (end > 12) atomicOr(&ring[(d0 + 3) & (kE3RingDw - 1)], w3);
        // piece offsets: out_off of every piece starting at this word
        const uint64_t ps = uni64(psrow[kb >> 6]);
        if (ps && ((ps >> lane) & 1)) {
          const uint64_t gk = T0 + (uint64_t)(kb + lane);
          uint32_t lo_i = pfirst, hi_i = plast;  // first piece with swo >= gk
          while (lo_i < hi_i) {
            const uint32_t mid = (lo_i + hi_i) >> 1;
            if (swo[mid] < gk) lo_i = mid + 1;
            else hi_i = mid;
          }
          for (uint32_t j = lo_i; j <= n && swo[j] == gk; ++j) out_off[j] = rpos + o;
        }
        rpos += stot;
        wave_lds_order();
        e3_flush(out, ring, fl, rpos >> 4, obase, lane);
      }

    // the wave's last, partial line
    if (rpos > fl * 16) {
      const int j0 = (int)((obase > fl * 16 ? obase : fl * 16) - fl * 16);
      e3_store_bytes(out, ring, fl, j0, (int)(rpos - fl * 16), lane);
    }
  }
}

__global__ __launch_bounds__(kE3Threads, CPK_E3_WPE) void encode3_kernel(
    const uint64_t *__restrict__ in, const uint64_t *__restrict__ swo, uint32_t n, uint32_t ntb,
    const uint32_t *__restrict__ tfirst, uint8_t *__restrict__ out, uint64_t *__restrict__ out_off,
    uint64_t *status, uint64_t *rbase, uint64_t *tstate, uint32_t ep, uint32_t *err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint64_t *lut = reinterpret_cast<const uint64_t *>(smem + kE3oLut);
  // the wave index through readfirstlane: hipcc's divergence analysis treats
  // threadIdx.x >> 6 as divergent, which would turn every wave-uniform branch
  // below into an exec-masked one
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  uint32_t *ring = reinterpret_cast<uint32_t *>(smem + kE3oRing + w * kE3RingBytes);
  fill_luts(reinterpret_cast<uint64_t *>(smem + kE3oLut), false);
  for (uint32_t i = lane_id(); i < kE3RingLines; i += 64)
    reinterpret_cast<uint4 *>(ring)[i] = make_uint4(0u, 0u, 0u, 0u);
  const uint64_t base = swo[0], N = swo[n];
  uint32_t nt = (uint32_t)((N - base + kE3TileWords - 1) / kE3TileWords);
  if (nt > ntb) nt = ntb;  // (reported by the plan kernel)
  __syncthreads();
  WPH_INIT
  const int tid = threadIdx.x;
  const uint32_t G = gridDim.x, g = blockIdx.x;
  // Two-stage pipeline over this workgroup's tiles t_i = g + i G ("round" i):
  // iteration i builds t_i's roles and publishes its packed size (front),
  // then finishes t_{i-1} (back).  t_{i-1}'s output offset is the base of
  // round i-1 (published by that round's last workgroup in its back stage)
  // plus the sizes of the round's g tiles before it (all published an
  // iteration ago): loads issued before the front, summed after it.
  for (uint32_t i = 0;; ++i) {
    const uint32_t t = g + i * G;
    uint64_t la[kE3MaxPer], lrb = 0;
    if (i > 0) {
      const uint32_t r0 = (i - 1) * G;  // first tile of round i-1
#pragma unroll
      for (int j = 0; j < kE3MaxPer; ++j) {
        const uint32_t q = tid + kE3Threads * j;
        la[j] = q < g ? ld_status(&status[r0 + q]) : e3_word(ep, 1u, 0);
      }
      lrb = i > 1 ? ld_status(&rbase[i - 1]) : e3_word(ep, 1u, 0);
    }
    // opaque per iteration: hipcc otherwise hoists ~100 per-lane addresses
    // and per-step row offsets out of the loop and spills them
    int wb = w * kE3WaveWords;
    asm volatile("" : "+s"(wb));
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    uint8_t *bcur = smem + kE3oBuf + (i & 1) * kE3BufBytes;
    uint8_t *bprev = smem + kE3oBuf + ((i & 1) ^ 1) * kE3BufBytes;
    if (t < nt) e3_front(in, swo, tfirst, bcur, tstate, ep, err, t, nt, base, N, w, wb, lane);
    WPH(0)
    __syncthreads();  // B2: t's totals and rows; t_{i-1}'s buffer is complete too
    WPH(1)
    if (t < nt && tid == 0) {  // t's packed size for the next round's offsets
      const int *sc = reinterpret_cast<const int *>(bcur + kE3bScr);
      uint64_t tot = 0;
      for (int q = 0; q < kE3Waves; ++q) tot += (uint32_t)sc[q];
      st_status(&status[t], e3_word(ep, 1u, tot));
    }
    if (i > 0) {
      // t_{i-1}'s words again (L2 / Infinity Cache), all in flight across the
      // look-back wait and ahead of any store of phase 3
      const uint32_t tp = t - gridDim.x;
      const uint64_t T0p = base + (uint64_t)tp * kE3TileWords;
      const int TWp = N - T0p < (uint64_t)kE3TileWords ? (int)(N - T0p) : kE3TileWords;
      uint64_t v[kE3Steps];
#pragma unroll
      for (int s = 0; s < kE3Steps; ++s) {
        const int k = wb + 64 * s + lane;
        const uint64_t x = in[T0p + (uint64_t)min(k, TWp - 1)];
        v[s] = k < TWp ? x : 0ull;
      }
      {
        // t_{i-1}'s offset: check the loads issued before the front (re-poll
        // what was not published yet: a lagging workgroup), sum them
        const uint32_t r0 = (i - 1) * G;
        uint32_t spins = 0;
        for (;;) {
          bool miss = e3_flag(lrb, ep) == 0;
#pragma unroll
          for (int j = 0; j < kE3MaxPer; ++j) miss = miss || e3_flag(la[j], ep) == 0;
          if (!__syncthreads_or(miss)) break;
          if (++spins > (1u << 16)) {  // cannot happen with a co-resident grid
            if (tid == 0) atomicOr(err, 4u);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
#pragma unroll
          for (int j = 0; j < kE3MaxPer; ++j) {
            const uint32_t q = tid + kE3Threads * j;
            if (q < g && e3_flag(la[j], ep) == 0) la[j] = ld_status(&status[r0 + q]);
          }
          if (e3_flag(lrb, ep) == 0) lrb = ld_status(&rbase[i - 1]);
        }
        uint64_t sum = 0;
#pragma unroll
        for (int j = 0; j < kE3MaxPer; ++j) sum += la[j] & kE3ValMask;
        for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
        uint64_t *ps = reinterpret_cast<uint64_t *>(bprev + kE3bScr + 64);
        if (lane == 0) ps[w] = sum;
        __syncthreads();
        int *sc = reinterpret_cast<int *>(bprev + kE3bScr);
        const uint64_t excl = (lrb & kE3ValMask) + ps[0] + ps[1] + ps[2] + ps[3];
        uint64_t tot = 0;
        for (int q = 0; q < kE3Waves; ++q) tot += (uint32_t)sc[q];
        if (tid == 0) {
          *reinterpret_cast<uint64_t *>(&sc[8]) = excl;
          if (g == G - 1) st_status(&rbase[i], e3_word(ep, 1u, excl + tot));  // next round's base
          const uint64_t T0 = base + (uint64_t)tp * kE3TileWords;
          if (T0 + (uint64_t)TWp == N)  // pieces starting at the end of the batch (and swo[n])
            for (int64_t j = n; j >= 0 && swo[j] == N; --j) out_off[j] = excl + tot;
        }
      }
      WPH(2)
      __syncthreads();  // B3: the tile's output offset
      WPH(3)
      e3_strings(in, swo, n, tfirst, out, out_off, lut, ring, bprev, tp, base, N, w, wb, lane, v);
    }
    WPH(4)
    if (t >= nt) break;
    __syncthreads();  // bprev is free for the next iteration's front
    WPH(5)
  }
  WPH_FLUSH(40)
}
