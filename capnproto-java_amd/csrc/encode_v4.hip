// Encoder v4: one wave per piece, two streaming passes, no cross-workgroup
// waits.  Included from packed_codec.hip (namespace cpk).
//
//   e4_size_kernel   each wave takes pieces from per-XCD tickets and walks
//                    its piece in 64-word steps (lane = word), carrying the
//                    run state in SGPRs from step to step: word class, run
//                    boundaries, the roles of PackedOutputStream.java:64-193
//                    per word, and the packed size of the piece;
//   e4_scan_*        exclusive scan of the sizes -> out_off[0..n];
//   e4_emit_kernel   the same walk again, now with the piece's output offset
//                    known: every word's packed string (tag, v_perm-compacted
//                    bytes, count) is OR-ed into a 2 KiB LDS ring at its byte
//                    position and complete 16-byte lines stream to memory.
//                    A head's count needs the end of its run, at most 256
//                    words on: the emit walk reads the size pass's boundary
//                    rows 4 steps ahead (rows and words one group of steps
//                    ahead of their use; the strings and their placement in
//                    encode_sp.hip's form: round 6, config-3 density -0.9 %)
// Traffic: U + (U + P) instead of U + P, in exchange for no barriers, no
// look-back and every wave independent (both passes are pure streams).

constexpr int kE4Waves = 4;
constexpr int kE4Threads = 64 * kE4Waves;
constexpr uint32_t kE4RingBytes = 2048;  // output ring per wave (<= 41 live lines)
// Each string is OR-ed from its first ring dword on without a wrap per
// dword: a string's last three dwords past the ring's end go to one overhang
// line, OR-ed into line 0 when that is stored (the ring holds at most 104
// unstored lines, so line 0's previous bytes are out by then).
constexpr uint32_t kE4Ov = 1u;                                    // overhang lines
constexpr uint32_t kE4RingStride = kE4RingBytes + 16 * kE4Ov;
constexpr uint32_t kE4oLut = 0;                                   // u64[256]
constexpr uint32_t kE4oRing = 2048;                               // u32[waves][512 (+ 164)]
constexpr uint32_t kE4Lds = kE4oRing + kE4Waves * kE4RingStride;  // 10 KiB (12.6 KiB with overhang)

// the size pass's row per 64-word step for the emit pass: run boundaries,
// literal-run members, heads (3 u64); at most 4 GiB of rows
constexpr uint64_t kE4RowBytes = 24;
constexpr uint64_t kE4MaxRows = (1ull << 32) / kE4RowBytes;

constexpr uint32_t kE4RingLines = kE4RingBytes / 16;
constexpr uint32_t kE4RingDw = kE4RingBytes / 4;

// nonzero-byte tag of a word (PackedOutputStream.java:64-117): bit i set iff
// byte i != 0.  SWAR: bit 7 of every byte of t = byte != 0, gathered by shifts.
#define E4_LD2(p) (*(p))
// the size pass's loads: nontemporal (U is read again only by the emit pass,
// long after; config-3 encode -2 %, r4AT_e4_size_nt_ab.log)
#define E4_SLD(p) ld_stream(p)

// lane l's 64-bit value, wave-uniform
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}

__device__ __forceinline__ uint32_t e4_tag(uint64_t v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  // bit 7 of each byte: the byte is nonzero (no carry crosses a byte); the
  // eight flags gathered by two u8 dot products with weights 2^k (9 VALU
  // instead of the 15 of shifts and ORs: round 5, config 2 encode -2.3 %,
  // config 4 -14 %)
  const uint32_t tl = (((lo & 0x7f7f7f7fu) + 0x7f7f7f7fu) | lo) & 0x80808080u;
  const uint32_t th = (((hi & 0x7f7f7f7fu) + 0x7f7f7f7fu) | hi) & 0x80808080u;
  return __builtin_amdgcn_udot4(th, 0x80402010u, __builtin_amdgcn_udot4(tl, 0x08040201u, 0u, false), false) >> 7;
}

// ring line r (OR its overhang line) / cleared
__device__ __forceinline__ uint4 e4_line(const uint32_t *ring, uint32_t r) {
  const uint4 *rl = reinterpret_cast<const uint4 *>(ring);
  uint4 v = rl[r];
  if (r < kE4Ov) {
    const uint4 o = rl[kE4RingLines + r];
    v.x |= o.x;
    v.y |= o.y;
    v.z |= o.z;
    v.w |= o.w;
  }
  return v;
}
__device__ __forceinline__ void e4_line_clear(uint32_t *ring, uint32_t r) {
  uint4 *rl = reinterpret_cast<uint4 *>(ring);
  rl[r] = make_uint4(0u, 0u, 0u, 0u);
  if (r < kE4Ov) rl[kE4RingLines + r] = make_uint4(0u, 0u, 0u, 0u);
}

// bytes [j0, j1) of global line L from the ring, then clears the ring line
__device__ __forceinline__ void e4_store_bytes(uint8_t *out, uint32_t *ring, uint64_t L, int j0,
                                               int j1, int lane) {
  const uint32_t r = (uint32_t)L & (kE4RingLines - 1);
  const uint4 val = e4_line(ring, r);
  if (lane >= j0 && lane < j1) {
    const uint32_t d = (lane & 8) ? ((lane & 4) ? val.w : val.z) : ((lane & 4) ? val.y : val.x);
    out[L * 16 + lane] = (uint8_t)(d >> (8 * (lane & 3)));
  }
  wave_lds_order();
  if (lane == 0) e4_line_clear(ring, r);
}

// stores the complete lines [fl, upto) of the ring; bytes below `lo` belong
// to the previous piece (only the piece's first line can hold them)
__device__ __forceinline__ void e4_flush(uint8_t *out, uint32_t *ring, uint64_t &fl, uint64_t upto,
                                         uint64_t lo, int lane) {
  if (fl >= upto) return;
  if (fl * 16 < lo) {
    e4_store_bytes(out, ring, fl, (int)(lo - fl * 16), 16, lane);
    ++fl;
  }
  for (uint64_t L0 = fl; L0 < upto; L0 += 64) {
    const uint64_t L = L0 + lane;
    if (L < upto) {
      const uint32_t r = (uint32_t)L & (kE4RingLines - 1);
      const uint4 val = e4_line(ring, r);
      e4_line_clear(ring, r);
      *reinterpret_cast<uint4 *>(out + L * 16) = val;
    }
  }
  fl = upto;
}

constexpr int kE4Wpe = 8;


#include "sp_roles.hip"  // SpSt, sp_roles: the run roles as mask algebra (shared with encode_sp.hip)


// ---- size pass: roles lane-parallel over a group of <= 64 steps ------------
// (the single pass's A2 form, encode_sp.hip sp_a2p, restated for a wave that
// walks one piece: lane j holds step j's masks; scalar helpers read them by
// readlane)
struct E4Grp {
  uint32_t zl, zh, dll, dlh, dl_, dh_;  // lane j: step j's Z / DL / D masks
};
__device__ __forceinline__ uint64_t e4g_z(const E4Grp &G, int j) { return sp_rl(G.zl, G.zh, j); }
__device__ __forceinline__ uint64_t e4g_dl(const E4Grp &G, int j) { return sp_rl(G.dll, G.dlh, j); }
__device__ __forceinline__ uint64_t e4g_d(const E4Grp &G, int j) { return sp_rl(G.dl_, G.dh_, j); }
// first D word at or after group position x (< lim), else lim
__device__ int e4g_first_d(const E4Grp &G, int cnt, int x, int lim) {
  if (x >= lim) return lim;
  int q = x >> 6;
  uint64_t m = e4g_d(G, q) & (~0ull << (x & 63));
  while (!m) {
    if (++q >= cnt) return lim;
    m = e4g_d(G, q);
  }
  return min(q * 64 + __builtin_ctzll(m), lim);
}
// the run state after the group's cnt steps (encode_sp.hip sp_state_at)
__device__ SpSt e4g_state_after(const E4Grp &G, int cnt, SpSt cst) {
  SpSt st = {0u, 0u, 0u};
  const uint64_t Zp = e4g_z(G, cnt - 1), DLp = e4g_dl(G, cnt - 1);
  if (Zp >> 63) {
    int q = cnt - 1;
    uint32_t zl = 0;
    uint64_t z = Zp;
    while (z == ~0ull) {
      zl += 64;
      if (--q < 0) break;
      z = e4g_z(G, q);
    }
    st.zl = zl + (q >= 0 ? (uint32_t)__builtin_clzll(~z) : cst.zl);
  }
  if (!(DLp >> 63)) return st;
  st.dlo = 1;
  int q = cnt - 1;
  uint64_t d = DLp;
  while (d == ~0ull) {
    if (--q < 0) break;
    d = e4g_dl(G, q);
  }
  const int P = 64 * cnt;
  int h;
  if (q >= 0 || !cst.dlo || !cst.hd) {
    const int start = q >= 0 ? 64 * q + 64 - __builtin_clzll(~d) : 0;
    h = e4g_first_d(G, cnt, start, P);
    if (h >= P) return st;
  } else {
    h = -(int)cst.hd;
  }
  for (;;) {
    const int h2 = e4g_first_d(G, cnt, max(h + 256, 0), P);
    if (h2 >= P) break;
    h = h2;
  }
  st.hd = (uint32_t)min(P - h, 256);
  return st;
}
__device__ __forceinline__ uint32_t e4g_from(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
// the group's bytes beyond its words' nonzero bytes (tags, counts, the zero
// byte of literal-run members).  Returns the steps it leaves out: those a D/L
// stretch enters longer than 192 words (its heads may chain within the step;
// the caller takes them one at a time, sp_roles on the state there)
__device__ __forceinline__ uint64_t e4g_bytes_par(const E4Grp &G, int cnt, uint32_t wrem, SpSt st, int lane,
                                                 uint64_t &bytes, uint64_t &memo, uint64_t &hco) {
  const bool act = lane < cnt;
  const uint64_t Z = act ? ((uint64_t)G.zl | ((uint64_t)G.zh << 32)) : 0ull;
  const uint64_t DL = act ? ((uint64_t)G.dll | ((uint64_t)G.dlh << 32)) : 0ull;
  const uint64_t D = act ? ((uint64_t)G.dl_ | ((uint64_t)G.dh_ << 32)) : 0ull;
  const uint64_t below = (1ull << lane) - 1;
  const uint32_t dlo = (uint32_t)wave_shr1((int)(uint32_t)(DL >> 63), (int)st.dlo);
  const uint32_t topdl = DL == ~0ull ? 64u : (uint32_t)__builtin_clzll(~DL);
  const uint64_t notall = __ballot(!act || DL != ~0ull);
  const uint64_t kdm = notall & below;
  const int kd = kdm ? 63 - __builtin_clzll(kdm) : -1;
  const uint32_t topdl_k = e4g_from(topdl, kd < 0 ? 0 : kd);
  const uint32_t len = kd >= 0 ? topdl_k + 64u * (uint32_t)(lane - 1 - kd)
                               : (st.dlo ? st.hd : 0u) + 64u * (uint32_t)lane;
  const bool cont = act && dlo && (DL & 1);
  const bool longc = cont && len > 192;
  const uint64_t lng = __ballot(longc);
  const uint64_t anyD = __ballot(act && D != 0);
  const bool topd = topdl > 0 && (D >> (64 - topdl)) != 0;
  const uint64_t TD = __ballot(act && topd);
  const uint64_t btw = anyD & below & (kd >= 0 ? (~0ull << kd) << 1 : ~0ull);
  const bool head = btw != 0 || (kd >= 0 ? ((TD >> kd) & 1) != 0 : (st.dlo && st.hd));
  const uint64_t cin = (cont && head) ? 1ull : 0ull;
  const uint64_t A = ((D << 1) | cin) & DL;
  const uint64_t C = (DL + A) ^ DL ^ A;
  const uint64_t Mem = DL & (A | C);
  const uint32_t zc = (uint32_t)wave_shr1((int)(uint32_t)(Z >> 63), st.zl ? 1 : 0);
  uint64_t Zh = Z & ~((Z << 1) | zc);
  {
    const uint32_t topz = Z == ~0ull ? 64u : (uint32_t)__builtin_clzll(~Z);
    const uint64_t kzm = __ballot(!act || Z != ~0ull) & below;
    const int kz = kzm ? 63 - __builtin_clzll(kzm) : -1;
    const uint32_t topz_k = e4g_from(topz, kz < 0 ? 0 : kz);
    const uint32_t zl = kz >= 0 ? topz_k + 64u * (uint32_t)(lane - 1 - kz) : st.zl + 64u * (uint32_t)lane;
    const uint32_t j0 = (256u - (zl & 255u)) & 255u;
    if (__ballot(act && zc && (Z & 1) && j0 < 64)) {
      const uint64_t pre = j0 >= 63 ? ~0ull : ((2ull << j0) - 1);
      if (act && zc && (Z & 1) && j0 < 64 && (Z & pre) == pre) Zh |= 1ull << j0;
    }
  }
  const uint32_t vr = act ? wrem - 64u * (uint32_t)lane : 0u;
  const uint64_t V = vr >= 64 ? ~0ull : ((1ull << vr) - 1);
  const uint64_t HC = Zh | (D & ~Mem), ZO = (Z & ~Zh) | ~V;
  const uint32_t b = (act && !longc) ? (uint32_t)(__builtin_popcountll(~ZO & ~Mem) +
                                                   __builtin_popcountll(Mem & ~D) + __builtin_popcountll(HC))
                                    : 0u;
  bytes += (uint32_t)__builtin_amdgcn_readlane(wave_incl_add((int)b), 63);
  memo = Mem;
  hco = HC;
  return lng;
}

// next piece for this wave from the per-XCD counters (as the decoder)
__device__ __forceinline__ uint32_t e4_next_piece(uint32_t *ticket, int &xq, int &dry, uint32_t n) {
  uint32_t seg;
  for (;;) {
    seg = take_ticket(ticket, xq);
    if (seg < n || ++dry >= 8) break;
    xq = (xq + 1) & 7;
  }
  return seg;
}

// ---- pass 1: packed size of every piece --------------------------------------
__global__ __launch_bounds__(kE4Threads, kE4Wpe) void e4_size_kernel(
    const uint64_t *__restrict__ in, const uint64_t *__restrict__ swo, uint32_t n,
    uint64_t *__restrict__ sizes, uint32_t *ticket, uint64_t hint, uint32_t *err,
    uint64_t *__restrict__ bvbuf, uint64_t stride, const uint32_t *skip, const uint32_t *order) {
  if (skip && __builtin_amdgcn_readfirstlane(*skip)) return;  // (the single pass took the batch)
  const int lane = lane_id();
  int xq = xcc_id(), dry = 0;
  for (;;) {
    const uint32_t tk = e4_next_piece(ticket, xq, dry, n);
    if (tk >= n) break;
    // (order: the pieces largest first)
    const uint32_t seg = order ? (uint32_t)__builtin_amdgcn_readfirstlane((int)order[tk]) : tk;
    const uint64_t w0 = swo[seg];
    const uint64_t W = swo[seg + 1] - w0;
    if (((hint && W > hint) || W >= (1ull << 31)) && lane == 0) atomicOr(err, 1u);
    if (W == 0) {  // an empty piece: no bytes (and no loads: it may sit at the end)
      if (lane == 0) sizes[seg] = 0;
      continue;
    }
    const uint64_t *src = in + w0;
    // this piece's step rows in bvbuf: `stride` rows per piece when the
    // size hint bounds them, else packed by word offset (disjoint: a piece
    // adds at most one partial step)
    uint64_t *bvp = bvbuf + 3 * (stride ? (uint64_t)seg * stride : (w0 - swo[0]) / 64 + seg);
    const uint64_t rows = stride ? stride : ~0ull;  // (a piece over the hint: error, no rows)
    // run state entering each group of 64 steps (the single pass's SpSt),
    // the previous step's last-word classes for the boundaries
    SpSt st = {0u, 0u, 0u};
    uint32_t zprev = 0, dlprev = 0;
    uint64_t bytes = 0;
    E4Grp G = {0u, 0u, 0u, 0u, 0u, 0u};
    uint32_t acc = 0;
    // (32-bit step / word indices: a piece is at most 2^31 words, Serialize
    // limits segments to 2^29 - 1, Serialize.java:45-53)
    const uint32_t W32 = (uint32_t)W, nsteps = (W32 + 63) >> 6;
    // software pipeline: the next kE4Pf steps' loads are in flight while
    // these are classified
    // steps of loads in flight ahead of the size pass's classification (8:
    // config-3 messages' e4 encode 7.06 -> 7.00 ms, config 2 6.39 -> 6.29
    // against 4, r4K_ab.log; 64 VGPRs, no spill at 8 workgroups per CU)
    // (4 and 16 measured neutral / +15 %, r4AL_ab.log)
    constexpr int PF = 8;
    uint64_t v[PF], vn[PF];
    // loads clamped to the piece's last word, not predicated (no exec-mask
    // branches around them); words past the end are masked by `valid`
    const uint32_t kl = W32 - 1;
#pragma unroll
    for (int j = 0; j < PF; ++j) v[j] = E4_SLD(src + min(((uint32_t)j << 6) + lane, kl));
    for (uint32_t s0 = 0; s0 < nsteps; s0 += PF) {
#pragma unroll
      for (int j = 0; j < PF; ++j) vn[j] = E4_SLD(src + min(((s0 + PF + j) << 6) + lane, kl));
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const uint32_t k = ((s0 + j) << 6) + lane;
        const bool valid = k < W32;
        if (s0 + j < nsteps) {
          // per word its tag and nonzero bytes; per step, into lane
          // (s0 + j) & 63, the zero-word / <= 1 zero byte / tag-0xff masks
          const uint32_t m = valid ? e4_tag(v[j]) : 0u;
          const uint32_t pc = (uint32_t)__builtin_popcount(m);
          acc += pc;
          const uint64_t Z = __ballot(valid && m == 0), DL = __ballot(pc >= 7), D = __ballot(m == 0xffu);
          const int jj = (int)((s0 + j) & 63);
          G.zl = sp_wl(G.zl, (uint32_t)Z, jj);
          G.zh = sp_wl(G.zh, (uint32_t)(Z >> 32), jj);
          G.dll = sp_wl(G.dll, (uint32_t)DL, jj);
          G.dlh = sp_wl(G.dlh, (uint32_t)(DL >> 32), jj);
          G.dl_ = sp_wl(G.dl_, (uint32_t)D, jj);
          G.dh_ = sp_wl(G.dh_, (uint32_t)(D >> 32), jj);
        }
      }
      if (((s0 + PF) & 63) == 0 || s0 + PF >= nsteps) {
        // a group of 64 steps (or the piece's last): its roles and bytes
        // lane-parallel, its boundary rows, the state it leaves
        const uint32_t g0 = s0 & ~63u;
        const int cnt = (int)min(64u, nsteps - g0);
        const uint32_t wrem = W32 - 64u * g0;
        // lane j: step j's literal-run members and heads (the emit pass's roles)
        uint64_t MemL = 0, HCL = 0;
        uint64_t lng = e4g_bytes_par(G, cnt, wrem, st, lane, bytes, MemL, HCL);
        // steps a long D/L stretch enters (~15 % of config-3 groups have
        // one or two): the sequential roles on the run state there
        while (lng) {
          const int j = __builtin_ctzll(lng);
          lng &= lng - 1;
          SpSt sj = j ? e4g_state_after(G, j, st) : st;
          const uint64_t Z = e4g_z(G, j), DL = e4g_dl(G, j), D = e4g_d(G, j);
          const uint32_t vr = wrem - 64u * (uint32_t)j;
          const uint64_t V = vr >= 64 ? ~0ull : ((1ull << vr) - 1);
          uint64_t Zh, Mem;
          sp_roles(Z, DL, D, sj, Zh, Mem);
          const uint64_t HC = Zh | (D & ~Mem), ZO = (Z & ~Zh) | ~V;
          bytes += (uint64_t)(__builtin_popcountll(~ZO & ~Mem) + __builtin_popcountll(Mem & ~D) +
                              __builtin_popcountll(HC));
          MemL = lane == j ? Mem : MemL;
          HCL = lane == j ? HC : HCL;
        }
        st = e4g_state_after(G, cnt, st);
        // run boundaries for the emit pass (e4_classify's BV): past the
        // piece's end, every M word, each zero run / D/L stretch's first word
        {
          const bool act = lane < cnt;
          const uint64_t Z = act ? ((uint64_t)G.zl | ((uint64_t)G.zh << 32)) : 0ull;
          const uint64_t DL = act ? ((uint64_t)G.dll | ((uint64_t)G.dlh << 32)) : 0ull;
          const uint32_t vr = act ? wrem - 64u * (uint32_t)lane : 0u;
          const uint64_t V = vr >= 64 ? ~0ull : ((1ull << vr) - 1);
          const uint64_t zp = (uint32_t)wave_shr1((int)(uint32_t)(Z >> 63), (int)zprev);
          const uint64_t dp = (uint32_t)wave_shr1((int)(uint32_t)(DL >> 63), (int)dlprev);
          const uint64_t BV = ~V | (V & ~Z & ~DL) | (Z & ~((Z << 1) | zp)) | (DL & ~((DL << 1) | dp));
          if (act && g0 + lane < rows) {
            uint64_t *row = bvp + 3ull * (g0 + lane);
            row[0] = BV;
            row[1] = MemL;
            row[2] = HCL;
          }
          zprev = (uint32_t)(e4g_z(G, cnt - 1) >> 63);
          dlprev = (uint32_t)(e4g_dl(G, cnt - 1) >> 63);
        }
      }
#pragma unroll
      for (int j = 0; j < PF; ++j) v[j] = vn[j];
    }
    // wave sum in two 16-bit halves (a piece's packed size may pass 2^31)
    const uint32_t thi = (uint32_t)wave_incl_add((int)(acc >> 16));
    const uint32_t tlo = (uint32_t)wave_incl_add((int)(acc & 0xffffu));
    if (lane == 63) sizes[seg] = ((uint64_t)thi << 16) + tlo + bytes;
  }
}

// ---- exclusive scan of the sizes -> out_off[0..n] ------------------------------
constexpr int kE4ScanThreads = 1024;
constexpr int kE4ScanPer = 4;  // sizes per thread per block
constexpr int kE4ScanBlock = kE4ScanThreads * kE4ScanPer;

__device__ __forceinline__ uint64_t e4_block_scan(uint64_t x, uint64_t *sh, uint64_t &total) {
  // inclusive scan over the block's 1024 threads (wave scans + one LDS pass)
  const int lane = lane_id(), w = wave_id();
  uint64_t v = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(v, d, 64);
    if (lane >= d) v += y;
  }
  if (lane == 63) sh[w] = v;
  __syncthreads();
  if (w == 0) {
    uint64_t t = lane < kE4ScanThreads / 64 ? sh[lane] : 0;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const uint64_t y = __shfl_up(t, d, 64);
      if (lane >= d) t += y;
    }
    if (lane < kE4ScanThreads / 64) sh[16 + lane] = t;
  }
  __syncthreads();
  total = sh[16 + kE4ScanThreads / 64 - 1];
  const uint64_t r = v + (w ? sh[16 + w - 1] : 0);
  __syncthreads();
  return r;
}

// block sums of kE4ScanBlock sizes each
__global__ __launch_bounds__(kE4ScanThreads) void e4_scan_reduce(const uint64_t *__restrict__ sizes,
                                                                 uint32_t n, uint64_t *bsum) {
  __shared__ uint64_t sh[32];
  const uint64_t b0 = (uint64_t)blockIdx.x * kE4ScanBlock;
  uint64_t x = 0;
#pragma unroll
  for (int j = 0; j < kE4ScanPer; ++j) {
    const uint64_t i = b0 + (uint64_t)j * kE4ScanThreads + threadIdx.x;
    x += i < n ? sizes[i] : 0;
  }
  uint64_t total;
  e4_block_scan(x, sh, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// exclusive scan of the block sums in place (one block; nb <= 1024 * 16)
__global__ __launch_bounds__(kE4ScanThreads) void e4_scan_top(uint64_t *bsum, uint32_t nb) {
  __shared__ uint64_t sh[32];
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += kE4ScanThreads) {
    const uint32_t i = b0 + threadIdx.x;
    const uint64_t x = i < nb ? bsum[i] : 0;
    uint64_t total;
    const uint64_t inc = e4_block_scan(x, sh, total);
    if (i < nb) bsum[i] = carry + inc - x;
    carry += total;
  }
}

// out_off[i] = exclusive prefix of sizes, out_off[n] = total
__global__ __launch_bounds__(kE4ScanThreads) void e4_scan_down(const uint64_t *__restrict__ sizes,
                                                               uint32_t n, const uint64_t *bsum,
                                                               uint64_t *__restrict__ out_off) {
  __shared__ uint64_t sh[32];
  // thread t owns sizes b0 + t*kE4ScanPer .. +kE4ScanPer-1 (contiguous)
  const uint64_t b0 = (uint64_t)blockIdx.x * kE4ScanBlock;
  const uint64_t i0 = b0 + (uint64_t)threadIdx.x * kE4ScanPer;
  uint64_t x[kE4ScanPer], s = 0;
#pragma unroll
  for (int j = 0; j < kE4ScanPer; ++j) {
    x[j] = i0 + j < n ? sizes[i0 + j] : 0;
    s += x[j];
  }
  uint64_t total;
  const uint64_t inc = e4_block_scan(s, sh, total);
  uint64_t o = bsum[blockIdx.x] + inc - s;
#pragma unroll
  for (int j = 0; j < kE4ScanPer; ++j) {
    if (i0 + j < n) out_off[i0 + j] = o;
    o += x[j];
    if (i0 + j + 1 == n) out_off[n] = o;
  }
}

// ---- pass 2: the packed bytes ----------------------------------------------------
// One step of the emit walk.  bv0..bv4: the run boundaries of this step and
// the next four (for the counts of heads whose run reaches past this step);
// mem / hc: this step's literal-run members and heads, all three from the
// size pass's rows.
__device__ __forceinline__ void e4_emit_step(uint64_t word, bool valid, uint64_t bv0,
                                             uint64_t bv1, uint64_t bv2, uint64_t bv3,
                                             uint64_t bv4, uint64_t mem, uint64_t hc, int lane,
                                             const uint64_t *lut, uint32_t *ring, uint8_t *out,
                                             uint64_t &rpos, uint64_t &fl, uint64_t obase) {
  // (encode_sp.hip's string form: per-lane selects on the rows' scalar
  // masks instead of per-lane mask bits and word classes)
  const uint32_t m = valid ? e4_tag(word) : 0u;  // (a word past the piece: no bytes)
  const uint64_t ZW = __ballot(m == 0);
  const uint32_t lo = (uint32_t)word, hi = (uint32_t)(word >> 32);
  const uint64_t sel = lut[m];
  const uint32_t c0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
  const uint32_t c1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
  uint32_t cz = 0, cd = 0;
  if (hc) {
    // a head's count: words to its run's end, at most 255 (:123-131,
    // :143-164) -- the next boundary after the lane in this step, else X
    // words past the step's end (v_ffbl: 0xffffffff for none)
    const uint32_t X = bv1 ? (uint32_t)__builtin_ctzll(bv1)
                           : bv2 ? 64u + (uint32_t)__builtin_ctzll(bv2)
                                 : bv3 ? 128u + (uint32_t)__builtin_ctzll(bv3)
                                       : bv4 ? 192u + (uint32_t)__builtin_ctzll(bv4) : 256u;
    const uint64_t e = (bv0 >> lane) >> 1;
    const uint32_t z_lo = sp_ffbl((uint32_t)e);
    const uint32_t z_hi = sp_ffbl((uint32_t)(e >> 32)) | 32u;
    const uint32_t tt = min(min(z_lo, z_hi), min((uint32_t)(63 - lane) + X, 255u));
    cz = sp_sel(0u, tt, hc & ZW);   // zero-run heads: the count after the 0x00 tag
    cd = sp_sel(0u, tt, hc & ~ZW);  // 0xFF heads: the count after the 8 bytes
  }
  const uint32_t c0p = c0 | cz;
  uint32_t s0 = m | (c0p << 8);
  uint32_t s1 = __builtin_amdgcn_alignbyte(c1, c0p, 3);
  uint32_t s2 = __builtin_amdgcn_alignbyte(cd, c1, 3);
  s0 = sp_sel(s0, lo, mem);
  s1 = sp_sel(s1, hi, mem);
  s2 = sp_sel(s2, 0u, mem);
  uint32_t nb = (uint32_t)__builtin_popcount(m) + sp_sel(1u, 2u, hc);
  nb = sp_sel(nb, 8u, mem);
  nb = sp_sel(nb, 0u, ZW & ~hc);  // a zero word that is no head, or past the piece
  const int incl = wave_incl_add((int)nb);
  const uint32_t o = (uint32_t)incl - nb;
  const uint32_t stot = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
  if (stot) {
    // OR the string into the ring at its output position (the ring's lines
    // are zero until written; bytes past a string are zero)
    // (the string shifted onto its byte by one v_perm per dword, selector
    // bytes [4 - b, 8 - b) of (s_k : s_k-1); from its first ring dword on,
    // past the ring's end into the overhang line)
    const uint32_t p = (uint32_t)rpos + o;
    const uint32_t b = p & 3;
    const uint32_t psel = 0x07060504u - __builtin_amdgcn_perm(0u, b, 0u);  // (b in every byte)
    const uint32_t d0 = __builtin_amdgcn_perm(s0, 0u, psel), d1 = __builtin_amdgcn_perm(s1, s0, psel);
    const uint32_t d2 = __builtin_amdgcn_perm(s2, s1, psel), d3 = __builtin_amdgcn_perm(0u, s2, psel);
    uint32_t *rp = ring + ((p >> 2) & (kE4RingDw - 1));
    if (nb) {
      atomicOr(rp, d0);
      atomicOr(rp + 1, d1);
      atomicOr(rp + 2, d2);
      atomicOr(rp + 3, d3);
    }
    rpos += stot;
    // complete lines go out 64 at a time (one full-wave store: flushing
    // every step's few lines cost 8 % more time); the ring holds at most
    // 63 + 41 lines
    if ((uint32_t)(rpos >> 4) - (uint32_t)fl >= 64u) {  // (32-bit: a 64-bit < is VALU work)
      wave_lds_order();
      e4_flush(out, ring, fl, fl + 64, obase, lane);
    }
  }
}

__global__ __launch_bounds__(kE4Threads, kE4Wpe) void e4_emit_kernel(
    const uint64_t *__restrict__ in, const uint64_t *__restrict__ swo, uint32_t n,
    const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out, uint32_t *ticket,
    const uint64_t *__restrict__ bvbuf, uint64_t stride, const uint32_t *skip,
    const uint64_t *__restrict__ sizes, uint64_t ocap, uint32_t *err, const uint32_t *order) {
  if (skip && __builtin_amdgcn_readfirstlane(*skip)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint64_t *lut = reinterpret_cast<const uint64_t *>(smem + kE4oLut);
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  uint32_t *ring = reinterpret_cast<uint32_t *>(smem + kE4oRing + w * kE4RingStride);
  fill_luts(reinterpret_cast<uint64_t *>(smem + kE4oLut), false);
  for (uint32_t i = lane; i < kE4RingLines + kE4Ov; i += 64)
    reinterpret_cast<uint4 *>(ring)[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  int xq = xcc_id(), dry = 0;
  for (;;) {
    const uint32_t tk = e4_next_piece(ticket, xq, dry, n);
    if (tk >= n) break;
    const uint32_t seg = order ? (uint32_t)__builtin_amdgcn_readfirstlane((int)order[tk]) : tk;
    const uint64_t w0 = swo[seg];
    const uint64_t W = swo[seg + 1] - w0;
    if (W == 0) continue;  // no bytes; no loads (it may sit at the end of the input)
    const uint64_t *src = in + w0;
    const uint64_t obase = out_off[seg];
    // a piece whose bytes would pass the caller's capacity is not written
    // (ArrayOutputStream.java:40-42 refuses such a write); reported
    if (obase + sizes[seg] > ocap) {
      if (lane == 0) atomicOr(err, kErrCap);
      continue;
    }
    uint64_t rpos = obase, fl = obase >> 4;
    // the boundaries of every step come from the size pass (bvbuf); past
    // the piece every word is a boundary.  Words: this group of four steps
    // and the next one's loads in flight.
    const uint32_t W32 = (uint32_t)W, nsteps = (W32 + 63) >> 6;  // (pieces < 2^31 words)
    if (stride && nsteps > stride) continue;  // over the size hint: reported, output undefined
    const uint64_t *bvp = bvbuf + 3 * (stride ? (uint64_t)seg * stride : (w0 - swo[0]) / 64 + seg);
    // steps of loads in flight ahead of the emit (2 and 8 measured 1-2 %
    // slower, r4AL_ab.log)
    constexpr int EPF = 4;
    uint64_t vc[EPF], vl[EPF];
    const uint32_t kl = W32 - 1;  // loads clamped, not predicated
#pragma unroll
    for (int j = 0; j < EPF; ++j) vc[j] = E4_LD2(src + min(((uint32_t)j << 6) + lane, kl));
    // the rows of a group's steps and the next four (3 x (EPF + 4) u64, one
    // per lane) by one vector load a group ahead, like the words: the
    // scalar loads of them at the group's start left their HBM latency
    // exposed once per group
    static_assert(3 * (EPF + 4) <= 64, "a group's rows fit the lanes");
    auto ldrows = [&](uint32_t g0) __attribute__((always_inline)) -> uint64_t {
      const uint32_t k = (uint32_t)lane / 3u, f = (uint32_t)lane - 3u * k;
      if (lane >= 3 * (EPF + 4)) return 0ull;
      return g0 + k < nsteps ? bvp[3 * g0 + (uint32_t)lane] : (f == 0 ? ~0ull : 0ull);
    };
    uint64_t rw = ldrows(0), rwn;
    for (uint32_t s0 = 0; s0 < nsteps; s0 += EPF) {
#pragma unroll
      for (int j = 0; j < EPF; ++j) vl[j] = E4_LD2(src + min(((s0 + EPF + j) << 6) + lane, kl));
      uint64_t bv[EPF + 4], mem[EPF], hc[EPF];
      rwn = ldrows(s0 + EPF);
#pragma unroll
      for (int j = 0; j < EPF + 4; ++j) bv[j] = rl64(rw, 3 * j);
#pragma unroll
      for (int j = 0; j < EPF; ++j) {
        mem[j] = rl64(rw, 3 * j + 1);
        hc[j] = rl64(rw, 3 * j + 2);
      }
#pragma unroll
      for (int j = 0; j < EPF; ++j) {
        if (s0 + j < nsteps)
          e4_emit_step(vc[j], ((s0 + j) << 6) + lane < W32, bv[j], bv[j + 1], bv[j + 2], bv[j + 3],
                       bv[j + 4], mem[j], hc[j], lane, lut, ring, out, rpos, fl, obase);
      }
#pragma unroll
      for (int j = 0; j < EPF; ++j) vc[j] = vl[j];
      rw = rwn;
    }
    wave_lds_order();
    e4_flush(out, ring, fl, rpos >> 4, obase, lane);
    // the piece's last, partial line
    if (rpos > fl * 16) {
      const int j0 = (int)((obase > fl * 16 ? obase : fl * 16) - fl * 16);
      e4_store_bytes(out, ring, fl, j0, (int)(rpos - fl * 16), lane);
    }
  }
}

// ---- encoder choice on the device (cpk_encode_batch, no host sync) --------
// min / max piece words of the batch (mm[0] preset to ~0, mm[1] to 0)
__global__ __launch_bounds__(256) void e4_minmax_kernel(const uint64_t *__restrict__ swo, uint32_t n,
                                                        uint32_t *mm, const uint64_t *__restrict__ in) {
  // (and one word per thread, one in each of G equal stretches of the
  // batch at a hashed position inside it -- not at a fixed phase, which
  // would alias with the pieces' starts: zero words counted into mm[3] for
  // the single pass's sparse form, e4_gate_kernel)
  {
    const uint64_t a = swo[0], T = swo[n] - a;
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x, G = (uint64_t)gridDim.x * 256;
    const uint64_t st = T / G, h = (uint32_t)(g * 2654435761u) ^ ((uint32_t)g >> 7);
    const uint64_t x = (in && T) ? in[a + g * T / G + (st ? h % st : 0)] : 1ull;
    const bool z = in && T && x == 0;
    const uint64_t zb = __ballot(z);
    if ((threadIdx.x & 63) == 0 && zb) atomicAdd(&mm[3], (uint32_t)__builtin_popcountll(zb));
    // (and the sampled words' packed bytes, tag + nonzero bytes, into mm[7])
    const int pb = wave_incl_add((in && T && x) ? 1 + __builtin_popcount(e4_tag(x)) : 0);
    if ((threadIdx.x & 63) == 63 && pb) atomicAdd(&mm[7], (uint32_t)pb);
  }
  // grid-stride over the pieces, one atomic pair per workgroup (one per
  // wave put 8 K same-address atomics in line at 1 Mi pieces: 97 us)
  __shared__ uint32_t red[2][4];
  uint32_t lo = 0xffffffffu, hi = 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint64_t w = swo[i + 1] - swo[i];
    const uint32_t w32 = w > 0xffffffffull ? 0xffffffffu : (uint32_t)w;
    lo = min(lo, w32);
    hi = max(hi, w32);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    lo = min(lo, (uint32_t)__shfl_xor((int)lo, d, 64));
    hi = max(hi, (uint32_t)__shfl_xor((int)hi, d, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = lo;
    red[1][threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) {
      lo = min(lo, red[0][k]);
      hi = max(hi, red[1][k]);
    }
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}
// like-sized pieces (the largest at most twice the smallest) of 4096 words
// or more: the single pass (measured crossover, 1 GiB batches, config 2 / 3:
// 2 Ki-word pieces 1.07 / 1.22 ms against the two passes' 0.87 / 0.89, 4 Ki
// words 0.69 / 0.82 against 0.85 / 0.87) (its ticket left at 0, the two-pass kernels told
// to skip, tickets[kTkGate + 2]); else the reverse (the single pass's
// ordered ticket exhausted)
// Among single-pass batches, those whose sampled words are at least 85 %
// zero take its sparse form (cpk_sparse: tickets[kTkGate + 6] = 1; config 4
// encode -7 %, config 2 +36 %).
// Dense batches (the sampled words' tags and nonzero bytes at least
// CPK_GATE_DENSE_PCT % of their bytes) take the two passes instead: there a
// wave's output overflows the single pass's ring and waits for its offset,
// while the two passes stream at ~5 TB/s.  Measured (1 Mi pieces of 8192
// words, profiles/r5q_density_sweep.log): config-3 density (sampled ~106 %)
// two passes 41.0 ms against the single pass's 51.4 (47.1 with the round-5
// flush); at ~78 % and below the single pass is ahead (37.0 / 38.2 ms, 31.3 /
// 36.5 at 56 %).
#ifndef CPK_GATE_DENSE_PCT
#define CPK_GATE_DENSE_PCT 90
#endif
// Batches with one piece far larger than the rest (a piece of over one
// 8192-word unit and at least 1/2048 of the batch's words: e.g. a single
// message's segments, DefaultAllocator doubling them) take the single pass
// too: the two passes give a piece one wave, which then runs alone long
// after the chip has finished the rest (a 4 MiB segment: ~5 ms per write,
// profiles/r6b_pbb.log), where the single pass splits it into units.  (At
// 2048 the single pass's cost on mixed sizes, ~2.4x the two passes' per
// word, equals one wave's time on the piece at ~5,000x less than the chip's
// rate.)
__global__ void e4_gate_kernel(uint32_t *tickets, uint32_t samples, uint32_t force, const uint64_t *swo,
                               uint32_t n) {
  const uint32_t lo = tickets[kTkGate], hi = tickets[kTkGate + 1];
  const uint64_t total = swo[n] - swo[0];
  const bool big = hi > 8192u && (uint64_t)hi * 2048u >= total;
  const bool like = (lo >= 4096u && 2u * lo >= hi) || big;
  const bool sparse = like && (force ? force == 2u : (uint64_t)tickets[kTkGate + 3] * 100u >= (uint64_t)samples * 85u);
  const bool dense = like && !big && !sparse && !force &&
                     (uint64_t)tickets[kTkGate + 7] * 100u >= (uint64_t)samples * 8u * CPK_GATE_DENSE_PCT;
  const bool sp = like && !dense;
  if (threadIdx.x == 0) {
    tickets[kTkGate + 6] = sparse ? 1u : 0u;
    tickets[kTkGate + 2] = sp ? 1u : 0u;
    tickets[kTkPlan] = sp ? 0u : 0x7fffffffu;
  }
}

