// encode_sp.hip -- single-pass encoder (the default).  Included from
// packed_codec.hip (namespace cpk); uses encode_v4.hip's e4_tag.
//
// One 256-thread workgroup per chunk of a piece (a unit, below), units taken
// in order from a ticket, the chunk held in VGPRs: wave w owns the 64-word
// steps [32w, 32w + 32) of the 8192-word chunk, lane = word.  Per unit:
//   A1  load the wave's steps (32 x 8 B per lane, all in flight); per word the
//       nonzero-byte tag m (PackedOutputStream.java:64-117; kept packed four
//       per VGPR); per step the Z / DL / D ballots (zero word, <= 1 zero
//       byte, tag 0xff), stashed lane-per-step and copied to LDS for the
//       other waves;
//   A2  the roles PackedOutputStream.write gives each word, per step, from
//       mask arithmetic and a carried state (scalar ALU): zero-run heads
//       (:119-131), literal-run members (:133-193: a carry-add smears each
//       0xFF head over the rest of its D/L stretch), 0xFF heads, run ends.
//       Each wave recomputes the state entering its first step from the
//       earlier steps' masks.  The packed bytes of the wave follow from
//       popcounts.  tools/step_model.py is this algebra in Python, checked
//       against the oracle (tests/test_step_model.py);
//   look-back  the unit's size is published and its offset found by a
//       decoupled look-back over the units before it (epoch-tagged 8-byte
//       status words);
//   B   each word's string (tag + v_perm-compacted bytes + count, or the 8
//       bytes of a literal-run member) OR-ed into a per-wave LDS ring at its
//       offset from a wave scan; complete 16-byte lines stream out.
// Work is ticketed per chunk of 8192 words ("unit"): a piece over one chunk
// is several units, each emitting its own bytes, the run state handed from
// chunk to chunk (the state a chunk leaves is published for the next);
// every unit is read once: traffic U + P for any mix of piece sizes.

#ifndef CPK_SP_WAVES
#define CPK_SP_WAVES 4
#endif
constexpr int kSpWaves = CPK_SP_WAVES;
constexpr int kSpThreads = 64 * kSpWaves;
constexpr int kSpWS = 128 / kSpWaves;          // steps per wave
constexpr int kSpCS = kSpWaves * kSpWS;        // steps per chunk (8192 words)
#ifndef CPK_SP_RELOAD
#define CPK_SP_RELOAD 0  // B reads the words again (L2) instead of keeping them in VGPRs from A1
#endif
#ifndef CPK_SP_RING
#define CPK_SP_RING 8192
#endif
constexpr uint32_t kSpRing = CPK_SP_RING;      // output ring per wave (bytes)
constexpr uint32_t kSpRingLines = kSpRing / 16;
constexpr uint32_t kSpRing4 = kSpRing / 4;       // (dwords)
static_assert(kSpRing % 16 == 0, "whole lines");
// ring line of relative line i (the dense form's 11 KiB ring is no power of two)
__device__ __forceinline__ uint32_t sp_rline(uint32_t i) {
  return (kSpRingLines & (kSpRingLines - 1)) == 0 ? (i & (kSpRingLines - 1)) : (i % kSpRingLines);
}
// overhang lines past the ring's end: a step's strings are laid out from the
// ring position of its first byte without wrapping, so up to a step's 640
// bytes + a string's spill land past the end (41 lines; the reader ORs line
// r < 41 with overhang line r).  Round 5: no per-string wrap (config 2
// encode -0.6 %, config 4 -1.8 %)
constexpr uint32_t kSpOvLines = 41;
constexpr uint32_t kSpRingStride = kSpRing + 16 * kSpOvLines;
constexpr uint32_t kSpoLut = 0;                                      // u64[256]
constexpr uint32_t kSpoMsk = 2048;                                   // u64[kSpCS][3]
constexpr uint32_t kSpoRing = kSpoMsk + kSpCS * 24;                  // per wave
constexpr uint32_t kSpoScr = kSpoRing + kSpWaves * kSpRingStride;    // u64[32]
constexpr uint32_t kSpLds = kSpoScr + 32 * 8;  // 53,056 B (dense form, 11 KiB rings), 24,384 B (sparse form)
static_assert(kSpWaves <= 16 && kSpWS >= 4 && kSpWS <= 32 && kSpWS % 4 == 0, "wave count");
static_assert(kSpoRing % 16 == 0 && kSpoScr % 16 == 0, "LDS alignment");
// scratch words: [0] ticket, [16..16 + waves) wave bytes, [5] piece offset,
// [6..9] chunk exit state (two parities x {zl, dlo | hd << 1}), [11] the piece
// (+ 1) whose offset [5] holds
// Steps are scheduled one at a time: hoisting later steps' LUT reads and
// lane reads ahead would keep them all live at once (VGPR spills).
#define CPK_SP_STEP_FENCE() __builtin_amdgcn_sched_barrier(0)
#ifndef CPK_SP_WPE
#define CPK_SP_WPE 3  // waves per SIMD the registers must allow (3 workgroups per CU)
#endif
constexpr int kSpWpe = CPK_SP_WPE;  // workgroups per CU (the grid: kSpWpe x CUs)
static_assert(kSpLds * kSpWpe <= 160u * 1024u, "the workgroups per CU must fit its LDS");

// status word per piece: [63:62] flag (1 aggregate, 2 inclusive prefix),
// [61:46] launch epoch, [45:0] value (a relaxed 8-byte agent-scope granule:
// the data is the flag, cdna_hip_programming.md Guideline 16 form R2)
constexpr uint64_t kSpValMask = (1ull << 46) - 1;
__device__ __forceinline__ uint64_t sp_word(uint32_t ep, uint32_t flag, uint64_t v) {
  return ((uint64_t)flag << 62) | ((uint64_t)(ep & 0xffffu) << 46) | (v & kSpValMask);
}
__device__ __forceinline__ uint32_t sp_flag(uint64_t w, uint32_t ep) {
  return (uint32_t)((w >> 46) & 0xffffu) == (ep & 0xffffu) ? (uint32_t)(w >> 62) : 0u;
}

// (SpSt and sp_roles: sp_roles.hip, included by encode_v4.hip; the sparse
// form's namespace includes its own copy, so its calls do not meet cpk's)
#if CPK_SP_OWN_ROLES
#include "sp_roles.hip"
#endif

__device__ __forceinline__ uint64_t sp_ld(const uint64_t *p) { return sp_uni(*p); }

// first D word at chunk position >= x and < lim, else lim
__device__ int sp_first_d(const uint64_t *msk, int x, int lim) {
  if (x >= lim) return lim;
  int q = x >> 6;
  uint64_t m = sp_ld(&msk[3 * q + 2]) & (~0ull << (x & 63));
  while (!m) {
    ++q;
    if (q * 64 >= lim) return lim;
    m = sp_ld(&msk[3 * q + 2]);
  }
  return min(q * 64 + __builtin_ctzll(m), lim);
}

// State entering chunk step s0 from the masks of the steps before it and
// the chunk's entering state (tools/step_model.py: state_at); dep is set
// when the result used the entering state (a zero run or D/L stretch over
// every step before s0)
__device__ SpSt sp_state_at(const uint64_t *msk, int s0, SpSt cst, bool &dep) {
  if (s0 == 0) {
    dep = true;
    return cst;
  }
  SpSt st = {0u, 0u, 0u};
  const uint64_t Zp = sp_ld(&msk[3 * (s0 - 1)]), DLp = sp_ld(&msk[3 * (s0 - 1) + 1]);
  if (Zp >> 63) {
    int q = s0 - 1;
    uint32_t zl = 0;
    uint64_t z = Zp;
    while (z == ~0ull) {
      zl += 64;
      if (--q < 0) break;
      z = sp_ld(&msk[3 * q]);
    }
    st.zl = zl + (q >= 0 ? (uint32_t)__builtin_clzll(~z) : cst.zl);
    dep |= q < 0;
  }
  if (!(DLp >> 63)) return st;
  st.dlo = 1;
  int q = s0 - 1;
  uint64_t d = DLp;
  while (d == ~0ull) {
    if (--q < 0) break;
    d = sp_ld(&msk[3 * q + 1]);
  }
  const int P = 64 * s0;
  int h;
  if (q >= 0 || !cst.dlo || !cst.hd) {
    const int start = q >= 0 ? 64 * q + 64 - __builtin_clzll(~d) : 0;
    h = sp_first_d(msk, start, P);
    if (h >= P) return st;
  } else {
    h = -(int)cst.hd;
  }
  dep |= q < 0;
  for (;;) {
    const int h2 = sp_first_d(msk, max(h + 256, 0), P);
    if (h2 >= P) break;
    h = h2;
  }
  st.hd = (uint32_t)min(P - h, 256);
  return st;
}

// words of class cls (0: Z, 1: DL) from chunk step s on (<= 256); la: the
// count continuing past the chunk's end
__device__ uint32_t sp_cont(const uint64_t *msk, int s, int cs, int cls, uint32_t la) {
  uint32_t r = 0;
  for (int q = s; r < 256; ++q) {
    if (q >= cs) {
      r += la;
      break;
    }
    const uint64_t m = sp_ld(&msk[3 * q + cls]);
    if (m != ~0ull) {
      r += (uint32_t)__builtin_ctzll(~m);
      break;
    }
    r += 64;
  }
  return min(r, 256u);
}

#ifndef CPK_SP_A1G
#define CPK_SP_A1G 8  // (reload form) steps whose loads A1 keeps in flight per group
#endif
struct SpRegs {
#if !CPK_SP_RELOAD
  uint64_t v[kSpWS];       // the words, step j in v[j]
#endif
  uint32_t mp[kSpWS / 4];  // tags, four per register
  uint32_t zl, zh, dll, dlh, dl_, dh_;                 // A1 stash: Z, DL, D (lane = step)
  uint32_t oml, omh, ohl, ohh, oel, oeh;               // A2 stash: Mem, HC, E
  uint32_t ox;                                         //   X: words past the step to the next run end
};

// A1: the wave's cnt steps at src (wrem piece words from src on); returns
// this lane's nonzero-byte count
// kFull: the wave holds kSpWS whole steps -- straight-line code, so each
// step waits only for its own load (vmcnt(kSpWS - 1 - j)); with the per-step
// branches of the general form the compiler waits for all of them at the
// first step
#if CPK_SP_RELOAD
// reload form: the words are not kept for B; loads in groups of CPK_SP_A1G
// steps, the next group's in flight while a group's tags are taken
template <bool kFull>
__device__ __forceinline__ uint32_t sp_a1(SpRegs &R, const uint64_t *__restrict__ src, uint32_t wrem,
                                          int cnt, int lane) {
  constexpr int G = CPK_SP_A1G;
  static_assert(kSpWS % G == 0, "A1 groups");
  uint64_t v[2][G];
  auto ld = [&](int j) __attribute__((always_inline)) -> uint64_t {
    return (src + j * 64)[kFull ? (uint32_t)lane : min((uint32_t)lane, min(wrem - 1 - 64u * j, 63u))];
  };
#pragma unroll
  for (int i = 0; i < G; ++i)
    if (kFull || i < cnt) v[0][i] = ld(i);
  uint32_t acc = 0;
#pragma unroll
  for (int g = 0; g < kSpWS / G; ++g) {
    if (g + 1 < kSpWS / G) {
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int j = (g + 1) * G + i;
        if (kFull || j < cnt) v[(g + 1) & 1][i] = ld(j);
      }
    }
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int j = g * G + i;
      if (kFull || j < cnt) {
        const bool valid = kFull || (uint32_t)lane < wrem - 64u * j;
        const uint32_t m = valid ? e4_tag(v[g & 1][i]) : 0u;
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
    }
    CPK_SP_STEP_FENCE();
  }
  return acc;
}
#else
template <bool kFull>
__device__ __forceinline__ uint32_t sp_a1(SpRegs &R, const uint64_t *__restrict__ src, uint32_t wrem,
                                          int cnt, int lane) {
  // loads clamped to the piece, not predicated: step j's lanes read
  // min(lane, last valid lane of the step) (one lane register for all steps)
  __builtin_amdgcn_s_setprio(1);  // (the loads out first)
#pragma unroll
  for (int j = 0; j < kSpWS; ++j)
    if (kFull || j < cnt)
      R.v[j] = ld_stream(&(src + j * 64)[kFull ? (uint32_t)lane : min((uint32_t)lane, min(wrem - 1 - 64u * j, 63u))]);
  __builtin_amdgcn_s_setprio(0);
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < kSpWS; ++j) {
    if (kFull || j < cnt) {
      // (lane vs a scalar bound: no per-step lane constants kept in registers)
      const bool valid = kFull || (uint32_t)lane < wrem - 64u * j;
      const uint32_t m = valid ? e4_tag(R.v[j]) : 0u;
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
#endif

// the wave's masks to LDS (lane j = step sa + j)
__device__ __forceinline__ void sp_put_masks(const SpRegs &R, uint64_t *msk, int sa, int cnt, int lane) {
  if (lane < cnt) {
    uint64_t *m = msk + 3 * (sa + lane);
    m[0] = (uint64_t)R.zl | ((uint64_t)R.zh << 32);
    m[1] = (uint64_t)R.dll | ((uint64_t)R.dlh << 32);
    m[2] = (uint64_t)R.dl_ | ((uint64_t)R.dh_ << 32);
  }
}

// A2, sequential form (scalar ALU, one step at a time): the roles of the
// wave's steps from the state entering its first step; stashes Mem
// (literal-run members), HC (heads with a count byte) and E (run ends) at
// lane = step (B needs no mask of the words without output: they are the
// zero words that are no head); returns the steps' packed bytes beyond
// their nonzero bytes.  nz0 / ndl0: bit 0 of the step after the wave's last.
// Used when a D/L stretch longer than 192 words enters a step (a literal run
// may end inside it); sp_a2p otherwise.
__device__ __forceinline__ uint32_t sp_a2_seq(SpRegs &R, int cnt, uint32_t wrem, SpSt st, uint32_t nz0, uint32_t ndl0) {
  uint32_t bytes = 0;
  for (int j = 0; j < cnt; ++j) {
    const uint64_t Z = sp_rl(R.zl, R.zh, j), DL = sp_rl(R.dll, R.dlh, j), D = sp_rl(R.dl_, R.dh_, j);
    const uint32_t vr = wrem - 64u * j;
    const uint64_t V = vr >= 64 ? ~0ull : ((1ull << vr) - 1);
    uint64_t Zh, Mem;
    sp_roles(Z, DL, D, st, Zh, Mem);
    const uint64_t HC = Zh | (D & ~Mem), ZO = (Z & ~Zh) | ~V;
    bytes += (uint32_t)(__builtin_popcountll(~ZO & ~Mem) + __builtin_popcountll(Mem & ~D) +
                        __builtin_popcountll(HC));
    uint64_t z0 = nz0, d0 = ndl0;
    if (j + 1 < cnt) {
      z0 = (uint32_t)__builtin_amdgcn_readlane((int)R.zl, j + 1) & 1u;
      d0 = (uint32_t)__builtin_amdgcn_readlane((int)R.dll, j + 1) & 1u;
    }
    const uint64_t E = (Z & ~((Z >> 1) | (z0 << 63))) | (DL & ~((DL >> 1) | (d0 << 63)));
    R.oml = sp_wl(R.oml, (uint32_t)Mem, j);
    R.omh = sp_wl(R.omh, (uint32_t)(Mem >> 32), j);
    R.ohl = sp_wl(R.ohl, (uint32_t)HC, j);
    R.ohh = sp_wl(R.ohh, (uint32_t)(HC >> 32), j);
    R.oel = sp_wl(R.oel, (uint32_t)E, j);
    R.oeh = sp_wl(R.oeh, (uint32_t)(E >> 32), j);
  }
  return bytes;
}

// value of v at lane src
__device__ __forceinline__ uint32_t sp_from(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

// A2, lane-parallel form: lane j computes step j's roles with 64-bit vector
// ops; what carries from step to step (the zero run's length, whether the
// D/L stretch entering a step already has its 0xFF head) comes from ballots
// over the steps.  Exact while every literal run that enters a step covers
// it to its end, i.e. no D/L stretch longer than 192 words enters a step:
// returns false (nothing written) when one does.  Same stash as sp_a2_seq.
__device__ __forceinline__ bool sp_a2p(SpRegs &R, int cnt, uint32_t wrem, SpSt st, uint32_t nz0,
                                       uint32_t ndl0, int lane, uint32_t &bytes) {
  const bool act = lane < cnt;
  const uint64_t Z = act ? ((uint64_t)R.zl | ((uint64_t)R.zh << 32)) : 0ull;
  const uint64_t DL = act ? ((uint64_t)R.dll | ((uint64_t)R.dlh << 32)) : 0ull;
  const uint64_t D = act ? ((uint64_t)R.dl_ | ((uint64_t)R.dh_ << 32)) : 0ull;
  const uint64_t below = (1ull << lane) - 1;  // steps before this one
  // ---- D/L stretch entering the step: its length (bounds the distance to
  // its last head) and whether it has a head yet
  const uint32_t dlo = (uint32_t)wave_shr1((int)(uint32_t)(DL >> 63), (int)st.dlo);
  const uint32_t topdl = DL == ~0ull ? 64u : (uint32_t)__builtin_clzll(~DL);
  const uint64_t notall = __ballot(!act || DL != ~0ull);
  const uint64_t kdm = notall & below;
  const int kd = kdm ? 63 - __builtin_clzll(kdm) : -1;  // last step before with a non-D/L word
  const uint32_t topdl_k = sp_from(topdl, kd < 0 ? 0 : kd);
  const uint32_t len = kd >= 0 ? topdl_k + 64u * (uint32_t)(lane - 1 - kd)
                               : (st.dlo ? st.hd : 0u) + 64u * (uint32_t)lane;
  const bool cont = act && dlo && (DL & 1);
  if (__ballot(cont && len > 192)) return false;
  const uint64_t anyD = __ballot(act && D != 0);
  const bool topd = topdl > 0 && (D >> (64 - topdl)) != 0;
  const uint64_t TD = __ballot(act && topd);
  const uint64_t btw = anyD & below & (kd >= 0 ? (~0ull << kd) << 1 : ~0ull);
  const bool head = btw != 0 || (kd >= 0 ? ((TD >> kd) & 1) != 0 : (st.dlo && st.hd));
  const uint64_t cin = (cont && head) ? 1ull : 0ull;
  const uint64_t A = ((D << 1) | cin) & DL;
  const uint64_t C = (DL + A) ^ DL ^ A;
  const uint64_t Mem = DL & (A | C);
  // ---- zero runs: heads at run starts and every 256 words
  const uint32_t zc = (uint32_t)wave_shr1((int)(uint32_t)(Z >> 63), st.zl ? 1 : 0);
  uint64_t Zh = Z & ~((Z << 1) | zc);
  {
    const uint32_t topz = Z == ~0ull ? 64u : (uint32_t)__builtin_clzll(~Z);
    const uint64_t kzm = __ballot(!act || Z != ~0ull) & below;
    const int kz = kzm ? 63 - __builtin_clzll(kzm) : -1;
    const uint32_t topz_k = sp_from(topz, kz < 0 ? 0 : kz);
    const uint32_t zl = kz >= 0 ? topz_k + 64u * (uint32_t)(lane - 1 - kz) : st.zl + 64u * (uint32_t)lane;
    const uint32_t j0 = (256u - (zl & 255u)) & 255u;
    if (__ballot(act && zc && (Z & 1) && j0 < 64)) {
      const uint64_t pre = j0 >= 63 ? ~0ull : ((2ull << j0) - 1);
      if (act && zc && (Z & 1) && j0 < 64 && (Z & pre) == pre) Zh |= 1ull << j0;
    }
  }
  // ---- per step: output masks, run ends, bytes
  const uint32_t vr = act ? wrem - 64u * (uint32_t)lane : 0u;
  const uint64_t V = vr >= 64 ? ~0ull : ((1ull << vr) - 1);
  const uint64_t HC = Zh | (D & ~Mem), ZO = (Z & ~Zh) | ~V;
  // bit 0 of the next step (lane + 1; the wave's last step: nz0 / ndl0)
  uint32_t zn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)Z, 0x130, 0xf, 0xf, false) & 1u;
  uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)DL, 0x130, 0xf, 0xf, false) & 1u;
  if (lane == cnt - 1) {
    zn = nz0;
    dn = ndl0;
  }
  const uint64_t E = (Z & ~((Z >> 1) | ((uint64_t)zn << 63))) | (DL & ~((DL >> 1) | ((uint64_t)dn << 63)));
  uint32_t b = act ? (uint32_t)(__builtin_popcountll(~ZO & ~Mem) + __builtin_popcountll(Mem & ~D) +
                                __builtin_popcountll(HC))
                   : 0u;
  bytes = (uint32_t)__builtin_amdgcn_readlane(wave_incl_add((int)b), 63);
  R.oml = (uint32_t)Mem;
  R.omh = (uint32_t)(Mem >> 32);
  R.ohl = (uint32_t)HC;
  R.ohh = (uint32_t)(HC >> 32);
  R.oel = (uint32_t)E;
  R.oeh = (uint32_t)(E >> 32);
  return true;
}

// X per step (lane = step): words past the step's end to the first run end
// after it (a head's count reaches that far), from the next step with a run
// end; past the wave's last step, Xlast.  At most 256.
__device__ __forceinline__ void sp_xs(SpRegs &R, int cnt, uint32_t Xlast, int lane) {
  const bool act = lane < cnt;
  const uint64_t E = (uint64_t)R.oel | ((uint64_t)R.oeh << 32);
  const uint64_t en = __ballot(act && E != 0);
  const uint64_t km = lane == 63 ? 0ull : (en & (~0ull << (lane + 1)));
  const int k = km ? __builtin_ctzll(km) : 64;
  const uint32_t ce = E ? (uint32_t)__builtin_ctzll(E) : 64u;
  const uint32_t ce_k = sp_from(ce, k & 63);
  uint32_t X = k < cnt ? 64u * (uint32_t)(k - lane - 1) + ce_k : 64u * (uint32_t)(cnt - 1 - lane) + Xlast;
  R.ox = min(X, 256u);
}

// ---- the output ring -----------------------------------------------------------
// A wave lays its strings out relative to its first output byte: relative
// line i (bytes [16 i, 16 i + 16)) lives at ring line i % kSpRingLines; a
// string crossing the ring's end spills into the overhang line, which belongs
// to ring line 0.  Its offset g0 in the output may not be known yet (the
// look-back); once it is, relative line t goes to output bytes
// [g0 + 16 t, g0 + 16 t + 16) as one 16-byte store at whatever alignment g0
// has (round 5: no longer shifted onto the 16-byte-aligned output lines,
// which took two ring lines and four v_alignbyte per line; encode -8 %).
__device__ __forceinline__ uint4 sp_ring_line(const uint32_t *ring, uint32_t i) {
  const uint4 *rl = reinterpret_cast<const uint4 *>(ring);
  const uint32_t r = sp_rline(i);
  uint4 v = rl[r];
  if (r < kSpOvLines) {
    const uint4 o = rl[kSpRingLines + r];
    v.x |= o.x;
    v.y |= o.y;
    v.z |= o.z;
    v.w |= o.w;
  }
  return v;
}
__device__ __forceinline__ void sp_ring_clear(uint32_t *ring, uint32_t i) {
  uint4 *rl = reinterpret_cast<uint4 *>(ring);
  const uint32_t r = sp_rline(i);
  rl[r] = make_uint4(0u, 0u, 0u, 0u);
  if (r < kSpOvLines) rl[kSpRingLines + r] = make_uint4(0u, 0u, 0u, 0u);
}
// relative lines [ft, upto) to the output at g0 + 16 t: 16-byte stores at
// any byte alignment (every byte of the wave's output is stored by exactly
// one lane, no line is assembled from two), each line cleared once stored
typedef unsigned int sp_u32x4u __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ void sp_flush_rel(uint8_t *out, uint32_t *ring, uint64_t g0, uint32_t &ft,
                                             uint32_t upto, int lane, uint64_t ocap) {
  for (uint32_t t0 = ft; t0 < upto; t0 += 64) {
    const uint32_t t = t0 + (uint32_t)lane;
    if (t < upto) {
      const uint4 v = sp_ring_line(ring, t);
      const uint64_t a = g0 + 16ull * t;
      if (a + 16 <= ocap) {
        const sp_u32x4u w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<sp_u32x4u *>(out + a));
      }
      sp_ring_clear(ring, t);
    }
  }
  ft = upto;
}

// B: the wave's strings, laid out relative to its first output byte.  Its
// offset is given (known) or fetched once kSpDefer steps are in the ring
// (getbase: wave 0 runs the piece's look-back meanwhile -- the other waves
// have had that many steps of work before they wait for it).
// steps laid out before the offset is needed (12 at 8 KiB)
constexpr int kSpDefer = (((int)(kSpRing - 16) / 640) & ~1);
// (every wave whose output fits its ring lays out all its steps before
// fetching the offset: the look-back then runs last, when the pieces before
// have published -- measured best)
static_assert(kSpDefer * 640 + 16 <= (int)kSpRing && kSpDefer % 2 == 0, "deferred steps must fit the ring");
template <class GetBase>
__device__ __forceinline__ void sp_b(SpRegs &R, int cnt, const uint64_t *lut, uint32_t *ring, uint8_t *out,
                                     bool known, bool fits, uint64_t g0, int lane, uint64_t ocap,
                                     const uint64_t *__restrict__ src, uint32_t wrem, GetBase getbase) {
#if CPK_SP_RELOAD
  // the words again (read by A1 moments ago: L2), 2 pairs ahead
  uint64_t pv[kSpWS];
  // only the lanes whose word is nonzero load it (a zero word's string
  // needs no bytes): a line of zero words is not fetched again at all
  auto ldw = [&](int j) __attribute__((always_inline)) {
    if (j < kSpWS && j < cnt) {
      const uint32_t m = (R.mp[j >> 2] >> (8 * (j & 3))) & 0xffu;
      pv[j] = m ? ld_stream(&(src + j * 64)[min((uint32_t)lane, min(wrem - 1 - 64u * j, 63u))]) : 0ull;
    }
  };
#pragma unroll
  for (int j = 0; j < 2 * 2; ++j) ldw(j);
#endif
  uint32_t rel = 0, ft = 0;
  // the output offset is wave-uniform: say so (readfirstlane), or the flush
  // condition and the line shift's switch on g0 & 15 compile to exec-masked
  // branches
  g0 = sp_uni(g0);
  const uint32_t l64 = 64u - (uint32_t)lane;
  // step j's string per lane (s0..s2, nb bytes)
  auto strings = [&](const int j, uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &nb)
      __attribute__((always_inline)) {
    const uint64_t Mem = sp_rl(R.oml, R.omh, j);
    const uint64_t HC = sp_rl(R.ohl, R.ohh, j);
    const uint32_t m = (R.mp[j >> 2] >> (8 * (j & 3))) & 0xffu;
#if CPK_SP_RELOAD
    const uint32_t lo = (uint32_t)pv[j], hi = (uint32_t)(pv[j] >> 32);
#else
    const uint32_t lo = (uint32_t)R.v[j], hi = (uint32_t)(R.v[j] >> 32);
#endif
    const uint64_t sel = lut[m];
    const uint32_t c0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
    const uint32_t c1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
    const bool zw = m == 0;
    // (the step's zero words as a mask: the head-count and byte-count
    // selects below take scalar mask algebra instead of per-lane selects)
    const uint64_t ZW = __ballot(zw);
    uint32_t cz = 0, cd = 0;
#if CPK_SP_HCALL
    // (the dense form: nearly every step has heads, no branch -- config 2
    // encode -0.9 %; the sparse form keeps it, +36 % without)
#else
    if (HC)
#endif
    {
      // a head's count: words to its run's end, at most 255 (:119-131, :143-164)
      const uint32_t X = (uint32_t)__builtin_amdgcn_readlane((int)R.ox, j);
      const uint64_t E = sp_rl(R.oel, R.oeh, j);
      const uint64_t e = E >> lane;
      // ctz of e, 0xffffffff when e == 0 (the next run end is past the step):
      // v_ffbl_b32 gives 0xffffffff for 0 itself (no compare / select)
      const uint32_t z_lo = sp_ffbl((uint32_t)e);
      const uint32_t z_hi = sp_ffbl((uint32_t)(e >> 32)) | 32u;  // (ctz < 32: | is +)
      const uint32_t tt = min(min(z_lo, z_hi), min(l64 + X, 255u));
      cz = sp_sel(0u, tt, HC & ZW);   // zero-run heads: the count after the 0x00 tag
      cd = sp_sel(0u, tt, HC & ~ZW);  // 0xFF heads: the count after the 8 bytes
    }
    // the string: tag, the nonzero bytes, the count after a 0x00 / 0xFF tag
    // (c0 is zero for a zero word); a literal-run member is its 8 bytes
    const uint32_t c0p = c0 | cz;
    s0 = m | (c0p << 8);
    s1 = __builtin_amdgcn_alignbyte(c1, c0p, 3);
    s2 = __builtin_amdgcn_alignbyte(cd, c1, 3);
    s0 = sp_sel(s0, lo, Mem);
    s1 = sp_sel(s1, hi, Mem);
    s2 = sp_sel(s2, 0u, Mem);
    nb = (uint32_t)__builtin_popcount(m) + sp_sel(1u, 2u, HC);
    nb = sp_sel(nb, 8u, Mem);
    // no bytes: a zero word that is no head -- a zero-run member, or a word
    // past the piece's end (A1 left its tag 0, and it is in no mask): the
    // ZO mask, without its two lane reads
    nb = sp_sel(nb, 0u, ZW & ~HC);
  };
  // a string OR-ed into the ring at relative byte p (r4 / relq: the ring
  // dword of the step's first byte rel and rel >> 2, wave-uniform -- the
  // ring position without a per-lane modulo: p - rel < 1,284)
  auto put = [&](uint32_t p, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t nb, uint32_t c)
      __attribute__((always_inline)) {
    // the string shifted left by p & 3 bytes over four dwords: one v_perm
    // each, selector bytes [4 - b, 8 - b) of (s_k : s_k-1)
    const uint32_t b = p & 3;
    const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, b, 0u);  // (b in every byte)
    const uint32_t d0 = __builtin_amdgcn_perm(s0, 0u, sel), d1 = __builtin_amdgcn_perm(s1, s0, sel);
    const uint32_t d2 = __builtin_amdgcn_perm(s2, s1, sel), d3 = __builtin_amdgcn_perm(0u, s2, sel);
    const uint32_t q = (p >> 2) + c;
    uint32_t *rp = ring + q;
    if (nb) {  // (zero-length strings would all hit one address)
      atomicOr(rp, d0);
      atomicOr(rp + 1, d1);
      atomicOr(rp + 2, d2);
      atomicOr(rp + 3, d3);
    }
  };
  // steps j and j + 1 (when j + 1 < cnt): both byte counts in one wave scan
  // (16-bit halves: a step's strings total at most 640 bytes)
  auto step = [&](const int j) __attribute__((always_inline)) {
#if CPK_SP_RELOAD
    ldw(j + 2 * 2);
    ldw(j + 2 * 2 + 1);
#endif
#if CPK_SP_SKIP
    // (the sparse form: a step of zero words and no head -- inside a zero
    // run -- has no bytes: its strings are not built, and a pair of them is
    // skipped whole)
    auto empty = [&](const int k) __attribute__((always_inline)) {
      const uint32_t m = (R.mp[k >> 2] >> (8 * (k & 3))) & 0xffu;
      return k >= cnt || (__ballot(m != 0u) == 0ull && sp_rl(R.ohl, R.ohh, k) == 0ull);
    };
    const bool ea = empty(j), eb = empty(j + 1);
    if (!(ea && eb))
#endif
    {
      uint32_t a0 = 0, a1 = 0, a2 = 0, na = 0, b0 = 0, b1 = 0, b2 = 0, nb2 = 0;
#if CPK_SP_SKIP
      if (!ea) strings(j, a0, a1, a2, na);
      if (!eb) strings(j + 1, b0, b1, b2, nb2);
#else
      strings(j, a0, a1, a2, na);
      if (j + 1 < cnt) strings(j + 1, b0, b1, b2, nb2);
#endif
      const uint32_t pk = na | (nb2 << 16);
      const uint32_t incl = (uint32_t)wave_incl_add((int)pk);
      const uint32_t stot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      if (stot) {
        const uint32_t ta = stot & 0xffffu;
        {
          // (per step, scalar: its first dword's ring position minus that dword)
          const uint32_t qa = rel >> 2, relb = rel + ta, qb = relb >> 2;
          put(rel + (incl & 0xffffu) - na, a0, a1, a2, na, qa % kSpRing4 - qa);
          put(relb + (incl >> 16) - nb2, b0, b1, b2, nb2, qb % kSpRing4 - qb);
        }
        rel += ta + (stot >> 16);
        // complete lines leave 64 at a time (one full-wave store)
        if (known) {
          const uint32_t done = rel >> 4;
          if (done - ft >= 64u) {
            wave_lds_order();
            sp_flush_rel(out, ring, g0, ft, ft + 64, lane, ocap);
            wave_lds_order();
          }
        }
      }
    }

    CPK_SP_STEP_FENCE();
  };
  // (two fully unrolled loops around the one place the offset may be fetched)
#pragma unroll
  for (int j = 0; j < kSpDefer; j += 2)
    if (j < cnt) step(j);
  if (!known && !fits && cnt > kSpDefer) {
    g0 = getbase();
    g0 = sp_uni(g0);
    known = true;
  }
#pragma unroll
  for (int j = kSpDefer; j < kSpWS; j += 2)
    if (j < cnt) step(j);
  if (!known) g0 = getbase();
  g0 = sp_uni(g0);
  wave_lds_order();
  const uint32_t done = rel >> 4, rem = rel & 15;
  sp_flush_rel(out, ring, g0, ft, done, lane, ocap);
  if (rem) {
    // the last, partial line: its bytes one per lane
    const uint4 v = sp_ring_line(ring, done);
    const uint64_t a = g0 + 16ull * done + (uint32_t)lane;
    if ((uint32_t)lane < rem && a < ocap) {
      const uint32_t d = (lane & 8) ? ((lane & 4) ? v.w : v.z) : ((lane & 4) ? v.y : v.x);
      out[a] = (uint8_t)(d >> (8 * (lane & 3)));
    }
    if (lane == 0) sp_ring_clear(ring, done);
  }
  wave_lds_order();
}

// Look-ahead past a chunk: the zero run / D/L stretch continuing from the
// chunk's end (<= 256 words each), from the next 4 steps' words.
__device__ __forceinline__ void sp_lookahead(const uint64_t *__restrict__ src, uint32_t avail, int lane,
                                             uint32_t &laz, uint32_t &ladl) {
  uint32_t rz = 0, rd = 0;
  bool oz = true, od = true;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool valid = (uint32_t)lane < (avail > 64u * j ? avail - 64u * j : 0u);
    const uint64_t x = valid ? (src + 64 * j)[lane] : 0ull;
    const uint32_t m = valid ? e4_tag(x) : 0u;
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

// the decoupled look-back (wave 0, all lanes; the piece's aggregate was
// published as soon as its size was known): returns the exclusive prefix,
// publishes the inclusive one
__device__ uint64_t sp_lookback(uint64_t *status, uint32_t p, uint64_t agg, uint32_t ep, uint32_t *err,
                                int lane) {
  if (p == 0) return 0;
  uint64_t excl = 0;
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
#ifdef CPK_PHASE_STATS
    if (lane == 0) atomicAdd(&g_phase[40], 1ull);  // polls
#endif
    if (__ballot(z)) {
#ifdef CPK_PHASE_STATS
      if (lane == 0) atomicAdd(&g_phase[42], 1ull);  // polls that met an unpublished predecessor
#endif
      if (++spins > (1u << 22)) {  // cannot happen: every predecessor is held by a running workgroup
        if (lane == 0) atomicOr(err, 4u);
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
  if (lane == 0) st_status(&status[p], sp_word(ep, 2u, excl + agg));
  return excl;
}

// (stats build: A1 alone into phase slot 7)
#ifdef CPK_PHASE_STATS
#define SP_A1_PARAMS , unsigned long long &wph_last, unsigned long long *wph_acc
#define SP_A1_ARGS , wph_last, wph_acc
#define SP_A1_STAMP WPH(7)
#else
#define SP_A1_PARAMS
#define SP_A1_ARGS
#define SP_A1_STAMP
#endif
// run state <-> a look-back value (zl < 2^31, dlo, hd <= 256: 41 bits)
__device__ __forceinline__ uint64_t sp_pack_state(SpSt s) {
  return (uint64_t)s.zl | ((uint64_t)s.dlo << 31) | ((uint64_t)s.hd << 32);
}
__device__ __forceinline__ SpSt sp_unpack_state(uint64_t v) {
  SpSt s = {(uint32_t)v & 0x7fffffffu, (uint32_t)(v >> 31) & 1u, (uint32_t)(v >> 32) & 0x1ffu};
  return s;
}

// One chunk's A1 + A2 for this wave (all waves call it; two barriers, three
// when the chunk continues a piece).  Returns the chunk's packed bytes (all
// waves); wbefore: bytes of the waves before this one.  The state entering
// the chunk is fresh (a piece's first chunk) or the run state the
// predecessor chunk of the piece published (prev, epoch-tagged, flag 2),
// waited for once this chunk's masks are in LDS; the state leaving it is
// published at next when the piece continues.
__device__ __forceinline__ uint64_t sp_chunk(SpRegs &R, const uint64_t *__restrict__ pw, uint32_t W,
                                             uint32_t c, uint64_t *msk, uint64_t *scr, uint64_t *prev,
                                             uint64_t *next, uint32_t ep, uint32_t *err, int w, int lane,
                                             int &cnt, uint32_t &Xlast, uint64_t &wbefore,
                                             uint64_t &wmine, const uint64_t *&wsrc,
                                             uint32_t &wrem_o SP_A1_PARAMS) {
  const uint32_t ns = (W + 63) >> 6;
  const uint32_t cs0 = c * kSpCS;
  const int cs = (int)min((uint32_t)kSpCS, ns - cs0);  // steps in this chunk
  // a chunk's steps spread over all waves (a short piece keeps every wave
  // busy, not wave 0 alone): per wave ceil(cs / waves), rounded up to a pair
  const int per = min(kSpWS, ((cs + kSpWaves - 1) / kSpWaves + 1) & ~1);
  const int sa = w * per;
  cnt = max(0, min(per, cs - sa));
  const uint32_t wfirst = (cs0 + (uint32_t)sa) * 64;  // the wave's first word
  const uint32_t wrem = cnt ? W - wfirst : 0;
  wsrc = pw + wfirst;
  wrem_o = wrem;
  uint32_t acc = 0;
  if (cnt) {
    if (cnt == kSpWS && wrem >= 64u * kSpWS) acc = sp_a1<true>(R, pw + wfirst, wrem, cnt, lane);
    else
      acc = sp_a1<false>(R, pw + wfirst, wrem, cnt, lane);
    sp_put_masks(R, msk, sa, cnt, lane);
  }
  SP_A1_STAMP
  __syncthreads();  // the chunk's masks in LDS
  SpSt cst = {0u, 0u, 0u};
  // the state leaving the chunk depends on the one entering it only when a
  // zero run or D/L stretch covers the whole chunk: otherwise it is
  // published now, before this chunk waits for its own entering state, so
  // the chunks of a piece do not wait on one another in a chain
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
    // the run state entering the chunk: the predecessor chunk (an earlier
    // ticket, so resident and running) publishes it after its own A2
    if (threadIdx.x == 0) {
      uint32_t spins = 0;
      uint64_t v;
      while (sp_flag(v = ld_status(prev), ep) != 2u) {
        if (++spins > (1u << 24)) {  // cannot happen: see above
          atomicOr(err, 4u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      scr[12] = v & kSpValMask;
    }
    __syncthreads();
    cst = sp_unpack_state(sp_ld(&scr[12]));
  }
  SpSt st = cst;
  uint32_t bytes = 0;
  const bool last = cnt && sa + cnt == cs;  // this wave holds the chunk's last step
  if (cnt) {
    bool dep_ = false;
    st = sp_state_at(msk, sa, cst, dep_);
    uint32_t nz0 = 0, ndl0 = 0;
    Xlast = 0;
    {
      // the step after the wave's last: in the chunk, or past it (look-ahead)
      uint32_t laz = 0, ladl = 0;
      const uint32_t wend = wfirst + 64u * cnt;
      if (last && wend < W) sp_lookahead(pw + wend, W - wend, lane, laz, ladl);
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
    // the state leaving the chunk, for the piece's next chunk
    bool dep_ = false;
    st = sp_state_at(msk, cs, cst, dep_);
    if (lane == 0) st_status(next, sp_word(ep, 2u, sp_pack_state(st)));
  }
  if (lane == 0) scr[16 + w] = bytes;
  __syncthreads();  // wave bytes in LDS
  uint64_t tot = 0;
  wbefore = 0;
  wmine = 0;
#pragma unroll
  for (int q = 0; q < kSpWaves; ++q) {
    const uint64_t b = sp_ld(&scr[16 + q]);
    if (q < w) wbefore += b;
    if (q == w) wmine = b;
    tot += b;
  }
  return tot;
}

// kMsg = false: piece p is words [swo[p], swo[p+1]) of `in`.  kMsg = true:
// pdesc[2p] = first word (bit 63: of `tin`, the segment tables) and
// pdesc[2p+1] = words.
// Units: a ticket is one chunk of kSpCS steps (8192 words) of one piece --
// utab[u] = piece << 32 | chunk, *nunits of them (utab == nullptr: every
// piece is one chunk, unit = piece).  Every unit publishes its packed bytes
// for the decoupled look-back over units, and a chunk that continues a
// piece takes the run state its predecessor leaves (ustate[u - 1]), so a
// large piece is encoded by many workgroups at once and read once (U + P),
// and no piece waits for a large one before it to be emitted.
template <bool kMsg>
__global__ __launch_bounds__(kSpThreads, CPK_SP_WPE) void sp_encode_kernel(
    const uint64_t *__restrict__ in, const uint64_t *__restrict__ swo,
    const uint64_t *__restrict__ pdesc, const uint64_t *__restrict__ tin, uint32_t n,
    uint8_t *__restrict__ out, uint64_t *__restrict__ out_off, uint64_t *status, uint32_t ep,
    uint32_t *ticket, const uint64_t *__restrict__ utab, const uint64_t *__restrict__ nunits,
    uint64_t *ustate, uint64_t hint, uint32_t *err, const uint64_t *ocapp, const uint32_t *pick, uint32_t mine,
    uint64_t ucap) {
  // (pick: the device gate's choice between this form and the other one)
  if (pick && (uint32_t)__builtin_amdgcn_readfirstlane((int)*pick) != mine) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // a bound on the output buffer's size: sum of 9 w + 1 over the pieces
  // (cpk_packed_bound(w) <= 9 w + 1), + 16
  // and the caller's capacity (cpk_encode_batch_cap): no line or byte at or
  // past it is stored
  const uint64_t ocap = min(kMsg ? *ocapp : 9 * (swo[n] - swo[0]) + n + 16, ucap);
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem + kSpoLut);
  uint64_t *msk = reinterpret_cast<uint64_t *>(smem + kSpoMsk);
  uint64_t *scr = reinterpret_cast<uint64_t *>(smem + kSpoScr);
  const int lane0 = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  uint32_t *ring = reinterpret_cast<uint32_t *>(smem + kSpoRing + w * kSpRingStride);
  fill_luts(lut, false);
  for (uint32_t i = lane0; i < kSpRingStride / 16; i += 64)
    reinterpret_cast<uint4 *>(ring)[i] = make_uint4(0u, 0u, 0u, 0u);
  SpRegs R;
  R.zl = R.zh = R.dll = R.dlh = R.dl_ = R.dh_ = 0;
  R.oml = R.omh = R.ohl = R.ohh = R.oel = R.oeh = 0;
  if (threadIdx.x == 0) scr[11] = 0;  // (LDS holds whatever the last kernel left)
  const uint32_t nu = utab ? (uint32_t)*nunits : n;
  WPH_INIT
  for (;;) {
    WPH(3)
    if (threadIdx.x == 0) scr[0] = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t t = (uint32_t)sp_ld(&scr[0]);
    __syncthreads();  // (scr[0] read by all before the next ticket)
    WPH(0)
    if (t >= nu) break;
    const uint64_t ud = utab ? utab[t] : (uint64_t)t << 32;
    const uint32_t p = (uint32_t)(ud >> 32), c = (uint32_t)ud;
    // an opaque copy of the lane id: nothing lane-dependent is hoisted out
    // of the unit loop into registers that stay live across it
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    uint64_t w0, W64;
    const uint64_t *base = in;
    if (kMsg) {
      w0 = pdesc[2 * (uint64_t)p];
      W64 = pdesc[2 * (uint64_t)p + 1];
      if (w0 >> 63) base = tin;
      w0 &= ~(1ull << 63);
    } else {
      w0 = swo[p];
      W64 = swo[p + 1] - w0;
    }
    // (with a unit table, a piece over the hint is one empty unit: see
    // sp_units_count_kernel)
    bool bad = W64 >= (1ull << 31) || (!utab && W64 > 64ull * kSpCS) || (utab && hint && W64 > hint);
    if ((bad || (hint && W64 > hint)) && threadIdx.x == 0 && c == 0) atomicOr(err, 1u);
    const uint32_t W = bad ? 0u : (uint32_t)W64;  // (unsupported: sized 0, output undefined)
    const uint64_t *pw = base + w0;
    const uint32_t nch = max((((W + 63) >> 6) + kSpCS - 1) / kSpCS, 1u);
    const bool lastc = c + 1 >= nch;  // (the piece's last chunk)
    int cnt = 0;
    uint32_t Xlast = 0;
    uint64_t wbefore = 0, wmine = 0;
    const uint64_t *wsrc = pw;
    uint32_t wrem = 0;
    const uint64_t ct = sp_chunk(R, pw, W, c, msk, scr, c ? ustate + (t - 1) : nullptr,
                                 lastc ? nullptr : ustate + t, ep, err, w, lane, cnt, Xlast, wbefore,
                                 wmine, wsrc, wrem SP_A1_ARGS);
    WPH(1)
    if (w == 0 && lane == 0) {
      // the unit's size, published before its strings are laid out: the
      // units after it find it there when they look back
      st_status(&status[t], sp_word(ep, t == 0 ? 2u : 1u, ct));
    }
    WPH(2)
    // the offset: the look-back (wave 0) runs once the waves have laid out
    // kSpDefer steps (or all of them, when they fit the ring)
    auto getoff = [&]() {
      const uint64_t excl = sp_lookback(status, t, ct, ep, err, lane);
      // (a unit whose bytes pass the caller's capacity: reported; its lines
      // past the capacity are not stored, ArrayOutputStream.java:40-42)
      if (lane == 0 && excl + ct > ucap) atomicOr(err, kErrCap);
      if (lane == 0) {
        scr[5] = excl;
        if (c == 0) out_off[p] = excl;
        if (p + 1 == n && lastc) out_off[n] = excl + ct;
        __builtin_amdgcn_s_waitcnt(0xc07f);  // (the offset before the flag)
        scr[11] = (uint64_t)t + 1;
      }
      return excl;
    };
    if (cnt) {
      auto getbase = [&]() -> uint64_t {
        WPH(4)
        if (w == 0) {
          const uint64_t excl = getoff();
          WPH(5)
          return excl + wbefore;
        }
        while ((uint32_t)sp_ld(&scr[11]) != t + 1) __builtin_amdgcn_s_sleep(1);
        WPH(6)
        return sp_ld(&scr[5]) + wbefore;
      };
      sp_b(R, cnt, lut, ring, out, false, wmine + 16 <= kSpRing, wbefore, lane, ocap,
           wsrc, wrem, getbase);
    } else if (w == 0) {
      getoff();  // wave 0 runs the look-back even without steps (an empty piece)
    }
    // (no wave takes the next ticket before the unit's offset is out: scr[5])
    while ((uint32_t)sp_ld(&scr[11]) != t + 1) __builtin_amdgcn_s_sleep(1);
    WPH(4)
  }
  WPH_FLUSH(32)
}

// piece descriptors in message order (table, segments; next message) and the
// tables' words (Serialize.java:256-273): message m's table goes to word
// mseg[m] / 2 + m of tbuf (room for (count + 2) / 2 words)
__global__ void sp_msg_prep_kernel(const uint64_t *__restrict__ swo, const uint64_t *__restrict__ mseg,
                                   uint32_t nm, uint64_t *__restrict__ pdesc, uint64_t *__restrict__ tbuf,
                                   uint64_t *__restrict__ ocap) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m == 0) {
    // output bound: segments 9 w + 1 each, tables (<= nseg / 2 + nm words) likewise, + 16
    const uint64_t nseg = mseg[nm];
    *ocap = 9 * (swo[nseg] - swo[0]) + nseg + 9 * (nseg / 2 + nm) + nm + 16;
  }
  if (m >= nm) return;
  const uint64_t s0 = mseg[m], s1 = mseg[m + 1];
  const uint32_t count = (uint32_t)(s1 - s0);
  const uint32_t tw = table_words(count);
  const uint64_t to = s0 / 2 + m;
  for (uint32_t k = 0; k < tw; ++k) tbuf[to + k] = table_word(swo, s0, count, k);
  uint64_t *d = pdesc + 2 * (s0 + m);
  d[0] = (1ull << 63) | to;
  d[1] = tw;
  for (uint64_t s = s0; s < s1; ++s) {
    d[2 * (1 + s - s0)] = swo[s];
    d[2 * (1 + s - s0) + 1] = swo[s + 1] - swo[s];
  }
}

// Units of the single-pass encoder (sp_encode_kernel): a piece of W words is
// max(1, ceil(W / 8192)) units, one per chunk.  ucnt[p] = its unit count
// (scanned into ustart by the e4 scan kernels), then utab[ustart[p] + k] =
// p << 32 | k.
// A piece the encoder cannot take (2^31 words or more, or over the caller's
// hint) is one unit of no words, exactly as sp_encode_kernel sizes it: the
// unit table then never outgrows the bound the host sized it by
// (sp_unit_bound: ceil(hint / 8192) units per piece).
__global__ void sp_units_count_kernel(const uint64_t *__restrict__ swo, const uint64_t *__restrict__ pdesc,
                                      uint32_t n, uint64_t hint, uint64_t *__restrict__ ucnt) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint64_t W = pdesc ? pdesc[2 * (uint64_t)p + 1] : swo[p + 1] - swo[p];
  if (W >= (1ull << 31) || (hint && W > hint)) W = 0;
  const uint64_t steps = (W + 63) >> 6;
  ucnt[p] = steps > (uint64_t)kSpCS ? (steps + kSpCS - 1) / kSpCS : 1;
}
__global__ void sp_units_fill_kernel(const uint64_t *__restrict__ ustart, uint32_t n, uint64_t *__restrict__ utab) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint64_t a = ustart[p], b = ustart[p + 1];
  for (uint64_t k = a; k < b; ++k) utab[k] = ((uint64_t)p << 32) | (k - a);
}
