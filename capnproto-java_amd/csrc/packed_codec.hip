// packed_codec.hip -- MI355X (gfx950, CDNA4) batched codec for Cap'n Proto's
// packed stream encoding, and its C ABI (include/capnp_packed.h).
//
// Reference semantics: runtime/src/main/java/org/capnproto/
//   PackedOutputStream.java:35-205 (encoder), PackedInputStream.java:35-140
//   (decoder).  One "piece" = one write()/read() call; pieces are independent
//   (PackedOutputStream.java:36-43 re-initialises all run state per call).
//
// Design (DESIGN.md has the full derivation and the rooflines):
//   encode_kernel  one 512-thread workgroup per piece (<= 8192 words), 16
//                  words per lane held in VGPRs, word classes from a SWAR
//                  nonzero-byte mask, run roles from three workgroup scans
//                  (run start, run end, byte offsets), the 0xFF literal-run
//                  chain walked only for D/L stretches > 256 words, the
//                  packed bytes compacted in LDS and stored as 16-byte lines.
//                  Piece output offsets come from a decoupled look-back over
//                  an ordered ticket, so the output is one contiguous stream.
//   decode_kernel  one 512-thread workgroup per piece: packed bytes staged in
//                  LDS, the tag chain found by speculative per-lane walks with
//                  pointer-doubling validation, then a gather-expand of every
//                  8-word output block from its covering record.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <thread>
#include <vector>

#include "../../include/capnp_packed.h"

namespace cpk {

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kChunk = 4;                       // contiguous words per lane chunk
constexpr int kJ = 4;                           // chunks per lane
constexpr int kWaveWords = 64 * kChunk * kJ;    // 1024
constexpr int kTileWords = kWaves * kWaveWords; // 8192
constexpr int kBig = 0x3fffffff;
// encoder geometry: 1024 threads, 8 words per lane (2 chunks of 4)
#ifndef CPK_ENC_WPE
#define CPK_ENC_WPE 8  // waves per SIMD the encoder's registers must allow (2 workgroups per CU)
#endif
constexpr int kEncThreads = 1024;
constexpr int kEncWaves = kEncThreads / 64;                 // 16
constexpr int kEncJ = kTileWords / (kEncThreads * kChunk);  // 2
constexpr int kEncWaveWords = 64 * kChunk * kEncJ;          // 512

// ---------------------------------------------------------------- LDS maps
// Encoder: staging for the packed bytes of one piece (bound 9*8192 = 73,728)
// plus 16 bytes of alignment pad and slack; then LUT, bitmaps, scratch.
constexpr uint32_t kEncStage = 9 * kTileWords + 64;
constexpr uint32_t kEncLut = kEncStage;                 // u64[256]
constexpr uint32_t kEncDbits = kEncLut + 2048;          // u32[256]
constexpr uint32_t kEncHbits = kEncDbits + 1024;        // u32[256]
constexpr uint32_t kEncScr = kEncHbits + 1024;          // int[128]
constexpr uint32_t kEncMasks = kEncScr + 512;           // u64[16 waves][8 steps][2]
constexpr uint32_t kEncLds = kEncMasks + 2048;          // 80,448 B -> 2 WG / CU

static_assert(kEncLut % 16 == 0, "lut must be aligned");
static_assert(kEncLds <= 81920, "2 encoder workgroups per CU");

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// ---- ticket counters ------------------------------------------------------
// One counter word saturates near 88 returning atomics per microsecond
// (MI355X_MICROARCH.md, row "dequeue").  Work with no order dependence (the
// decoder) is sharded per XCD: the k-th ticket taken from counter x is item
// 8k + x, every item is taken exactly once, and a wave whose counter runs
// dry moves on to the next counter, so coverage never depends on where the
// waves were placed (the XCD id only picks the first counter).  Work whose
// items depend on their predecessors (the encoders' look-back) keeps one
// ordered counter.
constexpr int32_t kMaxSegmentWords = (1 << 28) - 1;  // Serialize.java:45
constexpr int kTkStride = 32;          // u32 words between counters (128 B)
constexpr int kTkEnc = 0;              // encoder counters [8]
constexpr int kTkDec = 8 * kTkStride;  // decoder counters [8]
constexpr int kTkPlan = 16 * kTkStride;
constexpr int kTkErr = 17 * kTkStride;
constexpr int kTkWords = 18 * kTkStride;
__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7;
}
// all 64 lanes call it (one folded +64 atomic per wave); the wave's item
__device__ __forceinline__ uint32_t take_ticket(uint32_t *ctr, int x) {
  const uint32_t t = atomicAdd(&ctr[x * kTkStride], 1u);
  return (((uint32_t)__builtin_amdgcn_readlane((int)t, 0) >> 6) << 3) | (uint32_t)x;
}
// ordered single-counter form
__device__ __forceinline__ uint32_t take_ordered(uint32_t *ctr) {
  const uint32_t t = atomicAdd(ctr, 1u);
  return (uint32_t)__builtin_amdgcn_readlane((int)t, 0) >> 6;
}
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// ------------------------------------------------------------ wave scans
// DPP forms (gfx9 row_shr / row_bcast): no lane-compare masks, no LDS.
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ int dpp(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, kCtrl, kRowMask, 0xf, false);
}
#define CPK_WAVE_SCAN(NAME, OP, ID)                         \
  __device__ __forceinline__ int NAME(int v) {              \
    v = OP(v, dpp<0x111>(ID, v));                           \
    v = OP(v, dpp<0x112>(ID, v));                           \
    v = OP(v, dpp<0x114>(ID, v));                           \
    v = OP(v, dpp<0x118>(ID, v));                           \
    v = OP(v, dpp<0x142, 0xa>(ID, v));                      \
    v = OP(v, dpp<0x143, 0xc>(ID, v));                      \
    return v;                                               \
  }
__device__ __forceinline__ int op_max(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int op_min(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ int op_add(int a, int b) { return a + b; }
CPK_WAVE_SCAN(wave_incl_max, op_max, -1)
CPK_WAVE_SCAN(wave_incl_add, op_add, 0)
CPK_WAVE_SCAN(wave_incl_min_fwd, op_min, 0x3fffffff)
// value of lane-1 (lane 0 gets `id`)
__device__ __forceinline__ int wave_shr1(int v, int id) { return dpp<0x138>(id, v); }
// suffix (right-to-left) inclusive min via lane reversal
__device__ __forceinline__ int wave_sufx_min(int v) {
  const int rl = 63 - (int)(threadIdx.x & 63);
  int r = __shfl(v, rl, 64);
  r = wave_incl_min_fwd(r);
  return __shfl(r, rl, 64);
}
__device__ __forceinline__ int readlane(int v, int l) {
  return __builtin_amdgcn_readlane(v, l);
}

// ---- diagnostic phase timing (built only with -DCPK_PHASE_STATS) ----------
// Thread 0 of each workgroup accumulates s_memtime deltas per phase in LDS
// (scr[96..127] as u64[16]) and adds them to g_phase at exit.  Shares of the
// total, not absolute times, are what a stats build is good for.
#ifdef CPK_PHASE_STATS
__device__ unsigned long long g_phase[64];
#define PH_INIT(scr)                                                         \
  unsigned long long ph_last = 0;                                            \
  unsigned long long *ph_acc = reinterpret_cast<unsigned long long *>(&(scr)[96]); \
  if (threadIdx.x < 16) ph_acc[threadIdx.x] = 0;                            \
  if (threadIdx.x == 0) ph_last = __builtin_amdgcn_s_memtime();
#define PH(i)                                                                \
  if (threadIdx.x == 0) {                                                    \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                    \
    ph_acc[i] += t_ - ph_last;                                               \
    ph_last = t_;                                                            \
  }
#define PH_ADD(i, v) if (threadIdx.x == 0) ph_acc[i] += (v);
#define PH_FLUSH(base)                                                       \
  __syncthreads();                                                           \
  if (threadIdx.x < 16) atomicAdd(&g_phase[(base) + threadIdx.x], ph_acc[threadIdx.x]);
// wave-level form (barrier-free kernels): per-wave sums, lane 0 flushes
#define WPH_INIT                                                             \
  unsigned long long wph_last = __builtin_amdgcn_s_memtime(), wph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define WPH(i)                                                               \
  {                                                                          \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                    \
    wph_acc[i] += t_ - wph_last;                                             \
    wph_last = t_;                                                           \
  }
#define WPH_FLUSH(base)                                                      \
  if ((threadIdx.x & 63) == 0)                                               \
    for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_phase[(base) + i_], wph_acc[i_]);
#else
#define PH_INIT(scr)
#define PH(i)
#define PH_ADD(i, v)
#define PH_FLUSH(base)
#define WPH_INIT
#define WPH(i)
#define WPH_FLUSH(base)
#endif

// nonzero-byte mask of a 32-bit half: bit b set iff byte b != 0
__device__ __forceinline__ uint32_t nzmask4(uint32_t d) {
  uint32_t t = (((d & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d) & 0x80808080u;
  uint32_t x = t >> 7;          // bits 0,8,16,24
  x |= x >> 7;                  // bits 0,1 8,9 16,17 ...
  x |= x >> 14;                 // bits 0..3
  return x & 0xfu;
}

// LUT entries.  compact: byte j = index of the j-th set bit of m (else 0x0C
// = zero byte for v_perm).  expand: byte i = popcount(m & ((1<<i)-1)) if bit
// i is set, else 0x0C.
__device__ void fill_luts(uint64_t *lut, bool expand) {
  int m = threadIdx.x;
  if (m < 256) {
    uint64_t v = 0;
    if (expand) {
      int c = 0;
      for (int i = 0; i < 8; ++i) {
        uint64_t s = (m >> i) & 1 ? (uint64_t)(c++) : 0x0cull;
        v |= s << (8 * i);
      }
    } else {
      int j = 0;
      for (int i = 0; i < 8; ++i)
        if ((m >> i) & 1) v |= (uint64_t)i << (8 * j++);
      for (; j < 8; ++j) v |= 0x0cull << (8 * j);
    }
    lut[m] = v;
  }
}

// Orders this wave's LDS accesses without waiting for them: DS instructions
// of one wave execute in issue order, so a later read sees earlier writes
// and atomics of every lane; only the compiler must not reorder across.
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wave_lds_sync() {
  // DS ops of one wave complete in order; this only stops the compiler
  // moving LDS accesses across the point and drains this lane's queue.
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");  // re-read LDS after this point (no forwarding)
}

// ------------------------------------------------------------ look-back
// status word per piece: [63:62] flag (1 aggregate, 2 inclusive prefix),
// [61:0] value.  One 8-byte relaxed agent-scope granule: the data is the
// flag (cdna_hip_programming.md Guideline 16, form R2).
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagInc = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;

__device__ __forceinline__ void st_status(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_status(uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Publish a tile's aggregate as early as it is known (one lane).
__device__ __forceinline__ void lb_publish(uint64_t *status, uint32_t tile, uint64_t agg) {
  st_status(&status[tile], (tile == 0 ? kFlagInc : kFlagAgg) | agg);
}
// Called by all 64 lanes of one wave after lb_publish.  Returns the
// exclusive prefix and publishes the inclusive one.
__device__ uint64_t lb_resolve(uint64_t *status, uint32_t tile, uint64_t agg) {
  const int lane = lane_id();
  if (tile == 0) return 0;
  uint64_t excl = 0;
  int64_t top = (int64_t)tile - 1;
  uint32_t spins = 0;
  for (;;) {
    int64_t idx = top - lane;
    uint64_t v = idx >= 0 ? ld_status(&status[idx]) : kFlagInc;
    uint64_t flag = v >> 62;
    uint64_t inc = __ballot(flag == 2);
    int first = inc ? __builtin_ctzll(inc) : 64;
    uint64_t rel = first >= 63 ? ~0ull : ((2ull << first) - 1);
    uint64_t zero = __ballot(flag == 0);
    if (zero & rel) {
      // bounded spin: a predecessor that never publishes must not hang the
      // GPU (it cannot happen with in-order tickets; belt and braces)
      if (++spins > (1u << 24)) break;
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    uint64_t val = (lane <= first) ? (v & kValMask) : 0;
    // wave sum of 64-bit values
    for (int d = 32; d >= 1; d >>= 1) val += __shfl_xor(val, d, 64);
    excl += val;
    if (first < 64) break;
    top -= 64;
  }
  if (lane == 0) st_status(&status[tile], kFlagInc | (excl + agg));
  return excl;
}

// Wide form: each poll reads the 256 nearest predecessors (4 per lane), so
// the inclusive-prefix frontier advances 256 items per memory round trip
// instead of 64 -- the bound on items per second when thousands of waves
// resolve at once.
__device__ uint64_t lb_resolve_wide(uint64_t *status, uint32_t tile, uint64_t agg) {
  const int lane = lane_id();
  if (tile == 0) return 0;
  uint64_t excl = 0;
  int64_t top = (int64_t)tile - 1;
  uint32_t spins = 0;
  for (;;) {
    uint64_t v[4];
    int fi = 4;  // first inclusive among this lane's four (nearest first)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t idx = top - 4 * lane - i;
      v[i] = idx >= 0 ? ld_status(&status[idx]) : kFlagInc;
    }
#pragma unroll
    for (int i = 3; i >= 0; --i)
      if ((v[i] >> 62) == 2) fi = i;
    const uint64_t has = __ballot(fi < 4);
    const int fl = has ? __builtin_ctzll(has) : 64;
    const int firstPos = fl < 64 ? 4 * fl + __builtin_amdgcn_readlane(fi, fl) : 256;
    bool z = false;
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pos = 4 * lane + i;
      if (pos <= firstPos) {
        z = z || (v[i] >> 62) == 0;
        sum += v[i] & kValMask;
      }
    }
    if (__ballot(z)) {
      if (++spins > (1u << 24)) break;  // cannot happen with in-order tickets
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    excl += sum;
    if (firstPos < 256) break;
    top -= 256;
  }
  if (lane == 0) st_status(&status[tile], kFlagInc | (excl + agg));
  return excl;
}

// ------------------------------------------------------------ encoder
struct WordInfo {
  uint32_t lo, hi;
};

// find first set bit in [from, to) of an LDS bitmap; returns `to` if none
__device__ int bm_next(const uint32_t *bits, int from, int to) {
  if (from >= to) return to;
  int d = from >> 5;
  uint32_t m = bits[d] & (~0u << (from & 31));
  while (!m) {
    ++d;
    if (d * 32 >= to) return to;
    m = bits[d];
  }
  int p = d * 32 + __builtin_ctz(m);
  return p < to ? p : to;
}
// any set bit in [lo, hi] (inclusive)?
__device__ bool bm_any(const uint32_t *bits, int lo, int hi) {
  if (lo > hi) return false;
  int d0 = lo >> 5, d1 = hi >> 5;
  for (int d = d0; d <= d1; ++d) {
    uint32_t m = bits[d];
    if (d == d0) m &= ~0u << (lo & 31);
    if (d == d1) m &= (hi & 31) == 31 ? ~0u : ((2u << (hi & 31)) - 1);
    if (m) return true;
  }
  return false;
}

// Re-materialise a value so masks derived from it earlier cannot be kept
// alive across a phase (hipcc otherwise CSEs ~60 per-word compare masks and
// spills the SGPRs).
#define CPK_OPAQUE(x) asm volatile("" : "+v"(x))

__device__ __forceinline__ int grp_of(uint32_t m) {
  // 0 = Z (all-zero word), 1 = D/L (<= 1 zero byte), 2 = M
  return m == 0 ? 0 : __builtin_popcount(m) >= 7 ? 1 : 2;
}
__device__ __forceinline__ uint32_t word_mask(uint32_t lo, uint32_t hi) {
  return nzmask4(lo) | (nzmask4(hi) << 4);
}

// Lane-per-word encoder.  A 1024-thread workgroup holds one piece of up to
// 8192 words: wave w owns words [512w, 512w + 512) as 8 steps of 64
// consecutive words (lane = word).  Runs, run ends, "last D" and byte
// offsets are 64-bit ballot masks + mbcnt inside a step, wave-uniform carries
// across steps, and one LDS exchange across waves.
constexpr int kSteps = kTileWords / (kEncThreads);   // 8 steps of 64 words per wave

__device__ __forceinline__ uint64_t lanemask_le() {
  const int l = lane_id();
  return l == 63 ? ~0ull : ((2ull << l) - 1);
}
// highest set bit of m as a lane index (m != 0)
__device__ __forceinline__ int hi_bit(uint64_t m) { return 63 - __builtin_clzll(m); }
__device__ __forceinline__ int lo_bit(uint64_t m) { return __builtin_ctzll(m); }
// number of set bits of m below this lane
__device__ __forceinline__ int mbcnt(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ---- tiled pieces: run state carried across 8192-word tiles --------------
// A piece longer than one tile is cut into tiles that are encoded by
// different workgroups.  What a tile's roles need from before it is the state
// of the run that crosses its first word (PackedOutputStream.java:119-161):
// a zero run's phase (heads every 256 words from the run start) or a D/L
// stretch's last 0xFF head.  Each tile publishes the state at its end in
// tstate[tau] ([63:62] flag, [33:32] group, [31:0] value):
//   LOCAL  value known: Z -> (tile end - run start) mod 256; D/L -> distance
//          from the tile end back to the last head (0 = no D yet); M -> none;
//   PASS   the whole tile continues one run and maps the state through
//          unchanged (zero run: 8192 is a multiple of 256) or, all-D, to
//          min(dist, 256) -- republished as LOCAL once resolved.
// A continued tile resolves its entry state by a look-back to the nearest
// LOCAL (tile 0 of every piece is LOCAL), the pattern of lb_resolve.
constexpr uint64_t kStLocal = 1ull << 62, kStPass = 2ull << 62;
constexpr int kNoHead = -(1 << 28);

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
// first D word at or after x (< W) from the D ballots of pass 1 (mks[2q+1]
// is the D mask of 64-word step q); W if none
__device__ int enc_first_d(const uint64_t *mks, int x, int W) {
  if (x >= W) return W;
  int q = x >> 6;
  uint64_t m = mks[2 * q + 1] & (~0ull << (x & 63));
  while (!m) {
    ++q;
    if (q * 64 >= W) return W;
    m = mks[2 * q + 1];
  }
  return min(q * 64 + __builtin_ctzll(m), W);
}
// walk the head chain from the first D >= x; distance from W back to the
// last head, 0 if there is none
__device__ int enc_chain_dist(const uint64_t *mks, int x, int W) {
  int last = -1;
  int h = enc_first_d(mks, x, W);
  while (h < W) {
    last = h;
    h = enc_first_d(mks, h + 256, W);
  }
  return last >= 0 ? W - last : 0;
}
// Exit state of a full tile from its final run (start sF, -1 if the run
// covers the whole tile; group gF) or 0 when it needs the entry state (a
// tile-long D/L stretch with L words).  mks: per 64-word step {S, D} masks.
__device__ uint64_t tile_exit_state(const uint64_t *mks, int W, int gF, int sF, bool allD) {
  if (gF == 2) return kStLocal | (2ull << 32);
  if (sF >= 0)
    return kStLocal | ((uint64_t)gF << 32) |
           (gF == 0 ? (uint64_t)((-sF) & 255) : (uint64_t)enc_chain_dist(mks, sF, W));
  if (gF == 0) return kStPass;
  if (allD) return kStPass | (1ull << 32);
  return 0;
}
// Entry state by look-back over tstate (all 64 lanes of one wave): the
// nearest LOCAL state before tau, PASS tiles composed on the way.  Returns
// the Z phase (g0 == 0) or the D/L head distance (0 = none yet).
__device__ uint32_t tile_entry_state(uint64_t *tstate, uint32_t tau, int g0) {
  const int lane = lane_id();
  int64_t top = (int64_t)tau - 1;
  bool sawD = false;
  uint64_t val = 0;
  uint32_t spins = 0;
  for (;;) {
    const int64_t idx = top - lane;
    const uint64_t v = idx >= 0 ? ld_status(&tstate[idx]) : kStLocal;
    const uint64_t loc = __ballot((v >> 62) == 1);
    const int first = loc ? __builtin_ctzll(loc) : 64;
    const uint64_t rel = first >= 63 ? ~0ull : ((2ull << first) - 1);
    if (__ballot((v >> 62) == 0) & rel) {
      if (++spins > (1u << 24)) break;  // cannot happen with in-order tickets
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    sawD = sawD || __ballot(lane < first && ((v >> 32) & 1)) != 0;
    if (first < 64) {
      val = readlane64(v, first);
      break;
    }
    top -= 64;
  }
  uint32_t x = (uint32_t)val;
  if (g0 == 0) return x & 255;
  if (sawD) x = (x == 0 || x > 256) ? 256u : x;
  return x;
}

// wave 0, all lanes: publish this tile's exit state, resolve its entry state
// into scr[69..71]
__device__ void enc_tile_state(const uint64_t *mks, int *scr, uint64_t *tstate, uint32_t tau,
                               int j, int W, bool lastTile, int g0, int gm1) {
  const int lane = lane_id();
  int sF = -1;
  bool allD = true;
  for (int q = 0; q < kEncWaves; ++q) {
    sF = max(sF, scr[q]);
    allD = allD && scr[76 + q] != 0;
  }
  uint64_t outv = 0;
  if (!lastTile) {
    outv = tile_exit_state(mks, W, scr[72], sF, allD);
    if (outv && lane == 0) st_status(&tstate[tau], outv);
  }
  int rsIn = -1, hlIn = kNoHead, cont = 0;
  if (j > 0 && W > 0 && g0 == gm1) {
    cont = g0 + 1;
    if (g0 != 2) {
      const uint32_t x = tile_entry_state(tstate, tau, g0);
      if (g0 == 0) {
        rsIn = -(int)x;
        if (!lastTile && outv == kStPass && lane == 0) st_status(&tstate[tau], kStLocal | (uint64_t)x);
      } else {
        rsIn = -kTileWords;  // forces the chain walk for the continued stretch
        hlIn = x ? -(int)x : kNoHead;
        if (!lastTile && (outv >> 62) == 2 && lane == 0)
          st_status(&tstate[tau], kStLocal | (1ull << 32) | (uint64_t)((x == 0 || x > 256) ? 256u : x));
      }
    }
  }
  if (!lastTile && !outv) {
    // one D/L stretch over the whole tile, with L words: its chain goes on
    // from the entry head
    outv = kStLocal | (1ull << 32) | (uint64_t)enc_chain_dist(mks, max(hlIn + 256, 0), W);
    if (lane == 0) st_status(&tstate[tau], outv);
  }
  if (lane == 0) {
    scr[69] = rsIn;
    scr[70] = hlIn;
    scr[71] = cont;
  }
}

// info word per (step, lane): [7:0] nonzero mask, [9:8] group,
// [10] member, [11] zero-run head, [15:12] bytes, [23:16] run count,
// [24] word of a D/L stretch longer than 256 words (chain walk decides)
template <bool kTiled>
__global__ __launch_bounds__(kEncThreads, CPK_ENC_WPE) void encode_kernel(
    const uint64_t *__restrict__ in, const uint64_t *__restrict__ swo, uint32_t n,
    uint8_t *__restrict__ out, uint64_t *__restrict__ out_off, uint64_t *status,
    uint32_t *ticket, const uint32_t *__restrict__ tmap, const uint64_t *__restrict__ toff,
    uint64_t *tstate, uint32_t *err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t *stage = smem;
  uint32_t *stage32 = reinterpret_cast<uint32_t *>(smem);
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem + kEncLut);
  uint32_t *dbits = reinterpret_cast<uint32_t *>(smem + kEncDbits);
  uint32_t *hbits = reinterpret_cast<uint32_t *>(smem + kEncHbits);
  int *scr = reinterpret_cast<int *>(smem + kEncScr);
  uint64_t *mks = reinterpret_cast<uint64_t *>(smem + kEncMasks);
  // scr[0..15] last run start per wave, [16..31] first run start,
  // [32..47] last D, [48..63] bytes per wave, [64..65] ticket, [66..67] base,
  // tiled only: [68] run end after the tile, [69] run start entering it,
  // [70] last 0xFF head entering it, [71] continued group + 1, [72] group of
  // the tile's last word, [76..91] all-D flag per wave

  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  fill_luts(lut, false);
  PH_INIT(scr)

  // tiled: work item = tile tau of T (pieces cut into 8192-word tiles, in
  // stream order); otherwise work item = piece
  const uint32_t T = kTiled ? (uint32_t)toff[n] : n;
  for (uint32_t it = 0;; ++it) {
    if (tid == 0) scr[64 + (it & 1)] = (int)atomicAdd(ticket, 1u);
    __syncthreads();  // also orders the previous piece's LDS use
    const uint32_t tau = (uint32_t)__builtin_amdgcn_readfirstlane(scr[64 + (it & 1)]);
    if (tau >= T) break;
    PH(0)
    uint32_t seg = tau;
    int j = 0;             // tile index within the piece
    bool lastTile = true;  // no tile of this piece follows
    uint64_t w0, rest = 0;  // rest: words of the piece after this tile
    int W;
    if (kTiled) {
      seg = (uint32_t)__builtin_amdgcn_readfirstlane((int)tmap[tau]);
      j = (int)(tau - (uint32_t)toff[seg]);
      const uint64_t p0 = swo[seg], pw = swo[seg + 1] - p0, tb = (uint64_t)j * kTileWords;
      const uint64_t rem = pw - tb;
      w0 = p0 + tb;
      W = rem < (uint64_t)kTileWords ? (int)rem : kTileWords;
      lastTile = rem <= (uint64_t)kTileWords;
      rest = rem - (uint64_t)W;
    } else {
      w0 = swo[seg];
      const uint64_t pw = swo[seg + 1] - w0;
      if (pw > (uint64_t)kTileWords) {  // max_seg_words hint was wrong
        if (tid == 0) atomicOr(err, 1u);
      }
      W = pw > (uint64_t)kTileWords ? kTileWords : (int)pw;
    }
    // per-piece opaque copies of this wave's / lane's first word: keep hipcc
    // from hoisting ~100 per-lane addresses out of the persistent loop
    int wb = __builtin_amdgcn_readfirstlane(w * (kSteps * 64));  // first word of this wave
    asm volatile("" : "+s"(wb));
    int k0 = wb + lane;
    asm volatile("" : "+v"(k0));

    // ---- pass 1: load, classify, run-start and D masks --------------------
    uint32_t info[kSteps];
    // run-start / D ballots of each step live in LDS (wave-private rows):
    // kept in SGPRs they spilled.
    uint64_t *mrow = mks + (wb >> 9) * (2 * kSteps);
#define SMASK(s) mrow[2 * (s)]
#define DMASK(s) mrow[2 * (s) + 1]
    const uint64_t *src = in + w0;
    // all 8 loads in flight at once (clamped, not predicated: no branches)
    uint64_t wv[kSteps];
    {
      const int kl = max(W - 1, 0);
#pragma unroll
      for (int s = 0; s < kSteps; ++s) wv[s] = W ? src[min(k0 + s * 64, kl)] : 0ull;
    }
    int gprev = 3;  // group of word wb - 1 (3 = none: a run starts at word 0)
    if (lane == 0 && (w > 0 ? wb - 1 < W : j > 0)) {
      uint64_t v = src[wb - 1];
      gprev = grp_of(word_mask((uint32_t)v, (uint32_t)(v >> 32)));
    }
    gprev = readlane(gprev, 0);
    const int gm1 = gprev;  // wave 0: group of the word before the tile
    bool allD = true;
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      const int k = k0 + s * 64;
      const uint64_t v = k < W ? wv[s] : 0ull;
      const uint32_t m = word_mask((uint32_t)v, (uint32_t)(v >> 32));
      const int g = k < W ? grp_of(m) : 3;
      const int gp = wave_shr1(g, gprev);
      const uint64_t sb = __ballot(g != 3 && g != gp);
      const uint64_t db = __ballot(k < W && m == 0xffu);
      allD = allD && db == ~0ull;
      if (lane == 0) {
        SMASK(s) = sb;
        DMASK(s) = db;
      }
      gprev = readlane(g, 63);
      info[s] = m | ((uint32_t)g << 8);
    }
    {
      int ls = -kBig, fs = kBig, ld = -1;  // -kBig: no start (below any carried start)
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        const uint64_t sb = SMASK(s), db = DMASK(s);
        if (sb) {
          ls = wb + s * 64 + hi_bit(sb);
          if (fs == kBig) fs = wb + s * 64 + lo_bit(sb);
        }
        if (db) ld = wb + s * 64 + hi_bit(db);
      }
      if (lane == 0) {
        scr[w] = ls;
        scr[16 + w] = fs;
        scr[32 + w] = ld;
        if (kTiled) scr[76 + w] = allD;
      }
    }
    if (kTiled && w == kEncWaves - 1) {
      // run end after the tile (looked up to 256 words ahead: counts cap at
      // 255, stretches longer than 256 words take the chain walk anyway)
      int look = W;
      if (!lastTile) {
        uint64_t v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint64_t p = (uint64_t)(64 * r + lane);
          v[r] = p < rest ? src[W + 64 * r + lane] : 0ull;
        }
        int gp = gprev;  // group of word W - 1
        look = W + 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int g = (uint64_t)(64 * r + lane) < rest
                            ? grp_of(word_mask((uint32_t)v[r], (uint32_t)(v[r] >> 32)))
                            : 3;
          const uint64_t b = __ballot(g != wave_shr1(g, gp));
          if (b && look == W + 256) look = W + 64 * r + lo_bit(b);
          gp = readlane(g, 63);
        }
      }
      if (lane == 0) {
        scr[68] = look;
        scr[72] = gprev;
      }
    }
    __syncthreads();
    if (kTiled) {
      if (w == 0) enc_tile_state(mks, scr, tstate, tau, j, W, lastTile, readlane((int)info[0], 0) >> 8 & 3, gm1);
      __syncthreads();
    }
    PH(1)
    // carries across waves: run start / last D entering this wave, first
    // run start after it
    int cS = kTiled ? scr[69] : -1, cD = -1, eOut = kTiled ? scr[68] : W;
    for (int q = 0; q < w; ++q) {
      cS = max(cS, scr[q]);
      cD = max(cD, scr[32 + q]);
    }
    for (int q = kEncWaves - 1; q > w; --q) eOut = scr[16 + q] < kBig ? min(eOut, scr[16 + q]) : eOut;
    // first run start in steps after s (within the wave), else eOut
    int nextS[kSteps];
    {
      int r = eOut;
#pragma unroll
      for (int s = kSteps - 1; s >= 0; --s) {
        nextS[s] = r;
        const uint64_t sb = SMASK(s);
        if (sb) r = wb + s * 64 + lo_bit(sb);
      }
    }

    // ---- pass 2: roles (PackedOutputStream.java:119-193 restated per word) --
    const uint64_t le = lanemask_le();
    int anyLong = 0;
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      const int k = k0 + s * 64;
      const int base = wb + s * 64;
      const uint32_t m = info[s] & 0xffu;
      const int g = (int)((info[s] >> 8) & 3);
      const uint64_t smask_s = SMASK(s), dmask_s = DMASK(s);
      const uint64_t sm = smask_s & le;
      const int rs = sm ? base + hi_bit(sm) : cS;          // run start s(k)
      const uint64_t sg = smask_s & ~le;
      const int re = sg ? base + lo_bit(sg) : nextS[s];    // run end e(k)
      const uint64_t dm = dmask_s & (le >> 1);             // D words before k
      const int rd = dm ? base + hi_bit(dm) : cD;          // last D before k
      uint32_t x = info[s];
      int nb = 0;
      if (g == 0) {
        // every 256th word of a zero run is a 0x00 head (the 255 cap, :125-127)
        if (((k - rs) & 255) == 0) {
          x |= 1u << 11;
          nb = 2;
        }
      } else if (g == 1) {
        if (re - rs > 256) {
          anyLong = 1;  // resolved by the chain walk below
          x |= 1u << 24;  // long-stretch word
          nb = 8;       // provisional: L words are 8 either way, D fixed below
        } else if (rd >= rs) {
          x |= 1u << 10;  // inside the 0xFF run of the stretch's first D
          nb = 8;
        } else {
          nb = m == 0xffu ? 10 : 8;
        }
      } else if (g == 2) {
        nb = 1 + __builtin_popcount(m);
      }
      const uint32_t cnt = (uint32_t)min(255, max(re - k - 1, 0));
      info[s] = (x & 0x10007ffu) | ((uint32_t)nb << 12) | (cnt << 16);
      if (smask_s) cS = base + hi_bit(smask_s);
      if (dmask_s) cD = base + hi_bit(dmask_s);
      __builtin_amdgcn_sched_barrier(0);
    }
    PH(2)
    if (__syncthreads_or(anyLong)) {
      // D/L stretch longer than 256 words: heads chain h1 = first D,
      // h' = first D at or after h + 256 (PackedOutputStream.java:145-161).
      if (tid < 256) dbits[tid] = 0;
      else if (tid < 512) hbits[tid - 256] = 0;
      __syncthreads();
      // bitmaps are built from the ballots: lane 0 / 1 write 32-bit halves
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        const int dw = (wb + s * 64) >> 5;
        if (lane == 0) {
          dbits[dw] = (uint32_t)DMASK(s);
          // a stretch continued from the previous tile: a start marker at 0
          hbits[dw] = (uint32_t)SMASK(s) | (kTiled && dw == 0 && scr[71] == 2 ? 1u : 0u);
        } else if (lane == 1) {
          dbits[dw + 1] = (uint32_t)(DMASK(s) >> 32);
          hbits[dw + 1] = (uint32_t)(SMASK(s) >> 32);
        }
      }
      __syncthreads();
      // run start of every long-stretch word, then clear hbits for heads
      int sl[kSteps];
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        sl[s] = 0;
        const int k = k0 + s * 64;
        if ((info[s] >> 24) & 1) {
          int d = k >> 5;
          uint32_t mm = hbits[d] & ((k & 31) == 31 ? ~0u : ((2u << (k & 31)) - 1));
          while (!mm) mm = hbits[--d];
          sl[s] = d * 32 + 31 - __builtin_clz(mm);
          if (kTiled && sl[s] == 0 && scr[71] == 2) sl[s] = -kTileWords;  // continued stretch
        }
      }
      __syncthreads();
      if (tid < 256) hbits[tid] = 0;
      __syncthreads();
      // walkers: the first word of each long stretch
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        const int k = k0 + s * 64;
        const int base = wb + s * 64;
        const uint64_t sg = SMASK(s) & ~lanemask_le();
        const int re = sg ? base + lo_bit(sg) : nextS[s];
        const bool st = (SMASK(s) >> lane) & 1;
        if (st && ((info[s] >> 8) & 3) == 1 && re - k > 256) {
          const int rw = min(re, W);
          int h = bm_next(dbits, k, rw);
          while (h < rw) {
            atomicOr(&hbits[h >> 5], 1u << (h & 31));
            const int p = h + 256;
            if (p >= rw) break;
            h = bm_next(dbits, p, rw);
          }
        }
      }
      if (kTiled && tid == 0 && scr[71] == 2) {
        // the continued stretch: its chain goes on from the last head of the
        // previous tile, h' = first D >= h + 256 (PackedOutputStream.java:145-161)
        int rw = scr[68];
        for (int q = 0; q < kEncWaves; ++q) rw = scr[16 + q] < kBig ? min(rw, scr[16 + q]) : rw;
        rw = min(rw, W);
        int h = bm_next(dbits, max(scr[70] + 256, 0), rw);
        while (h < rw) {
          atomicOr(&hbits[h >> 5], 1u << (h & 31));
          const int p = h + 256;
          if (p >= rw) break;
          h = bm_next(dbits, p, rw);
        }
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        const int k = k0 + s * 64;
        const uint32_t m = info[s] & 0xffu;
        if ((info[s] >> 24) & 1) {
          // member iff a head of its stretch lies in [k - 255, k - 1]
          bool mem = bm_any(hbits, max(max(sl[s], k - 255), 0), k - 1);
          if (kTiled && sl[s] < 0) mem = mem || k - 255 <= scr[70];
          const int nb = mem ? 8 : (m == 0xffu ? 10 : 8);
          info[s] = (info[s] & ~(0xfu << 12)) | ((uint32_t)nb << 12) | (mem ? (1u << 10) : 0u);
        }
      }
    }
    PH(3)

    // ---- bytes per wave -> piece offsets -----------------------------------
    {
      int tot = 0;
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        const uint32_t nb = (info[s] >> 12) & 15u;
        tot += __popcll(__ballot(nb & 1)) + 2 * __popcll(__ballot(nb & 2)) +
               4 * __popcll(__ballot(nb & 4)) + 8 * __popcll(__ballot(nb & 8));
      }
      if (lane == 0) scr[48 + w] = tot;
    }
    __syncthreads();
    int wbytes = 0, total = 0;
    for (int q = 0; q < kEncWaves; ++q) {
      const int t = scr[48 + q];
      if (q < w) wbytes += t;
      total += t;
    }
    // publish the aggregate now; the prefix is resolved after compaction
    if (tid == 0) lb_publish(status, tau, (uint64_t)total);
    // zero the staging lines this piece uses (the strings are OR-ed in)
    {
      const int nl = (total + 19) >> 4;
      uint4 z = {0u, 0u, 0u, 0u};
      for (int c = tid; c < nl; c += kEncThreads) reinterpret_cast<uint4 *>(stage)[c] = z;
    }
    __syncthreads();
    PH(4)

    // ---- pass 3: packed strings into LDS ------------------------------------
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      const uint32_t x = info[s];
      const uint32_t nb = (x >> 12) & 15u;
      const uint64_t b0 = __ballot(nb & 1), b1 = __ballot(nb & 2), b2 = __ballot(nb & 4),
                     b3 = __ballot(nb & 8);
      const int o = wbytes + mbcnt(b0) + 2 * mbcnt(b1) + 4 * mbcnt(b2) + 8 * mbcnt(b3);
      wbytes += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2) + 8 * __popcll(b3);
      if (nb == 0) continue;
      // the words are re-read here (L2 / Infinity-Cache hit) instead of being
      // held in 16 VGPRs across the passes: 2 workgroups per CU instead of 1
      const uint64_t v = src[k0 + s * 64];
      const uint32_t l = (uint32_t)v, h = (uint32_t)(v >> 32), m = x & 0xffu;
      uint32_t d0, d1, d2;
      if (x & (1u << 10)) {  // literal-run member: 8 bytes verbatim
        d0 = l;
        d1 = h;
        d2 = 0;
      } else {  // tag + nonzero bytes (+ count after 0x00 / 0xFF tags)
        const uint64_t sel = lut[m];
        const uint32_t c0 = __builtin_amdgcn_perm(h, l, (uint32_t)sel);
        const uint32_t c1 = __builtin_amdgcn_perm(h, l, (uint32_t)(sel >> 32));
        const uint32_t cnt = (x >> 16) & 0xffu;
        d0 = m | (c0 << 8);
        d1 = (c0 >> 24) | (c1 << 8);
        d2 = c1 >> 24;
        if (m == 0) d0 |= cnt << 8;
        else if (m == 0xffu) d2 |= cnt << 8;
      }
      // place bytes [o, o + nb): dword-shift the 3-dword string
      const uint32_t sh = (uint32_t)(o & 3) * 8u;
      const uint64_t s01 = (uint64_t)d0 | ((uint64_t)d1 << 32);
      const uint64_t lo64 = s01 << sh;
      const uint64_t hi64 = ((uint64_t)d2 << sh) | (sh ? (s01 >> (64 - sh)) : 0ull);
      uint32_t *dst = stage32 + (o >> 2);
      // four unconditional ORs into the zeroed stage (the bytes past the
      // string are zero): no exec-mask branches around the LDS ops
      atomicOr(&dst[0], (uint32_t)lo64);
      atomicOr(&dst[1], (uint32_t)(lo64 >> 32));
      atomicOr(&dst[2], (uint32_t)hi64);
      atomicOr(&dst[3], (uint32_t)(hi64 >> 32));
      __builtin_amdgcn_sched_barrier(0);  // one step at a time: bounds VGPRs
    }
    PH(5)

    // ---- decoupled look-back (wave 0), overlapped with the compaction -----
    if (w == 0) {
      uint64_t b = lb_resolve(status, tau, (uint64_t)total);
      if (lane == 0) {
        *reinterpret_cast<uint64_t *>(&scr[66]) = b;
        if (j == 0) out_off[seg] = b;
        if (tau == T - 1) out_off[n] = b + (uint64_t)total;
      }
    }
    __syncthreads();
    PH(6)
    // ---- store: 16-byte lines, byte stores at the two shared edges --------
    // staged byte x is global byte base + x; line L covers global
    // [A + 16L, A + 16L + 16), A = base & ~15, i.e. staged x = 16L - pad.
    {
      const uint64_t base = *reinterpret_cast<uint64_t *>(&scr[66]);
      const int pad = (int)(base & 15);
      const int tb = pad + total;
      uint8_t *gbase = out + (base - (uint64_t)pad);
      const int nl = (tb + 15) >> 4;
      const uint32_t sh = (uint32_t)((16 - pad) & 3);  // (16L - pad) & 3
      for (int c = tid; c < nl; c += kEncThreads) {
        const int lo16 = c * 16, hi16 = lo16 + 16;
        if (lo16 >= pad && hi16 <= tb) {
          const uint32_t *a = stage32 + ((lo16 - pad) >> 2);
          uint32_t e0 = a[0], e1 = a[1], e2 = a[2], e3 = a[3], e4 = sh ? a[4] : 0u;
          uint4 v;
          v.x = __builtin_amdgcn_alignbyte(e1, e0, sh);
          v.y = __builtin_amdgcn_alignbyte(e2, e1, sh);
          v.z = __builtin_amdgcn_alignbyte(e3, e2, sh);
          v.w = __builtin_amdgcn_alignbyte(e4, e3, sh);
          *reinterpret_cast<uint4 *>(gbase + lo16) = v;
        } else {
          const int bb0 = max(lo16, pad), bb1 = min(hi16, tb);
          for (int b = bb0; b < bb1; ++b) gbase[b] = stage[b - pad];
        }
      }
    }
    PH(7)
#undef SMASK
#undef DMASK
  }
  PH_FLUSH(0)
}

// ------------------------------------------------------------ encoder v2
// Wave-per-tile encoder: no workgroup barriers.  A wave takes the next tile
// (1024 words of a piece, in stream order) from an ordered ticket and
//   1. loads its words (one per lane per 64-word step) and classifies them:
//      nonzero-byte mask, group, run-start / D ballots (a wave-private LDS
//      row per step), plus a 256-word look-ahead for the end of the run
//      crossing the tile end;
//   2. publishes its exit run state (tile_exit_state) and, when its first
//      run continues the previous tile's, resolves its entry state;
//   3. walks the 16 steps in order with wave-uniform carries -- run start,
//      last D, last 0xFF head of the current stretch -- and gives every word
//      its role (PackedOutputStream.java:64-193 restated per word, see
//      DESIGN.md): within one 64-word step a stretch that continues from
//      before has at most one new head (heads are >= 256 words apart) and a
//      stretch that starts in the step has its first D as head;
//   4. publishes its packed size and resolves its output offset by
//      decoupled look-back;
//   5. builds each word's packed string (tag + v_perm-compacted bytes +
//      count), ORs it into a 1 KiB wave-private LDS ring at its output
//      offset, and streams complete 16-byte lines to memory; only the lines
//      shared with the neighbouring tiles take byte stores.
// Per-word state lives in LDS between the passes (rolled loops keep the
// registers at <= 64 per lane).
constexpr int kE2Words = 1024;                 // words per tile (multiple of 256)
constexpr int kE2Steps = kE2Words / 64;        // 16
constexpr int kE2Threads = 256;                // 4 independent waves
constexpr uint32_t kE2Ring = 1024;             // output ring per wave (bytes)
constexpr uint32_t kE2Info = kE2Ring;                      // u32[16][64] per-word roles
constexpr uint32_t kE2Mks = kE2Info + kE2Words * 4;        // u64[16][2] {S, D}
constexpr uint32_t kE2Nxs = kE2Mks + kE2Steps * 16;        // int[16] first start after step
constexpr uint32_t kE2WaveLds = kE2Nxs + kE2Steps * 4;     // 5,440
constexpr uint32_t kE2Lds = 2048 + 4 * kE2WaveLds;         // 23,808 B
#ifndef CPK_E2_WPE
#define CPK_E2_WPE 6  // LDS (23.8 KB per workgroup) allows 6 workgroups per CU
#endif

// stores bytes [lo, hi) of global line L from the ring, then clears them
__device__ __forceinline__ void e2_store_partial(uint8_t *out, uint8_t *ring, uint64_t L, int lo,
                                                 int hi) {
  const int lane = lane_id();
  if (lane >= lo && lane < hi) {
    const uint32_t rp = (uint32_t)((L * 16 + lane) & (kE2Ring - 1));
    out[L * 16 + lane] = ring[rp];
    ring[rp] = 0;
  }
}

__global__ __launch_bounds__(kE2Threads, CPK_E2_WPE) void encode2_kernel(
    const uint64_t *__restrict__ in, const uint64_t *__restrict__ swo, uint32_t n,
    uint8_t *__restrict__ out, uint64_t *__restrict__ out_off, uint64_t *status,
    uint32_t *ticket, const uint32_t *__restrict__ tmap, const uint64_t *__restrict__ toff,
    uint64_t *tstate) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem);
  const int lane = lane_id(), w = wave_id();
  uint8_t *wl = smem + 2048 + w * kE2WaveLds;
  uint8_t *ring = wl;
  uint32_t *ring32 = reinterpret_cast<uint32_t *>(ring);
  uint32_t *inf = reinterpret_cast<uint32_t *>(wl + kE2Info);  // [s * 64 + lane]
  uint64_t *mks = reinterpret_cast<uint64_t *>(wl + kE2Mks);   // [2s] S, [2s+1] D
  int *nxs = reinterpret_cast<int *>(wl + kE2Nxs);
  fill_luts(lut, false);
  for (int i = lane; i < (int)(kE2Ring / 16); i += 64)
    reinterpret_cast<uint4 *>(ring)[i] = uint4{0u, 0u, 0u, 0u};
  __syncthreads();  // the only block-wide barrier: LUT ready
  const uint32_t T = (uint32_t)toff[n];
  // ordered tickets; the next one is requested while the current tile runs
  uint32_t tnext = take_ordered(ticket);
  WPH_INIT
  for (;;) {
    const uint32_t tau = tnext;
    if (tau >= T) break;
    tnext = take_ordered(ticket);
    const uint32_t seg = (uint32_t)__builtin_amdgcn_readfirstlane((int)tmap[tau]);
    const int j = (int)(tau - (uint32_t)toff[seg]);
    const uint64_t p0 = swo[seg], pw = swo[seg + 1] - p0;
    const uint64_t tb = (uint64_t)j * kE2Words, rem = pw - tb;
    const int W = rem < (uint64_t)kE2Words ? (int)rem : kE2Words;
    const bool lastTile = rem <= (uint64_t)kE2Words;
    const int rl = (int)min(rem - (uint64_t)W, (uint64_t)256);  // look-ahead words
    const uint64_t *src = in + p0 + tb;
    int k0 = lane;
    asm volatile("" : "+v"(k0));  // keep per-lane addresses out of the loop head
    const int kl = max(W - 1, 0);
    WPH(0)

    // ---- 1: loads, classes, ballots ----------------------------------------
    int gm1 = 3;  // group of the word before the tile (3: none)
    if (j > 0) {
      const uint64_t v = src[-1];
      gm1 = grp_of(word_mask((uint32_t)v, (uint32_t)(v >> 32)));
    }
    int gprev = gm1, sF = -1;
    bool allD = true;
    {
      uint64_t wv[kE2Steps];
#pragma unroll
      for (int s = 0; s < kE2Steps; ++s) wv[s] = W ? src[min(k0 + 64 * s, kl)] : 0ull;
#pragma unroll
      for (int s = 0; s < kE2Steps; ++s) {
        const int k = k0 + 64 * s;
        const uint64_t v = k < W ? wv[s] : 0ull;
        const uint32_t m = word_mask((uint32_t)v, (uint32_t)(v >> 32));
        const int g = k < W ? grp_of(m) : 3;
        const uint64_t S = __ballot(g != 3 && g != wave_shr1(g, gprev));
        const uint64_t D = __ballot(k < W && m == 0xffu);
        if (lane == 0) {
          mks[2 * s] = S;
          mks[2 * s + 1] = D;
        }
        allD = allD && D == ~0ull;
        if (S) sF = 64 * s + hi_bit(S);
        gprev = readlane(g, 63);
        inf[64 * s + lane] = m | ((uint32_t)g << 8);
      }
    }
    const int gF = gprev;  // group of word 1023 (full tiles)
    int look = W;          // first run start after the tile, capped 256 on
    if (!lastTile) {
      uint64_t la[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) la[r] = src[W + min(64 * r + k0, rl - 1)];
      look = W + 256;
      int gp = gprev;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int g = 64 * r + lane < rl ? grp_of(word_mask((uint32_t)la[r], (uint32_t)(la[r] >> 32))) : 3;
        const uint64_t b = __ballot(g != wave_shr1(g, gp));
        if (b && look == W + 256) look = W + 64 * r + lo_bit(b);
        gp = readlane(g, 63);
      }
    }
    wave_lds_sync();
    // nxs[s] := first run start after step s
    if (lane == 0) {
      int r = look;
      for (int s = kE2Steps - 1; s >= 0; --s) {
        nxs[s] = r;
        const uint64_t S = mks[2 * s];
        if (S) r = 64 * s + lo_bit(S);
      }
    }

    // ---- 2: exit state out, entry state in ----------------------------------
    WPH(1)
    uint64_t outv = 0;
    if (!lastTile) {
      outv = tile_exit_state(mks, W, gF, sF, allD);
      if (outv && lane == 0) st_status(&tstate[tau], outv);
    }
    const int g0 = __builtin_amdgcn_readfirstlane((int)inf[0]) >> 8 & 3;
    const bool cont = j > 0 && W > 0 && g0 == gm1;
    int rsC = 0, hC = kNoHead;  // run start / last 0xFF head before the step
    if (cont && g0 != 2) {
      const uint32_t x = tile_entry_state(tstate, tau, g0);
      if (g0 == 0) {
        rsC = -(int)x;
        if (!lastTile && outv == kStPass && lane == 0) st_status(&tstate[tau], kStLocal | (uint64_t)x);
      } else {
        hC = x ? -(int)x : kNoHead;
        if (!lastTile && (outv >> 62) == 2 && lane == 0)
          st_status(&tstate[tau], kStLocal | (1ull << 32) | (uint64_t)((x == 0 || x > 256) ? 256u : x));
      }
    }
    if (!lastTile && !outv) {
      outv = kStLocal | (1ull << 32) | (uint64_t)enc_chain_dist(mks, max(hC + 256, 0), W);
      if (lane == 0) st_status(&tstate[tau], outv);
    }
    wave_lds_sync();

    // ---- 3: roles (PackedOutputStream.java:64-193 per word) -----------------
    WPH(2)
    const uint64_t le = lanemask_le(), lt = le >> 1;
    int gC = gm1, rdC = -kBig, total = 0;
#pragma unroll 1
    for (int s = 0; s < kE2Steps; ++s) {
      const int base = 64 * s;
      const int k = k0 + base;
      const uint64_t S = mks[2 * s], D = mks[2 * s + 1];
      const int nx = nxs[s];
      const uint32_t x = inf[base + lane];
      const uint32_t m = x & 0xffu;
      const int g = (int)((x >> 8) & 3);
      const int fst = S ? lo_bit(S) : 64;  // first run start in the step
      // the D/L stretch continuing into the step: its new head, if any, is
      // the first D at or after hC + 256 before the step's first run start
      int hNew = kNoHead;
      if (gC == 1 && fst > 0) {
        const int t0 = hC == kNoHead ? 0 : max(hC + 256 - base, 0);
        if (t0 < fst) {
          const uint64_t sg = (fst == 64 ? ~0ull : ((1ull << fst) - 1)) & (~0ull << t0);
          const uint64_t c = D & sg;
          if (c) hNew = base + lo_bit(c);
        }
      }
      const uint64_t sle = S & le, sgt = S & ~le, dlt = D & lt;
      const int rs = sle ? base + hi_bit(sle) : rsC;
      const int re = sgt ? base + lo_bit(sgt) : nx;
      const int rd = dlt ? base + hi_bit(dlt) : rdC;
      uint32_t flags = 0;
      int nb = 0;
      if (g == 0) {
        // a 0x00 head every 256 words of a zero run (the 255 cap, :119-131)
        if (((k - rs) & 255) == 0) {
          flags = 1u << 11;
          nb = 2;
        }
      } else if (g == 1) {
        bool mem;
        if (lane < fst) {  // stretch continuing from before the step
          mem = k != hNew && ((hC != kNoHead && k <= hC + 255) || (hNew != kNoHead && k > hNew));
        } else {           // stretch started in this step: its first D heads
          mem = rd >= rs;
        }
        flags = mem ? (1u << 10) : 0u;
        nb = mem ? 8 : (m == 0xffu ? 10 : 8);
      } else if (g == 2) {
        nb = 1 + __builtin_popcount(m);
      }
      const uint32_t cnt = (uint32_t)min(255, max(re - k - 1, 0));
      inf[base + lane] = m | flags | ((uint32_t)nb << 12) | (cnt << 16);
      total += __popcll(__ballot(nb & 1)) + 2 * __popcll(__ballot(nb & 2)) +
               4 * __popcll(__ballot(nb & 4)) + 8 * __popcll(__ballot(nb & 8));
      // carries into the next step
      const int gL = readlane(g, 63);
      if (gL == 1) {
        if (S) {
          const uint64_t dm = D & (~0ull << hi_bit(S));
          hC = dm ? base + lo_bit(dm) : kNoHead;
        } else if (hNew != kNoHead) {
          hC = hNew;
        }
      } else {
        hC = kNoHead;
      }
      if (S) rsC = base + hi_bit(S);
      if (D) rdC = base + hi_bit(D);
      gC = gL;
    }

    // ---- 4: output offset by look-back --------------------------------------
    WPH(3)
    if (lane == 0) lb_publish(status, tau, (uint64_t)total);
    const uint64_t obase = lb_resolve(status, tau, (uint64_t)total);
    if (lane == 0) {
      if (j == 0) out_off[seg] = obase;
      if (tau == T - 1) out_off[n] = obase + (uint64_t)total;
    }
    wave_lds_sync();

    // ---- 5: strings -> LDS ring -> 16-byte lines ---------------------------
    WPH(4)
    const int pad = (int)(obase & 15);
    const uint64_t L0 = obase >> 4;
    uint64_t fl = (obase + 15) >> 4;  // next whole line to store
    bool headDone = pad == 0;
    int off = 0;
    // the words again (L2 / Infinity-Cache hits: the tile was read moments
    // ago), one step ahead
    uint64_t vn = W ? src[min(k0, kl)] : 0ull;
#pragma unroll 1
    for (int s = 0; s < kE2Steps; ++s) {
      const uint64_t v = vn;
      if (s + 1 < kE2Steps) vn = W ? src[min(k0 + 64 * (s + 1), kl)] : 0ull;
      const uint32_t x = inf[64 * s + lane];
      const int nb = (int)((x >> 12) & 15u);
      const int incl = wave_incl_add(nb);
      const int o = off + incl - nb;
      off += readlane(incl, 63);
      if (nb) {
        const uint32_t l = (uint32_t)v, h = (uint32_t)(v >> 32), m = x & 0xffu;
        uint32_t d0, d1, d2;
        if (x & (1u << 10)) {  // literal-run member: 8 bytes verbatim
          d0 = l;
          d1 = h;
          d2 = 0;
        } else {  // tag + nonzero bytes (+ count after 0x00 / 0xFF tags)
          const uint64_t sel = lut[m];
          const uint32_t c0 = __builtin_amdgcn_perm(h, l, (uint32_t)sel);
          const uint32_t c1 = __builtin_amdgcn_perm(h, l, (uint32_t)(sel >> 32));
          const uint32_t cnt = (x >> 16) & 0xffu;
          d0 = m | (c0 << 8);
          d1 = (c0 >> 24) | (c1 << 8);
          d2 = c1 >> 24;
          if (m == 0) d0 |= cnt << 8;
          else if (m == 0xffu) d2 |= cnt << 8;
        }
        const uint32_t rp = (uint32_t)((obase + (uint64_t)o) & (kE2Ring - 1));
        const uint32_t sh = (rp & 3) * 8u;
        const uint64_t s01 = (uint64_t)d0 | ((uint64_t)d1 << 32);
        const uint64_t lo64 = s01 << sh;
        const uint64_t hi64 = ((uint64_t)d2 << sh) | (sh ? (s01 >> (64 - sh)) : 0ull);
        const uint32_t q = rp >> 2;
        const int end = (int)(rp & 3) + nb;
        constexpr uint32_t kMask = kE2Ring / 4 - 1;
        atomicOr(&ring32[q], (uint32_t)lo64);
        if (end > 4) atomicOr(&ring32[(q + 1) & kMask], (uint32_t)(lo64 >> 32));
        if (end > 8) atomicOr(&ring32[(q + 2) & kMask], (uint32_t)hi64);
        if (end > 12) atomicOr(&ring32[(q + 3) & kMask], (uint32_t)(hi64 >> 32));
      }
      wave_lds_sync();
      if (!headDone && off >= 16 - pad) {
        e2_store_partial(out, ring, L0, pad, 16);
        headDone = true;
      }
      const uint64_t le16 = (obase + (uint64_t)off) >> 4;  // lines below are complete
      for (uint64_t L = fl + (uint64_t)lane; L < le16; L += 64) {
        uint4 *rl4 = reinterpret_cast<uint4 *>(ring + ((L * 16) & (kE2Ring - 1)));
        *reinterpret_cast<uint4 *>(out + L * 16) = *rl4;
        *rl4 = uint4{0u, 0u, 0u, 0u};
      }
      if (le16 > fl) fl = le16;
      wave_lds_sync();
    }
    // the tail line (shared with the next tile) and a head line never filled
    const uint64_t done = obase + (uint64_t)total;
    if (!headDone) {
      if (total) e2_store_partial(out, ring, L0, pad, pad + total);
    } else if (done & 15) {
      e2_store_partial(out, ring, done >> 4, 0, (int)(done & 15));
    }
    wave_lds_sync();
    WPH(5)
  }
  WPH_FLUSH(32)
}

// Tile plan for the tiled encoder: toff[i] = first tile of piece i (one tile
// per 8192 words, at least one per piece), toff[n] = T, tmap[tau] = piece of
// tile tau.  Single pass: 8192 pieces per workgroup, in ticket order, block
// prefixes by look-back.  Tiles beyond `cap` (a wrong max_seg_words hint) are
// reported in *err and not planned.
constexpr int kPlanThreads = 1024, kPlanPer = 8;
template <int kTW>
__global__ __launch_bounds__(kPlanThreads) void tile_plan_kernel(
    const uint64_t *__restrict__ swo, uint32_t n, uint64_t *__restrict__ toff,
    uint32_t *__restrict__ tmap, uint64_t cap, uint64_t *pstatus, uint32_t *ticket,
    uint32_t *err) {
  __shared__ int wsum[kPlanThreads / 64];
  __shared__ uint32_t blk_s;
  __shared__ uint64_t base_s;
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  if (tid == 0) blk_s = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t blk = blk_s;
  const uint64_t i0 = (uint64_t)blk * (kPlanThreads * kPlanPer) + (uint64_t)tid * kPlanPer;
  int c[kPlanPer];
  int t = 0;
#pragma unroll
  for (int q = 0; q < kPlanPer; ++q) {
    const uint64_t i = i0 + q;
    c[q] = 0;
    if (i < n) {
      const uint64_t pw = swo[i + 1] - swo[i];
      c[q] = pw == 0 ? 1 : (int)((pw + kTW - 1) / kTW);
    }
    t += c[q];
  }
  const int incl = wave_incl_add(t);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int wex = 0, tot = 0;
  for (int q = 0; q < kPlanThreads / 64; ++q) {
    if (q < w) wex += wsum[q];
    tot += wsum[q];
  }
  if (tid == 0) lb_publish(pstatus, blk, (uint64_t)tot);
  if (w == 0) {
    const uint64_t b = lb_resolve(pstatus, blk, (uint64_t)tot);
    if (lane == 0) base_s = b;
  }
  __syncthreads();
  uint64_t o = base_s + (uint64_t)(wex + incl - t);
#pragma unroll
  for (int q = 0; q < kPlanPer; ++q) {
    const uint64_t i = i0 + q;
    if (i < n) {
      toff[i] = o;
      for (int k = 0; k < c[q]; ++k) {
        if (o + k < cap) tmap[o + k] = (uint32_t)i;
        else atomicOr(err, 2u);
      }
      if (i == n - 1) toff[n] = o + c[q] < cap ? o + c[q] : cap;
      o += c[q];
    }
  }
}

// ------------------------------------------------------------ decoder
// Wave-per-piece decoder.  Each wave owns one piece at a time and consumes
// its packed bytes in windows of 64 chunks starting at a known tag position e:
//   1. lane l walks its chunk [e + Cl, e + Cl + C) from the chunk start,
//      speculatively treating it as a tag; visited positions form a bit mask
//      per lane, and the walk tallies its output words;
//   2. from its exit, each lane walks on until it lands on a position its
//      owner visited (the two walks coincide from there: the tag chain is a
//      function of the position);
//   3. the lanes reachable from lane 0 (whose chunk starts at the true tag e)
//      under "lane -> owner of its landing point" hold every true record
//      (pointer doubling);
//   4. on-path lanes' word counts -> wave scan; they re-walk their true
//      records to check the reference's error conditions and write, for
//      every 4-word output block, the record covering it; all 64 lanes then
//      gather-expand the blocks (PackedInputStream.java:82-134 per word).
// No barriers: up to 32 pieces in flight per CU.
constexpr int kDecThreads = 256;               // 4 independent waves
#ifndef CPK_DEC_WPE
#define CPK_DEC_WPE 8  // workgroups per CU the register budget is sized for
#endif
#ifndef CPK_DEC_CHUNK
#define CPK_DEC_CHUNK 48
#endif
// Lane chunks C of 48 bytes (3 KiB windows, 6 workgroups per CU by LDS):
// measured against 28 / 32 / 64 at 131,072 pieces, 48 is fastest on configs
// 2 and 3 (config 2 decode 5.07 -> 4.82 ms), 6 % slower on the sparse config 4
constexpr uint32_t kDecChunk = CPK_DEC_CHUNK;
constexpr uint32_t kWin = 64 * kDecChunk;         // packed bytes resolved per window
constexpr uint32_t kWinBuf = (kWin + 15 + 32 + 16 + 15) & ~15u;  // + pad, look-ahead, slack
#ifndef CPK_DEC_ROUND
#define CPK_DEC_ROUND 1280  // (8 workgroups per CU with 48-byte chunks; larger rounds cost occupancy)
#endif
constexpr int kRound = CPK_DEC_ROUND;  // output words expanded per round
#ifndef CPK_DEC_BLK
#define CPK_DEC_BLK 4  // (4: 64 lanes cover a window's blocks in fewer, fuller passes; measured faster than 8)
#endif
constexpr int kBlk = CPK_DEC_BLK;  // output words per expansion block
// a lane's visited positions: one bit per chunk byte
typedef std::conditional<(kDecChunk <= 32), uint32_t, uint64_t>::type VisMask;
static_assert(kDecChunk <= 64, "visited mask bits");
// the visited masks (phases 1-3) and the block map (phase 5) share LDS
constexpr uint32_t kDecWaveLds = kWinBuf + (4 * (kRound / kBlk) > 64 * sizeof(VisMask)
                                                ? 4 * (kRound / kBlk)
                                                : 64 * sizeof(VisMask));
constexpr int kWinLinesPerLane = (int)((kWin + 47 + 15) / 16 + 63) / 64;
constexpr uint32_t kDecLds = 2048 + 4 * kDecWaveLds;                // 15,616

__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
  return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d, 64));
  return v;
}

// The record whose tag is at piece position q: its byte length and output
// words (PackedInputStream.java:82-134).  The tag and both possible count
// bytes are read together: one LDS round trip per record on the walks.
struct DecRec {
  uint32_t len, nw;
};
__device__ __forceinline__ DecRec rec_at(const uint8_t *pkw, uint32_t q) {
  const uint32_t tag = pkw[q], c1 = pkw[q + 1], c9 = pkw[q + 9];
  // masks, not nested selects (hipcc turns those into exec-mask branches)
  const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
  DecRec r;
  r.len = 1u + __builtin_popcount(tag) + (zm & 1u) + (fm & (8u * c9 + 1u));
  r.nw = 1u + (zm & c1) + (fm & c9);
  return r;
}

// 8 bytes at piece position x: from the LDS window when loaded, otherwise
// (tail of a literal run reaching past the window) straight from memory
__device__ __forceinline__ uint64_t read8(const uint8_t *pkw, uint32_t x, uint32_t lend,
                                         const uint8_t *gpiece, uint32_t glim, uint32_t ph,
                                         uint32_t e) {
  // The LDS read is unconditional (position clamped to the window start e,
  // which has 12 buffer bytes after it whatever the window's size): with
  // both reads under one branch hipcc merged them into flat loads.
  // LDS-aligned dwords: piece position x sits at byte phase (x + ph) & 3 of
  // the 16-byte aligned window buffer.
  const bool inw = x + 12 <= lend;
  const uint32_t xl = inw ? x : e;
  uint32_t sh = (xl + ph) & 3;
  const uint32_t *pl = reinterpret_cast<const uint32_t *>(pkw + ((int64_t)xl - sh));  // (signed: xl < sh)
  uint32_t d0 = pl[0], d1 = pl[1], d2 = pl[2];
  if (!inw) {
    // address-aligned dwords of the packed buffer, none at or past the
    // readable limit glim (piece-relative: the piece's end rounded up to a
    // 16-byte line; bytes there are never part of a valid record)
    sh = (uint32_t)(reinterpret_cast<uintptr_t>(gpiece + x) & 3);
    const uint32_t *p = reinterpret_cast<const uint32_t *>(gpiece + ((int64_t)x - sh));  // (stays global)
    const int64_t xa = (int64_t)x - sh;  // piece position of p[0] (>= -3: the
    d0 = xa < glim ? p[0] : 0u;           // bytes before the piece are the buffer's)
    d1 = xa + 4 < glim ? p[1] : 0u;
    d2 = (sh && xa + 8 < glim) ? p[2] : 0u;
  }
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// kStream = false: piece i's packed bytes are [in_off[i], in_off[i+1]) and a
//   piece that fills before its range ends is CPK_ETRAILING.
// kStream = true: packed streams, each a wave's: the pieces of stream j,
//   [spc[j], spc[j+1]), are decoded back to back from its bytes
//   [sbeg[j], send[j]); each read() fills its piece and leaves the rest of
//   the stream to the next (PackedInputStream.java:35-140 as Serialize.read
//   calls it, Serialize.java:165-175).  in_off[piece] is written with the
//   piece's start and send_out[j] with the stream's end.  sbeg == nullptr:
//   one stream, pieces 0..n-1, bytes [0, avail).
struct DecStreams {
  const uint64_t *sbeg, *send, *spc;
  uint32_t ns;
  uint64_t *send_out;
};
template <bool kStream>
__global__ __launch_bounds__(kDecThreads, CPK_DEC_WPE) void decode_kernel(
    const uint8_t *__restrict__ packed, uint64_t *__restrict__ in_off,
    const uint64_t *__restrict__ swo, uint32_t n, uint64_t *__restrict__ out,
    int32_t *__restrict__ status, uint32_t *ticket, uint64_t avail, DecStreams sd) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem);
  const int lane = lane_id(), w = wave_id();
  uint8_t *wl = smem + 2048 + w * kDecWaveLds;
  uint8_t *wbuf = wl;                                            // window bytes
  uint32_t *blk = reinterpret_cast<uint32_t *>(wl + kWinBuf);    // [256]
  VisMask *visa = reinterpret_cast<VisMask *>(blk);  // [64], over the block map
  fill_luts(lut, true);
  __syncthreads();  // the only block-wide barrier: LUT ready
  int xq = xcc_id(), dry = 0;
  WPH_INIT
  uint64_t scur = 0;      // stream mode: start of the next piece
  uint64_t slim = avail;  //   end of the stream's bytes
  int sfail = CPK_OK;     //   a failed piece stops the stream
  uint32_t snext = 0, sende = 0, sj = 0;  // next piece, end of the stream's pieces, stream

  for (uint32_t sidx = 0;; ++sidx) {
    // every branch below is on wave-uniform (SGPR) values: the compiler
    // must not turn the piece / window loops into divergent loops
    // All 64 lanes add 1 (hipcc folds it into one +64 atomic): no lane-0-only
    // branch at the loop head, which hipcc otherwise structurised into a
    // divergent loop re-running piece 0.  Tickets count in units of 64.
    uint32_t seg = sidx;
    if (!kStream) {
      for (;;) {
        seg = take_ticket(ticket, xq);
        if (seg < n || ++dry >= 8) break;
        xq = (xq + 1) & 7;  // this counter ran dry: help the next one
      }
    } else {
      // the next stream with pieces (empty streams end where they begin)
      bool more = true;
      while (snext >= sende) {
        uint32_t j;
        for (;;) {
          j = take_ticket(ticket, xq);
          if (j < sd.ns || ++dry >= 8) break;
          xq = (xq + 1) & 7;
        }
        if (j >= sd.ns) {
          more = false;
          break;
        }
        sj = j;
        snext = sd.sbeg ? (uint32_t)sd.spc[j] : 0u;
        sende = sd.sbeg ? (uint32_t)sd.spc[j + 1] : n;
        scur = sd.sbeg ? sd.sbeg[j] : 0;
        slim = sd.sbeg ? sd.send[j] : avail;
        sfail = CPK_OK;
        if (snext >= sende) sd.send_out[j] = scur;
      }
      if (!more) break;
      seg = snext++;
    }
    if (seg >= n) break;
    const uint64_t w0 = swo[seg];
    const int W = (int)(swo[seg + 1] - w0);
    const uint64_t a = kStream ? scur : in_off[seg];
    const uint32_t P = kStream ? (uint32_t)min(slim - scur, (uint64_t)0xffffffffu)
                               : (uint32_t)(in_off[seg + 1] - a);
    if (kStream && sfail != CPK_OK) {
      status[seg] = sfail;
      if (seg + 1 == sende) sd.send_out[sj] = scur;
      continue;
    }
    const uint8_t *gp = packed + a;
    const uint32_t glim = (uint32_t)(((a + P + 15) & ~15ull) - a);  // readable bytes
    uint64_t *dst = out + w0;
    int st = CPK_OK;
    uint32_t e = 0;  // true tag position (piece-relative)
    int ow = 0;      // output words produced
    if (W == 0) st = (P == 0 || kStream) ? CPK_OK : CPK_ETRAILING;  // read() of 0 bytes
    while (W != 0) {
      if (e >= P) {
        if (ow < W) st = CPK_ETRUNC;  // ArrayInputStream EOF -> DecodeException
        break;
      }
      if (ow >= W) break;  // (trailing input is flagged by the record check)
      const uint32_t wend = min(e + kWin, P);
      WPH(0)
      // ---- window load: LDS byte x <-> packed[(a + e) & ~15 + x] ----------
      const uint32_t padw = (uint32_t)((a + e) & 15);
      const uint32_t ebase = e - padw;  // piece position of wbuf[0]
      const uint32_t need = min(e + kWin + 32, P) - ebase;  // <= kWin + 47 bytes
      const uint32_t lines = (need + 15) >> 4;
      const uint4 *gsrc = reinterpret_cast<const uint4 *>(gp - padw + e);
      // all of a lane's lines (<= 3) in flight at once, then the LDS writes:
      // one memory latency per window instead of one per line
      {
        uint4 l[kWinLinesPerLane];
#pragma unroll
        for (int j = 0; j < kWinLinesPerLane; ++j) {
          const uint32_t L = lane + 64 * j;
          l[j] = L < lines ? gsrc[L] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < kWinLinesPerLane; ++j) {
          const uint32_t L = lane + 64 * j;
          if (L < lines) reinterpret_cast<uint4 *>(wbuf)[L] = l[j];
        }
      }
      const uint32_t lend = ebase + 16 * lines;  // loaded piece positions < lend
      // pkw[q] = packed byte q (signed 64-bit offset: ebase is negative when
      // the piece starts mid-line)
      const uint8_t *pkw = wbuf + (int64_t)padw - (int64_t)e;
      const uint32_t ph = (padw - e) & 3;  // LDS byte phase of piece position 0
      wave_lds_order();

      WPH(1)
      // ---- 1: speculative chunk walks --------------------------------------
      const uint32_t cb = e + kDecChunk * lane;
      const uint32_t ce = min(cb + kDecChunk, wend);
      VisMask vis = 0;
      uint32_t X = cb, wt = 0;  // wt: output words of the walk
      if (cb < wend) {
        uint32_t pos = cb;
        while (pos < ce) {
          vis |= (VisMask)1 << (pos - cb);
          const DecRec r = rec_at(pkw, pos);
          wt += r.nw;
          pos += r.len;
        }
        X = pos;
      }
      visa[lane] = vis;
      wave_lds_order();
      // ---- 2: walk on until landing on a visited position -------------------
      uint32_t S = X, lw = 0;  // lw: output words of the landing walk
      if (cb < wend) {
        while (S < wend) {
          const uint32_t r = S - e;
          const uint32_t ow_ = r / kDecChunk;
          if ((visa[ow_] >> (r - ow_ * kDecChunk)) & 1) break;
          const DecRec rr = rec_at(pkw, S);
          lw += rr.nw;
          S += rr.len;
        }
      }
      WPH(2)
      // ---- 3: true chain over lanes -----------------------------------------
      // lane j's successor is the owner of its landing point (always a later
      // lane); the true records are on the lanes reachable from lane 0, found
      // by pointer doubling (6 rounds cover a chain of 64)
      int nx = (cb < wend && S < wend) ? (int)((S - e) / kDecChunk) : 64;
      uint64_t R = 1ull << lane;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const int src = (nx & 63) << 2;
        const uint32_t rlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)R);
        const uint32_t rhi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(R >> 32));
        const int nn = __builtin_amdgcn_ds_bpermute(src, nx);
        if (nx < 64) {
          R |= ((uint64_t)rhi << 32) | rlo;
          nx = nn;
        }
      }
      const uint64_t onmask = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)R, 0)) |
                              ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(R >> 32), 0) << 32);
      const uint32_t enext =
          (uint32_t)__builtin_amdgcn_readlane((int)S, 63 - __builtin_clzll(onmask));
      // each on-path lane hands its landing point to its successor
      wave_lds_order();  // (phase 2's reads of visa are done)
      if (((onmask >> lane) & 1) && S < wend) visa[(S - e) / kDecChunk] = (VisMask)S;
      wave_lds_order();
      const uint32_t entry = lane == 0 ? e : (uint32_t)visa[lane];
      const bool on = (onmask >> lane) & 1;
      WPH(3)
      // ---- 4: output words of each lane's true records ----------------------
      // [entry, S) = the walk's records from entry (a position the walk
      // visited) plus the landing walk: the walk's words minus those before
      // entry (usually one or two records of a false start)
      int myw = 0;
      if (on) {
        uint32_t pre = 0;
        for (uint32_t q = cb; q < entry;) {
          const DecRec r = rec_at(pkw, q);
          pre += r.nw;
          q += r.len;
        }
        myw = (int)(wt - pre + lw);
      }
      const int inc = wave_incl_add(myw);
      const int T = readlane(inc, 63);
      const int o0 = inc - myw;  // window-relative output of this lane's first record
      WPH(4)
      // ---- 5: error checks, block map, expansion (rounds of 2048 words) -----
      bool failed = false;
      uint32_t fin = 0;  // end of the record that fills the piece (if any)
      // errors and the filling record can only occur in a window reaching the
      // piece's last word or within one window plus one record of its end
      const bool chk = (ow + T >= W) || (P - e < 3 * kWin);
      for (int rb = 0; rb < T; rb += kRound) {
        int err = 0x7fffffff;
        // after the first round only the lanes whose output meets this round
        if (on && (rb == 0 || (o0 < rb + kRound && o0 + myw > rb))) {
          int o = o0;
          for (uint32_t q = entry; q < S;) {
            const uint32_t tag = pkw[q], c1 = pkw[q + 1], c9 = pkw[q + 9];
            const uint32_t ntag = 1 + __builtin_popcount(tag);
            const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
            const int nw = 1 + (int)((zm & c1) + (fm & c9));
            const uint32_t adv = ntag + (zm & 1u) + (fm & (8u * c9 + 1u));
            const int oo = ow + o;
            if (chk && rb == 0 && oo < W && err == 0x7fffffff) {
              // PackedInputStream.java:53-138: truncated tag bytes / count /
              // literal run -> EOF DecodeException; run past the piece ->
              // DecodeException / BufferOverflowException
              int code = 0;
              if (q + ntag > P) code = 2;
              else if (tag == 0 || tag == 0xffu) {
                if (q + (tag ? 10u : 2u) > P) code = 2;
                else if (oo + nw > W) code = 3;
                else if (q + adv > P) code = 2;
              }
              if (!kStream && !code && oo + nw == W && q + adv < P) code = 4;
              if (code) err = (int)(((q - e) << 3) | (uint32_t)code);  // window-relative
              if (oo + nw == W) fin = q + adv;
            }
            // blocks of this round whose first word this record covers
            const int lo = max(o, rb), hi = min(o + nw, rb + kRound);
            // window-relative record position (< 2 KiB) | offset in the run
            for (int bb = (lo + kBlk - 1) & ~(kBlk - 1); bb < hi; bb += kBlk)
              blk[(bb - rb) / kBlk] = (q - e) | ((uint32_t)(bb - o) << 16);
            o += nw;
            q += adv;
          }
        }
        if (rb == 0) {
          err = __builtin_amdgcn_readfirstlane(wave_min(err));
          if (err != 0x7fffffff) {
            st = -(err & 7);
            failed = true;
            break;
          }
          fin = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_max_u(fin));
        }
        wave_lds_order();
        WPH(5)
        const int nb = (min(min(kRound, T - rb), W - ow - rb) + kBlk - 1) / kBlk;
        for (int b = lane; b < nb; b += 64) {
          const uint32_t v = blk[b];
          uint32_t q = e + (v & 0xffffu);
          int ofs = (int)(v >> 16);
          const int wbase = ow + rb + kBlk * b;  // piece word of the block's first word
          uint64_t words[kBlk];
#pragma unroll
          for (int i = 0; i < kBlk; ++i) {
            // PackedInputStream.java:84-134 per word: zero run, 0xFF literal
            // run (tag word, then the counted words), or a tagged word
            // (the count bytes are read with the tag: one LDS round trip)
            const uint32_t tag = pkw[q], c1 = pkw[q + 1], c9 = pkw[q + 9];
            uint64_t x;
            int nw;
            uint32_t adv;
            if (tag == 0) {
              x = 0;
              nw = 1 + c1;
              adv = 2;
            } else if (tag == 0xffu) {
              const uint32_t rn = c9;
              nw = 1 + (int)rn;
              adv = 10 + 8 * rn;
              x = read8(pkw, ofs == 0 ? q + 1 : q + 10 + 8 * (uint32_t)(ofs - 1), lend, gp, glim, ph, e);
            } else {
              const uint64_t raw = read8(pkw, q + 1, lend, gp, glim, ph, e);
              const uint64_t sel = lut[tag];
              const uint32_t rl = (uint32_t)raw, rh = (uint32_t)(raw >> 32);
              const uint32_t x0 = __builtin_amdgcn_perm(rh, rl, (uint32_t)sel);
              const uint32_t x1 = __builtin_amdgcn_perm(rh, rl, (uint32_t)(sel >> 32));
              x = (uint64_t)x0 | ((uint64_t)x1 << 32);
              nw = 1;
              adv = 1 + __builtin_popcount(tag);
            }
            words[i] = x;
            // past the window's last word: stay put (never stored)
            if (++ofs == nw && wbase + i + 1 < ow + T) {
              q += adv;
              ofs = 0;
            }
          }
          const int kw = min(kBlk, min(ow + T, W) - wbase);
          uint64_t *d = dst + wbase;
          if (kw == kBlk && ((reinterpret_cast<uintptr_t>(d) & 15) == 0)) {
#pragma unroll
            for (int i = 0; i < kBlk; i += 2) {
              uint4 v4;
              v4.x = (uint32_t)words[i];
              v4.y = (uint32_t)(words[i] >> 32);
              v4.z = (uint32_t)words[i + 1];
              v4.w = (uint32_t)(words[i + 1] >> 32);
              *reinterpret_cast<uint4 *>(d + i) = v4;
            }
          } else {
#pragma unroll
            for (int i = 0; i < kBlk; ++i)
              if (i < kw) d[i] = words[i];
          }
        }
        wave_lds_order();  // blk reused by the next round
        WPH(6)
      }
      if (failed) break;
      if (ow + T >= W && fin) {  // the piece is full: next piece starts at fin
        ow = W;
        e = fin;
        break;
      }
      ow += T;
      e = enext;
    }
    status[seg] = st;  // every lane the same value: no lane-dependent branch
    if (kStream) {
      in_off[seg] = a;
      scur = a + e;
      sfail = st;
      if (seg + 1 == sende) sd.send_out[sj] = scur;
    }
  }
  WPH_FLUSH(16)
}

// ------------------------------------------------------------ messages
// Serialize.read over PackedInputStream for a batch of packed messages whose
// byte ranges are known (Serialize.java:119-178): a thread per message reads
// the segment table (two read() calls: the first word, then 4 * (count & ~1)
// bytes), validates it, and the segments are then decoded as one packed
// stream per message by decode_kernel<true>.

// one read() of `words` words, byte-serial (tables are at most 257 words):
// PackedInputStream.java:35-140 as the oracle restates it
// (oracle/packed_oracle.c:cpko_unpack); f(word index, word) per word
template <class F>
__device__ int serial_read(const uint8_t *p, uint64_t n, uint64_t &ip, uint32_t words, F f) {
  if (words == 0) return CPK_OK;
  uint32_t wi = 0;
  for (;;) {
    if (ip >= n) return CPK_ETRUNC;
    const uint32_t tag = p[ip++];
    uint64_t w = 0;
    for (int i = 0; i < 8; ++i)
      if ((tag >> i) & 1) {
        if (ip >= n) return CPK_ETRUNC;
        w |= (uint64_t)p[ip++] << (8 * i);
      }
    f(wi++, w);
    if (tag == 0 || tag == 0xffu) {
      if (ip >= n) return CPK_ETRUNC;
      const uint32_t run = p[ip++];
      if (run > words - wi) return CPK_EOVERRUN;
      if (tag == 0) {
        for (uint32_t k = 0; k < run; ++k) f(wi++, 0ull);
      } else {
        if (n - ip < 8ull * run) return CPK_ETRUNC;
        for (uint32_t k = 0; k < run; ++k) {
          uint64_t v = 0;
          for (int i = 0; i < 8; ++i) v |= (uint64_t)p[ip + i] << (8 * i);
          ip += 8;
          f(wi++, v);
        }
      }
    }
    if (wi == words) return CPK_OK;
  }
}

// the table of message m: status, segment count, total words; on OK the
// packed position after the table.  emit(i, size) per segment.
template <class F>
__device__ int read_table(const uint8_t *p, uint64_t n, uint64_t limit, uint64_t &ip,
                          uint32_t &count, uint64_t &total, F emit) {
  uint64_t first = 0;
  int st = serial_read(p, n, ip, 1, [&](uint32_t, uint64_t w) { first = w; });
  if (st) return st;
  const int32_t raw = (int32_t)(uint32_t)first;
  if (raw < 0 || raw > 511) return CPK_EFRAME;  // Serialize.java:128-131
  count = (uint32_t)raw + 1;
  const int32_t s0 = (int32_t)(uint32_t)(first >> 32);
  if (s0 < 0) return CPK_EFRAME;  // :135-137
  total = (uint64_t)s0;
  bool neg = false, big = s0 > kMaxSegmentWords;
  emit(0u, (uint32_t)s0);
  if (count > 1) {  // :144-157
    const uint32_t c = count;
    st = serial_read(p, n, ip, (count & ~1u) / 2, [&](uint32_t i, uint64_t w) {
      for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t k = 2 * i + h;  // moreSizes[k] = segment k + 1
        if (k + 1 < c) {
          const int32_t v = (int32_t)(uint32_t)(w >> (32 * h));
          neg |= v < 0;
          big |= v > kMaxSegmentWords;
          total += (uint64_t)(uint32_t)v;
          emit(k + 1, (uint32_t)v);
        }
      }
    });
    if (st) return st;
    if (neg) return CPK_EFRAME;  // :150-153 (the first negative size throws)
  }
  if (total > limit) return CPK_EFRAME;  // :160-162
  // makeByteBufferForWords (:45-53) throws for a segment over 2^28 - 1 words
  // when that segment is allocated: the message fails either way
  if (big) return CPK_EFRAME;
  return CPK_OK;
}

// pass 1: per message its table's status, segment count, words and the
// packed position of segment 0
__global__ void msg_table_kernel(const uint8_t *__restrict__ packed, const uint64_t *__restrict__ moff,
                                 uint32_t nm, uint64_t limit, uint64_t *__restrict__ mwords,
                                 uint64_t *__restrict__ mcount, uint64_t *__restrict__ mbeg,
                                 int32_t *__restrict__ mstatus) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const uint64_t a = moff[m];
  uint64_t ip = 0, total = 0;
  uint32_t count = 0;
  const int st = read_table(packed + a, moff[m + 1] - a, limit, ip, count, total,
                            [](uint32_t, uint32_t) {});
  mstatus[m] = st;
  mwords[m] = st ? 0 : total;
  mcount[m] = st ? 0 : count;
  mbeg[m] = a + ip;
}

// pass 2: the segments' word offsets (segment table read again)
__global__ void msg_swo_kernel(const uint8_t *__restrict__ packed, const uint64_t *__restrict__ moff,
                               uint32_t nm, uint64_t limit, const uint64_t *__restrict__ mwoff,
                               const uint64_t *__restrict__ mseg, const int32_t *__restrict__ mstatus,
                               uint64_t *__restrict__ swo) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  if (m == nm - 1) swo[mseg[nm]] = mwoff[nm];
  if (mstatus[m] != CPK_OK) return;
  const uint64_t a = moff[m], s0 = mseg[m];
  uint64_t ip = 0, total = 0, acc = mwoff[m];
  uint32_t count = 0;
  read_table(packed + a, moff[m + 1] - a, limit, ip, count, total, [&](uint32_t i, uint32_t sz) {
    swo[s0 + i] = acc;
    acc += sz;
  });
}

// pass 4: a message's status: its table's, else its first failed segment's
// (a failure stops the stream: the last segment carries it), else
// CPK_ETRAILING when the segments end before the message's bytes do
__global__ void msg_final_kernel(const uint64_t *__restrict__ moff, uint32_t nm,
                                 const uint64_t *__restrict__ mseg, const uint64_t *__restrict__ mend,
                                 const int32_t *__restrict__ seg_status, int32_t *__restrict__ mstatus) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm || mstatus[m] != CPK_OK) return;
  const int32_t st = seg_status[mseg[m + 1] - 1];
  mstatus[m] = st != CPK_OK ? st : (mend[m] != moff[m + 1] ? CPK_ETRAILING : CPK_OK);
}

// ---- message write: Serialize.write = table piece + segment pieces --------
// PackedOutputStream.write (:35-205) byte-serial over a word source, as the
// oracle restates it (oracle/packed_oracle.c:cpko_pack); for the segment
// tables (a thread per message).  word(i) -> word i; emit(byte).
template <class Wf, class Ef>
__device__ void serial_pack(uint32_t nwords, Wf word, Ef emit) {
  uint32_t i = 0;
  while (i < nwords) {
    const uint64_t w = word(i++);
    uint32_t tag = 0;
    for (int b = 0; b < 8; ++b) tag |= ((w >> (8 * b)) & 0xffu) ? (1u << b) : 0u;
    emit(tag);
    for (int b = 0; b < 8; ++b)
      if ((tag >> b) & 1) emit((uint32_t)(w >> (8 * b)) & 0xffu);
    if (tag == 0) {  // :119-131
      uint32_t run = 0;
      while (i < nwords && run < 255 && word(i) == 0) {
        ++run;
        ++i;
      }
      emit(run);
    } else if (tag == 0xffu) {  // :133-193: stop before a word with >= 2 zero bytes
      uint32_t run = 0;
      while (i < nwords && run < 255) {
        const uint64_t x = word(i);
        int z = 0;
        for (int b = 0; b < 8; ++b) z += ((x >> (8 * b)) & 0xffu) == 0;
        if (z >= 2) break;
        ++run;
        ++i;
      }
      emit(run);
      for (uint32_t k = i - run; k < i; ++k) {
        const uint64_t x = word(k);
        for (int b = 0; b < 8; ++b) emit((uint32_t)(x >> (8 * b)) & 0xffu);
      }
    }
  }
}

// word k of message m's segment table (Serialize.java:256-273): ints
// [count - 1, size_0 .. size_{count-1}, 0 pad], (count + 2) & ~1 of them
__device__ __forceinline__ uint64_t table_word(const uint64_t *swo, uint64_t s0, uint32_t count,
                                               uint32_t k) {
  uint32_t v[2];
  for (int h = 0; h < 2; ++h) {
    const uint32_t j = 2 * k + h;
    v[h] = j == 0 ? count - 1 : (j <= count ? (uint32_t)(swo[s0 + j] - swo[s0 + j - 1]) : 0u);
  }
  return (uint64_t)v[0] | ((uint64_t)v[1] << 32);
}
__device__ __forceinline__ uint32_t table_words(uint32_t count) { return ((count + 2) & ~1u) / 2; }

// packed size of every message's table
__global__ void msg_table_size_kernel(const uint64_t *__restrict__ swo,
                                      const uint64_t *__restrict__ mseg, uint32_t nm,
                                      uint64_t *__restrict__ tsize) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const uint64_t s0 = mseg[m];
  const uint32_t count = (uint32_t)(mseg[m + 1] - s0);
  uint64_t nb = 0;
  serial_pack(table_words(count), [&](uint32_t k) { return table_word(swo, s0, count, k); },
              [&](uint32_t) { ++nb; });
  tsize[m] = nb;
}

// piece sizes in message order: table, then its segments
__global__ void msg_interleave_kernel(const uint64_t *__restrict__ mseg, uint32_t nm,
                                      const uint64_t *__restrict__ tsize,
                                      const uint64_t *__restrict__ ssize, uint64_t *__restrict__ comb) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const uint64_t s0 = mseg[m], s1 = mseg[m + 1];
  uint64_t *c = comb + s0 + m;
  c[0] = tsize[m];
  for (uint64_t s = s0; s < s1; ++s) c[1 + s - s0] = ssize[s];
}

// each segment's packed offset (from the message-order offsets), and the
// tables' packed bytes
__global__ void msg_table_emit_kernel(const uint64_t *__restrict__ swo,
                                      const uint64_t *__restrict__ mseg, uint32_t nm,
                                      const uint64_t *__restrict__ poff, uint64_t *__restrict__ soff,
                                      uint8_t *__restrict__ out) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const uint64_t s0 = mseg[m], s1 = mseg[m + 1];
  const uint64_t *c = poff + s0 + m;
  for (uint64_t s = s0; s < s1; ++s) soff[s] = c[1 + s - s0];
  uint8_t *o = out + c[0];
  const uint32_t count = (uint32_t)(s1 - s0);
  serial_pack(table_words(count), [&](uint32_t k) { return table_word(swo, s0, count, k); },
              [&](uint32_t b) { *o++ = (uint8_t)b; });
}

// ------------------------------------------------------------ bench support
struct FastRand {
  int32_t x, y, z, w;
};
// benchmark/src/main/java/org/capnproto/benchmark/Common.java:31-38
__device__ __forceinline__ uint32_t fr_next(FastRand &r) {
  uint32_t ux = (uint32_t)r.x;
  uint32_t tmp = ux ^ (ux << 11);
  r.x = r.y;
  r.y = r.z;
  r.z = r.w;
  uint32_t w = (uint32_t)r.w;
  w = w ^ (uint32_t)(r.w >> 19) ^ tmp ^ (uint32_t)((int32_t)tmp >> 8);
  r.w = (int32_t)w;
  return w;
}
__device__ __forceinline__ uint64_t splitmix64(uint64_t &s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void generate_kernel(cpk_gen_params p, const uint64_t *__restrict__ swo, uint32_t n,
                                uint64_t *__restrict__ out) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n; s += gridDim.x * blockDim.x) {
    uint64_t sd = 0x1d2acd47ull ^ ((uint64_t)p.cfg << 40) ^ ((uint64_t)s * 0xD1B54A32D192ED03ull);
    uint64_t a = splitmix64(sd), b = splitmix64(sd);
    FastRand r{(int32_t)(uint32_t)a, (int32_t)(uint32_t)(a >> 32), (int32_t)(uint32_t)b,
               (int32_t)(uint32_t)(b >> 32)};
    if ((r.x | r.y | r.z | r.w) == 0) r.w = 1;
    uint64_t w0 = swo[s], w1 = swo[s + 1];
    bool zero = (uint64_t)fr_next(r) < p.t_zero0;
    for (uint64_t k = 0; k < w1 - w0; ++k) {
      if (k) {
        uint32_t t = fr_next(r);
        zero = zero ? !((uint64_t)t < p.t_z2n) : ((uint64_t)t < p.t_n2z);
      }
      uint64_t v = 0;
      if (!zero) {
        for (int bb = 0; bb < 8; ++bb) {
          uint32_t t = fr_next(r);
          uint64_t byte = ((uint64_t)t < p.t_qbyte) ? 0 : (uint64_t)(1 + (t >> 8) % 255);
          v |= byte << (8 * bb);
        }
      }
      out[w0 + k] = v;
    }
  }
}

__global__ void mismatch_kernel(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b,
                                uint64_t words, unsigned long long *cnt) {
  unsigned long long c = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words;
       i += (uint64_t)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

#include "encode_v3.hip"
#include "encode_v4.hip"

}  // namespace cpk

// ================================================================ C ABI
struct HostPipe;  // host_pipe.hip: staging of the host-memory forms

struct cpk_ctx_s {
  int device;
  int cus;
  uint64_t *status;       // look-back words
  uint64_t status_cap;    // entries
  uint32_t *tickets;      // cpk::kTkWords words: per-XCD counters, plan ticket, error bits
  void *plan;             // tiled encode: toff | tmap | pstatus | tstate
  uint64_t plan_cap;      // bytes
  int encoder;            // 4: size + emit passes (default); 1-3: earlier encoders
  uint32_t *e3_tfirst;    // encoder v3: tile -> first piece starting in it
  uint64_t *e3_status;    //   look-back word per tile
  uint64_t *e3_tstate;    //   exit run state per tile
  uint64_t e3_cap;        //   tiles the arrays hold (+2)
  uint32_t epoch;         //   launch epoch tagging the look-back words, 1..65535
  int e3_grid;            //   workgroups of encode3_kernel resident at once
  uint64_t *e4_bv;        // encoder v4: run boundaries per 64-word step
  uint64_t e4_bv_cap;     //   entries
  HostPipe *pipe;         // cpk_encode_host / cpk_decode_host staging (lazy)
};

namespace {
int hip_ok(hipError_t e) { return e == hipSuccess ? CPK_OK : CPK_EDEVICE; }

struct DeviceGuard {
  int prev;
  explicit DeviceGuard(int d) {
    hipGetDevice(&prev);
    if (prev != d) hipSetDevice(d);
  }
  ~DeviceGuard() {
    int cur;
    hipGetDevice(&cur);
    if (cur != prev) hipSetDevice(prev);
  }
};

int ensure_status(cpk_ctx ctx, uint64_t n) {
  if (n <= ctx->status_cap) return CPK_OK;
  if (ctx->status) hipFree(ctx->status);
  ctx->status = nullptr;
  uint64_t cap = n < 1024 ? 1024 : n + n / 4;
  if (hipMalloc(&ctx->status, cap * sizeof(uint64_t)) != hipSuccess) {
    ctx->status_cap = 0;
    return CPK_ENOMEM;
  }
  ctx->status_cap = cap;
  return CPK_OK;
}
int ensure_plan(cpk_ctx ctx, uint64_t bytes) {
  if (bytes <= ctx->plan_cap) return CPK_OK;
  if (ctx->plan) hipFree(ctx->plan);
  ctx->plan = nullptr;
  uint64_t cap = bytes + bytes / 4;
  if (hipMalloc(&ctx->plan, cap) != hipSuccess) {
    ctx->plan_cap = 0;
    return CPK_ENOMEM;
  }
  ctx->plan_cap = cap;
  return CPK_OK;
}
uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

// Encoder v3 (encode_v3.hip): plan kernel + persistent tile kernel.  The
// tile count is bounded from the size hint (or read back when there is none);
// a batch larger than the bound is reported through the error word.
int e3_encode(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t n, uint64_t hint,
              void *d_out, uint64_t *d_out_off, hipStream_t s) {
  const uint64_t TW = cpk::kE3TileWords;
  uint64_t ntb;
  if (hint) {
    ntb = ((uint64_t)n * hint + TW - 1) / TW;
  } else {
    uint64_t ends[2];
    if (hipMemcpyAsync(&ends[0], d_swo, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&ends[1], d_swo + n, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return CPK_EDEVICE;
    ntb = (ends[1] - ends[0] + TW - 1) / TW;
  }
  if (ntb > 0xfffffff0ull) return CPK_EUNSUPPORTED;
  bool fresh = false;
  if (ntb + 2 > ctx->e3_cap) {
    if (ctx->e3_tfirst) hipFree(ctx->e3_tfirst);
    if (ctx->e3_status) hipFree(ctx->e3_status);
    if (ctx->e3_tstate) hipFree(ctx->e3_tstate);
    ctx->e3_tfirst = nullptr;
    ctx->e3_status = ctx->e3_tstate = nullptr;
    ctx->e3_cap = 0;
    uint64_t cap = ntb + 2 + (ntb + 2) / 4;
    if (cap < 1024) cap = 1024;
    if (hipMalloc(&ctx->e3_tfirst, cap * 4) != hipSuccess ||
        hipMalloc(&ctx->e3_status, cap * 16) != hipSuccess ||  // tile sizes | round bases
        hipMalloc(&ctx->e3_tstate, cap * 8) != hipSuccess)
      return CPK_ENOMEM;
    ctx->e3_cap = cap;
    fresh = true;
  }
  if (++ctx->epoch > 0xffffu) {
    ctx->epoch = 1;
    fresh = true;
  }
  if (fresh && (hipMemsetAsync(ctx->e3_status, 0, ctx->e3_cap * 16, s) != hipSuccess ||
                hipMemsetAsync(ctx->e3_tstate, 0, ctx->e3_cap * 8, s) != hipSuccess))
    return CPK_EDEVICE;
  uint32_t *err = ctx->tickets + cpk::kTkErr;
  uint64_t pb = ((uint64_t)n + 2 + 255) / 256;
  if (pb > 4096) pb = 4096;
  hipLaunchKernelGGL(cpk::e3_plan_kernel, dim3((unsigned)pb), dim3(256), 0, s, d_swo, n,
                     (uint32_t)ntb, ctx->e3_tfirst, d_out_off, hint, err);
  if (ntb == 0) return hip_ok(hipGetLastError());
  uint64_t grid = (uint64_t)ctx->e3_grid;
  if (grid > (uint64_t)cpk::kE3Threads * cpk::kE3MaxPer) grid = (uint64_t)cpk::kE3Threads * cpk::kE3MaxPer;
  if (grid > ntb) grid = ntb;
  hipLaunchKernelGGL(cpk::encode3_kernel, dim3((unsigned)grid), dim3(cpk::kE3Threads), cpk::kE3Lds,
                     s, (const uint64_t *)d_in, d_swo, n, (uint32_t)ntb,
                     (const uint32_t *)ctx->e3_tfirst, (uint8_t *)d_out, d_out_off,
                     ctx->e3_status, ctx->e3_status + ctx->e3_cap, ctx->e3_tstate, ctx->epoch,
                     err);
  return hip_ok(hipGetLastError());
}
}  // namespace

#include "host_pipe.hip"

extern "C" {

int cpk_abi_version(void) { return CPK_ABI_VERSION; }

#ifdef CPK_PHASE_STATS
// diagnostic builds only: read and clear the per-phase cycle sums
int cpk_debug_phase_stats(unsigned long long *host64) {
  if (hipMemcpyFromSymbol(host64, HIP_SYMBOL(cpk::g_phase), 64 * 8) != hipSuccess) return CPK_EDEVICE;
  unsigned long long z[64] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(cpk::g_phase), z, sizeof z) == hipSuccess ? CPK_OK : CPK_EDEVICE;
}
#endif

const char *cpk_status_string(int s) {
  switch (s) {
    case CPK_OK: return "ok";
    case CPK_EINVAL: return "invalid argument / misaligned piece";
    case CPK_ETRUNC: return "premature end of packed input";
    case CPK_EOVERRUN: return "packed run past the end of the piece";
    case CPK_ETRAILING: return "piece filled before the end of its packed bytes";
    case CPK_EFRAME: return "invalid segment table";
    case CPK_ENOMEM: return "out of device memory";
    case CPK_EDEVICE: return "HIP runtime error";
    case CPK_EUNSUPPORTED: return "piece not supported by this build";
    default: return "unknown status";
  }
}

uint64_t cpk_packed_bound(uint64_t words) { return 8 * words + 2 * ((words + 1) / 2); }

uint64_t cpk_batch_packed_capacity(const uint64_t *h_swo, uint32_t n) {
  uint64_t s = 0;
  for (uint32_t i = 0; i < n; ++i) s += cpk_packed_bound(h_swo[i + 1] - h_swo[i]);
  return s + 16;
}

int cpk_ctx_create(int device, cpk_ctx *out) {
  if (!out) return CPK_EINVAL;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
    return CPK_EDEVICE;
  DeviceGuard g(device);
  cpk_ctx c = (cpk_ctx)calloc(1, sizeof(cpk_ctx_s));
  if (!c) return CPK_ENOMEM;
  c->device = device;
  {
    const char *e = getenv("CPK_ENCODER");
    // CPK_ENCODER selects an encoder for A/B runs; v4 (size + emit passes,
    // wave per piece) is the default, measured fastest on every config
    c->encoder = (e && e[0] == '1') ? 1 : (e && e[0] == '3') ? 3 : (e && e[0] == '2') ? 2 : 4;
  }
  if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    c->cus = 256;
  if (hipMalloc(&c->tickets, cpk::kTkWords * 4) != hipSuccess ||
      hipMemset(c->tickets, 0, cpk::kTkWords * 4) != hipSuccess) {
    free(c);
    return CPK_ENOMEM;
  }
  if (hipFuncSetAttribute((const void *)cpk::encode_kernel<false>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, cpk::kEncLds) != hipSuccess ||
      hipFuncSetAttribute((const void *)cpk::encode_kernel<true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, cpk::kEncLds) != hipSuccess ||
      hipFuncSetAttribute((const void *)cpk::encode2_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize, cpk::kE2Lds) != hipSuccess ||
      hipFuncSetAttribute((const void *)cpk::decode_kernel<false>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, cpk::kDecLds) != hipSuccess ||
      hipFuncSetAttribute((const void *)cpk::encode3_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize, cpk::kE3Lds) != hipSuccess) {
    hipFree(c->tickets);
    free(c);
    return CPK_EDEVICE;
  }
  {
    // persistent grid of encode3_kernel: every workgroup resident at once
    // (its look-back waits on other workgroups).  The occupancy answer can be
    // one block per CU high for SGPR-heavy kernels (MI355X_MICROARCH.md,
    // Residency), so one block per CU is kept in reserve.
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)cpk::encode3_kernel,
                                                     cpk::kE3Threads, cpk::kE3Lds) != hipSuccess ||
        occ < 1)
      occ = 1;
    const char *rs = getenv("CPK_E3_RESERVE");  // blocks per CU kept in reserve (tuning)
    const int reserve = rs ? atoi(rs) : 1;
    if (occ > reserve) occ -= reserve;
    c->e3_grid = occ * c->cus;
  }
  *out = c;
  return CPK_OK;
}

void cpk_ctx_destroy(cpk_ctx ctx) {
  if (!ctx) return;
  DeviceGuard g(ctx->device);
  if (ctx->status) hipFree(ctx->status);
  if (ctx->plan) hipFree(ctx->plan);
  if (ctx->tickets) hipFree(ctx->tickets);
  if (ctx->e3_tfirst) hipFree(ctx->e3_tfirst);
  if (ctx->e3_status) hipFree(ctx->e3_status);
  if (ctx->e3_tstate) hipFree(ctx->e3_tstate);
  if (ctx->e4_bv) hipFree(ctx->e4_bv);
  pipe_destroy(ctx->pipe);
  free(ctx);
}

int cpk_ctx_device(cpk_ctx ctx) { return ctx ? ctx->device : -1; }

// Encoder v4 (encode_v4.hip): size pass, scan, emit pass.  Pieces of any
// size; a piece over the hint is reported (output undefined).  The size pass
// leaves each 64-word step's run boundaries for the emit pass: `stride` rows
// per piece from the hint, or packed by word offset when there is no hint (the
// batch's word count is then read back, synchronising the stream).
int e4_encode(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t n, uint64_t hint,
              void *d_out, uint64_t *d_out_off, hipStream_t s) {
  const uint32_t nb = (uint32_t)((n + cpk::kE4ScanBlock - 1) / cpk::kE4ScanBlock);
  int rc = ensure_status(ctx, (uint64_t)n + nb + 1);
  if (rc) return rc;
  uint64_t stride = hint ? (hint + 63) / 64 : 0, rows;
  if (stride && stride > (1ull << 29) / n) stride = 0;  // (> 4 GiB of rows: pack them; no overflow)
  if (stride) {
    rows = (uint64_t)n * stride;
  } else {
    uint64_t ends[2];
    if (hipMemcpyAsync(&ends[0], d_swo, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&ends[1], d_swo + n, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return CPK_EDEVICE;
    rows = (ends[1] - ends[0]) / 64 + n + 1;
  }
  if (rows > ctx->e4_bv_cap) {
    if (ctx->e4_bv) hipFree(ctx->e4_bv);
    ctx->e4_bv = nullptr;
    ctx->e4_bv_cap = 0;
    const uint64_t cap = rows + rows / 4;
    if (hipMalloc(&ctx->e4_bv, cap * 8) != hipSuccess) return CPK_ENOMEM;
    ctx->e4_bv_cap = cap;
  }
  uint64_t *sizes = ctx->status, *bsum = ctx->status + n;
  if (hipMemsetAsync(ctx->tickets, 0, cpk::kTkErr * 4, s) != hipSuccess) return CPK_EDEVICE;
  unsigned grid = (unsigned)(8 * ctx->cus);
  if (grid > (n + cpk::kE4Waves - 1) / cpk::kE4Waves) grid = (n + cpk::kE4Waves - 1) / cpk::kE4Waves;
  hipLaunchKernelGGL(cpk::e4_size_kernel, dim3(grid), dim3(cpk::kE4Threads), 0, s,
                     (const uint64_t *)d_in, d_swo, n, sizes, ctx->tickets + cpk::kTkEnc, hint,
                     ctx->tickets + cpk::kTkErr, ctx->e4_bv, stride);
  hipLaunchKernelGGL(cpk::e4_scan_reduce, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)sizes, n, bsum);
  hipLaunchKernelGGL(cpk::e4_scan_top, dim3(1), dim3(cpk::kE4ScanThreads), 0, s, bsum, nb);
  hipLaunchKernelGGL(cpk::e4_scan_down, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)sizes, n, (const uint64_t *)bsum, d_out_off);
  hipLaunchKernelGGL(cpk::e4_emit_kernel, dim3(grid), dim3(cpk::kE4Threads), cpk::kE4Lds, s,
                     (const uint64_t *)d_in, d_swo, n, (const uint64_t *)d_out_off,
                     (uint8_t *)d_out, ctx->tickets + cpk::kTkDec, (const uint64_t *)ctx->e4_bv,
                     stride);
  return hip_ok(hipGetLastError());
}

int cpk_encode_messages(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t nseg,
                        const uint64_t *d_msg_seg_off, uint32_t nm, uint64_t max_seg_words,
                        void *d_out, uint64_t *d_out_off, void *stream) {
  if (!ctx || !d_out_off || (nm && !d_msg_seg_off) || (nseg && !d_swo)) return CPK_EINVAL;
  if (((uintptr_t)d_out & 15) || ((uintptr_t)d_in & 7)) return CPK_EINVAL;
  if (max_seg_words == 0) return CPK_EINVAL;  // (a bound is needed for the step rows)
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (nm == 0) return hip_ok(hipMemsetAsync(d_out_off, 0, 8, s));
  const uint64_t np = (uint64_t)nm + nseg;  // pieces: a table per message + the segments
  if (np > 0xffffffffull) return CPK_EINVAL;
  const uint32_t nb = (uint32_t)((np + cpk::kE4ScanBlock - 1) / cpk::kE4ScanBlock);
  // scratch: segment sizes | table sizes | message-order sizes | segment offsets | block sums
  int rc = ensure_status(ctx, (uint64_t)nseg + nm + np + nseg + nb + 1);
  if (rc) return rc;
  uint64_t *ssize = ctx->status, *tsize = ssize + nseg, *comb = tsize + nm, *soff = comb + np;
  uint64_t *bsum = soff + nseg;
  uint64_t stride = (max_seg_words + 63) / 64;
  if (nseg && stride > (1ull << 29) / nseg) return CPK_EUNSUPPORTED;  // (> 4 GiB of step rows)
  const uint64_t rows = (uint64_t)(nseg ? nseg : 1) * stride;
  if (rows > ctx->e4_bv_cap) {
    if (ctx->e4_bv) hipFree(ctx->e4_bv);
    ctx->e4_bv = nullptr;
    ctx->e4_bv_cap = 0;
    const uint64_t cap = rows + rows / 4;
    if (hipMalloc(&ctx->e4_bv, cap * 8) != hipSuccess) return CPK_ENOMEM;
    ctx->e4_bv_cap = cap;
  }
  if (hipMemsetAsync(ctx->tickets, 0, cpk::kTkErr * 4, s) != hipSuccess) return CPK_EDEVICE;
  const unsigned tb = 256, tg = (nm + tb - 1) / tb;
  unsigned grid = (unsigned)(8 * ctx->cus);
  if (grid > (nseg + cpk::kE4Waves - 1) / cpk::kE4Waves) grid = (nseg + cpk::kE4Waves - 1) / cpk::kE4Waves;
  if (nseg)
    hipLaunchKernelGGL(cpk::e4_size_kernel, dim3(grid), dim3(cpk::kE4Threads), 0, s,
                       (const uint64_t *)d_in, d_swo, nseg, ssize, ctx->tickets + cpk::kTkEnc,
                       max_seg_words, ctx->tickets + cpk::kTkErr, ctx->e4_bv, stride);
  hipLaunchKernelGGL(cpk::msg_table_size_kernel, dim3(tg), dim3(tb), 0, s, d_swo, d_msg_seg_off, nm,
                     tsize);
  hipLaunchKernelGGL(cpk::msg_interleave_kernel, dim3(tg), dim3(tb), 0, s, d_msg_seg_off, nm,
                     (const uint64_t *)tsize, (const uint64_t *)ssize, comb);
  hipLaunchKernelGGL(cpk::e4_scan_reduce, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)comb, (uint32_t)np, bsum);
  hipLaunchKernelGGL(cpk::e4_scan_top, dim3(1), dim3(cpk::kE4ScanThreads), 0, s, bsum, nb);
  hipLaunchKernelGGL(cpk::e4_scan_down, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)comb, (uint32_t)np, (const uint64_t *)bsum, d_out_off);
  hipLaunchKernelGGL(cpk::msg_table_emit_kernel, dim3(tg), dim3(tb), 0, s, d_swo, d_msg_seg_off, nm,
                     (const uint64_t *)d_out_off, soff, (uint8_t *)d_out);
  if (nseg)
    hipLaunchKernelGGL(cpk::e4_emit_kernel, dim3(grid), dim3(cpk::kE4Threads), cpk::kE4Lds, s,
                       (const uint64_t *)d_in, d_swo, nseg, (const uint64_t *)soff, (uint8_t *)d_out,
                       ctx->tickets + cpk::kTkDec, (const uint64_t *)ctx->e4_bv, stride);
  return hip_ok(hipGetLastError());
}

int cpk_encode_batch(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t n,
                     uint64_t max_seg_words, void *d_out, uint64_t *d_out_off, void *stream) {
  if (!ctx || (!d_swo && n) || !d_out_off) return CPK_EINVAL;
  if (((uintptr_t)d_out & 15) || ((uintptr_t)d_in & 7)) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return hip_ok(hipMemsetAsync(d_out_off, 0, 8, s));
  if (ctx->encoder == 3) return e3_encode(ctx, d_in, d_swo, n, max_seg_words, d_out, d_out_off, s);
  if (ctx->encoder == 4) return e4_encode(ctx, d_in, d_swo, n, max_seg_words, d_out, d_out_off, s);
  // counters (not the error word: that is cleared by cpk_ctx_take_error)
  if (hipMemsetAsync(ctx->tickets, 0, cpk::kTkErr * 4, s) != hipSuccess) return CPK_EDEVICE;
  const bool v2 = ctx->encoder == 2;
  if (!v2 && max_seg_words != 0 && max_seg_words <= (uint64_t)cpk::kTileWords) {
    // one workgroup per piece
    int rc = ensure_status(ctx, n);
    if (rc) return rc;
    if (hipMemsetAsync(ctx->status, 0, (size_t)n * 8, s) != hipSuccess) return CPK_EDEVICE;
    unsigned grid = (unsigned)(2 * ctx->cus);
    if (grid > n) grid = n;
    hipLaunchKernelGGL(cpk::encode_kernel<false>, dim3(grid), dim3(cpk::kEncThreads), cpk::kEncLds,
                       s, (const uint64_t *)d_in, d_swo, n, (uint8_t *)d_out, d_out_off, ctx->status,
                       ctx->tickets, (const uint32_t *)nullptr, (const uint64_t *)nullptr,
                       (uint64_t *)nullptr, ctx->tickets + cpk::kTkErr);
    return hip_ok(hipGetLastError());
  }
  // tiled: pieces cut into tiles (1024 words for the wave-per-tile encoder,
  // 8192 for the workgroup one); the tile count is bounded from the hint, or
  // from the batch's word count when there is no hint
  const uint64_t tw = v2 ? (uint64_t)cpk::kE2Words : (uint64_t)cpk::kTileWords;
  uint64_t tiles;
  if (max_seg_words) {
    tiles = (uint64_t)n * ((max_seg_words + tw - 1) / tw);
  } else {
    uint64_t ends[2];
    if (hipMemcpyAsync(&ends[0], d_swo, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&ends[1], d_swo + n, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return CPK_EDEVICE;
    tiles = (uint64_t)n + (ends[1] - ends[0]) / tw;
  }
  const uint64_t blocks = ((uint64_t)n + cpk::kPlanThreads * cpk::kPlanPer - 1) /
                          (cpk::kPlanThreads * cpk::kPlanPer);
  const uint64_t o_tmap = align256(((uint64_t)n + 1) * 8);
  const uint64_t o_pst = o_tmap + align256(tiles * 4);
  const uint64_t o_tst = o_pst + align256(blocks * 8);
  const uint64_t bytes = o_tst + align256(tiles * 8);
  int rc = ensure_plan(ctx, bytes);
  if (rc) return rc;
  rc = ensure_status(ctx, tiles);
  if (rc) return rc;
  uint8_t *plan = (uint8_t *)ctx->plan;
  uint64_t *toff = (uint64_t *)plan;
  uint32_t *tmap = (uint32_t *)(plan + o_tmap);
  uint64_t *pst = (uint64_t *)(plan + o_pst);
  uint64_t *tst = (uint64_t *)(plan + o_tst);
  if (hipMemsetAsync(pst, 0, blocks * 8, s) != hipSuccess ||
      hipMemsetAsync(tst, 0, tiles * 8, s) != hipSuccess ||
      hipMemsetAsync(ctx->status, 0, tiles * 8, s) != hipSuccess)
    return CPK_EDEVICE;
  if (v2) {
    hipLaunchKernelGGL(cpk::tile_plan_kernel<cpk::kE2Words>, dim3((unsigned)blocks),
                       dim3(cpk::kPlanThreads), 0, s, d_swo, n, toff, tmap, tiles, pst,
                       ctx->tickets + cpk::kTkPlan, ctx->tickets + cpk::kTkErr);
    // persistent: 6 workgroups of 4 independent waves per CU
    unsigned grid = (unsigned)(6 * ctx->cus);
    if (grid > (tiles + 3) / 4) grid = (unsigned)((tiles + 3) / 4);
    hipLaunchKernelGGL(cpk::encode2_kernel, dim3(grid), dim3(cpk::kE2Threads), cpk::kE2Lds, s,
                       (const uint64_t *)d_in, d_swo, n, (uint8_t *)d_out, d_out_off, ctx->status,
                       ctx->tickets, (const uint32_t *)tmap, (const uint64_t *)toff, tst);
    return hip_ok(hipGetLastError());
  }
  hipLaunchKernelGGL(cpk::tile_plan_kernel<cpk::kTileWords>, dim3((unsigned)blocks),
                     dim3(cpk::kPlanThreads), 0, s, d_swo, n, toff, tmap, tiles, pst,
                     ctx->tickets + cpk::kTkPlan, ctx->tickets + cpk::kTkErr);
  unsigned grid = (unsigned)(2 * ctx->cus);
  if (grid > tiles) grid = (unsigned)tiles;
  hipLaunchKernelGGL(cpk::encode_kernel<true>, dim3(grid), dim3(cpk::kEncThreads), cpk::kEncLds, s,
                     (const uint64_t *)d_in, d_swo, n, (uint8_t *)d_out, d_out_off, ctx->status,
                     ctx->tickets, (const uint32_t *)tmap, (const uint64_t *)toff, tst,
                     ctx->tickets + cpk::kTkErr);
  return hip_ok(hipGetLastError());
}

int cpk_ctx_take_error(cpk_ctx ctx, void *stream) {
  if (!ctx) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  uint32_t e = 0;
  if (hipMemcpyAsync(&e, ctx->tickets + cpk::kTkErr, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CPK_EDEVICE;
  if (e && hipMemsetAsync(ctx->tickets + cpk::kTkErr, 0, 4, s) != hipSuccess) return CPK_EDEVICE;
  // bits 0, 1: a piece over its size hint (encoder / tile plan); bit 2: a
  // cross-workgroup wait timed out (a grid larger than the device holds at
  // once -- cannot happen by design)
  return e ? ((e & 4u) ? CPK_EDEVICE : CPK_EINVAL) : CPK_OK;
}

int cpk_decode_batch(cpk_ctx ctx, const void *d_packed, const uint64_t *d_in_off,
                     const uint64_t *d_swo, uint32_t n, void *d_out, int32_t *d_status,
                     void *stream) {
  if (!ctx || (n && (!d_in_off || !d_swo || !d_status))) return CPK_EINVAL;
  if (((uintptr_t)d_packed & 15) || ((uintptr_t)d_out & 7)) return CPK_EINVAL;
  if (n == 0) return CPK_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(ctx->tickets + cpk::kTkDec, 0, 8 * cpk::kTkStride * 4, s) != hipSuccess)
    return CPK_EDEVICE;
  // persistent: up to 8 blocks of 4 independent waves per CU (32 pieces in
  // flight), as many as the LDS holds
  const unsigned per_cu = (unsigned)min(8u, 160u * 1024u / cpk::kDecLds);
  unsigned grid = per_cu * (unsigned)ctx->cus;
  if (grid > (n + 3) / 4) grid = (n + 3) / 4;
  hipLaunchKernelGGL(cpk::decode_kernel<false>, dim3(grid), dim3(cpk::kDecThreads), cpk::kDecLds, s,
                     (const uint8_t *)d_packed, const_cast<uint64_t *>(d_in_off), d_swo, n,
                     (uint64_t *)d_out, d_status, ctx->tickets + cpk::kTkDec, (uint64_t)0,
                     cpk::DecStreams{nullptr, nullptr, nullptr, 0, nullptr});
  return hip_ok(hipGetLastError());
}

int cpk_decode_stream(cpk_ctx ctx, const void *d_packed, uint64_t avail,
                      const uint64_t *d_swo, uint32_t n, void *d_out, uint64_t *d_in_off,
                      int32_t *d_status, void *stream) {
  if (!ctx || (n && (!d_in_off || !d_swo || !d_status))) return CPK_EINVAL;
  if (((uintptr_t)d_packed & 15) || ((uintptr_t)d_out & 7)) return CPK_EINVAL;
  if (n == 0) return CPK_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(ctx->tickets + cpk::kTkDec, 0, 8 * cpk::kTkStride * 4, s) != hipSuccess)
    return CPK_EDEVICE;
  // one stream: one wave works, the others find no ticket
  hipLaunchKernelGGL(cpk::decode_kernel<true>, dim3(1), dim3(cpk::kDecThreads), cpk::kDecLds, s,
                     (const uint8_t *)d_packed, d_in_off, d_swo, n, (uint64_t *)d_out, d_status,
                     ctx->tickets + cpk::kTkDec, avail,
                     cpk::DecStreams{nullptr, nullptr, nullptr, 1, d_in_off + n});
  return hip_ok(hipGetLastError());
}

int cpk_decode_messages(cpk_ctx ctx, const void *d_packed, const uint64_t *d_msg_off, uint32_t nm,
                        uint64_t traversal_limit_words, void *d_out, uint64_t out_cap_words,
                        uint64_t *d_seg_word_off, uint64_t *d_seg_in_off, int32_t *d_seg_status,
                        uint32_t seg_cap, uint64_t *d_msg_seg_off, int32_t *d_msg_status,
                        uint64_t *h_totals, void *stream) {
  if (!ctx || !h_totals || (nm && (!d_msg_off || !d_msg_seg_off || !d_msg_status))) return CPK_EINVAL;
  if (((uintptr_t)d_packed & 15) || ((uintptr_t)d_out & 7)) return CPK_EINVAL;
  h_totals[0] = h_totals[1] = 0;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (nm == 0) return hip_ok(hipMemsetAsync(d_msg_seg_off, 0, 8, s));
  // scratch: words | begin | words offsets [nm+1] | block sums x2
  const uint32_t nb = (uint32_t)((nm + cpk::kE4ScanBlock - 1) / cpk::kE4ScanBlock);
  int rc = ensure_status(ctx, 3ull * nm + 1 + 2ull * nb);
  if (rc) return rc;
  uint64_t *mwords = ctx->status, *mbeg = mwords + nm, *mwoff = mbeg + nm;
  uint64_t *bs0 = mwoff + nm + 1, *bs1 = bs0 + nb;
  const unsigned tb = 256, tg = (nm + tb - 1) / tb;
  // the segment counts go to d_msg_seg_off[0..nm) and are scanned into it
  // (e4_scan_down: each thread reads its entries before it writes them)
  hipLaunchKernelGGL(cpk::msg_table_kernel, dim3(tg), dim3(tb), 0, s, (const uint8_t *)d_packed,
                     d_msg_off, nm, traversal_limit_words, mwords, d_msg_seg_off, mbeg, d_msg_status);
  hipLaunchKernelGGL(cpk::e4_scan_reduce, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)mwords, nm, bs0);
  hipLaunchKernelGGL(cpk::e4_scan_reduce, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)d_msg_seg_off, nm, bs1);
  hipLaunchKernelGGL(cpk::e4_scan_top, dim3(1), dim3(cpk::kE4ScanThreads), 0, s, bs0, nb);
  hipLaunchKernelGGL(cpk::e4_scan_top, dim3(1), dim3(cpk::kE4ScanThreads), 0, s, bs1, nb);
  hipLaunchKernelGGL(cpk::e4_scan_down, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)mwords, nm, (const uint64_t *)bs0, mwoff);
  hipLaunchKernelGGL(cpk::e4_scan_down, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)d_msg_seg_off, nm, (const uint64_t *)bs1, d_msg_seg_off);
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(&h_totals[0], mwoff + nm, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(&h_totals[1], d_msg_seg_off + nm, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CPK_EDEVICE;
  if (h_totals[0] > out_cap_words || h_totals[1] > seg_cap) return CPK_ENOMEM;
  if (h_totals[1] && (!d_seg_word_off || !d_seg_in_off || !d_seg_status)) return CPK_EINVAL;
  if (!d_seg_word_off) return CPK_OK;  // (no segments: every table failed)
  hipLaunchKernelGGL(cpk::msg_swo_kernel, dim3(tg), dim3(tb), 0, s, (const uint8_t *)d_packed,
                     d_msg_off, nm, traversal_limit_words, (const uint64_t *)mwoff,
                     (const uint64_t *)d_msg_seg_off, (const int32_t *)d_msg_status, d_seg_word_off);
  if (h_totals[1]) {
    if (hipMemsetAsync(ctx->tickets + cpk::kTkDec, 0, 8 * cpk::kTkStride * 4, s) != hipSuccess)
      return CPK_EDEVICE;
    const unsigned per_cu = (unsigned)min(8u, 160u * 1024u / cpk::kDecLds);
    unsigned grid = per_cu * (unsigned)ctx->cus;
    if (grid > (nm + 3) / 4) grid = (nm + 3) / 4;
    // the stream ends overwrite the words array (no longer needed)
    hipLaunchKernelGGL(cpk::decode_kernel<true>, dim3(grid), dim3(cpk::kDecThreads), cpk::kDecLds, s,
                       (const uint8_t *)d_packed, d_seg_in_off, (const uint64_t *)d_seg_word_off,
                       (uint32_t)h_totals[1], (uint64_t *)d_out, d_seg_status,
                       ctx->tickets + cpk::kTkDec, (uint64_t)0,
                       cpk::DecStreams{mbeg, d_msg_off + 1, d_msg_seg_off, nm, mwords});
    hipLaunchKernelGGL(cpk::msg_final_kernel, dim3(tg), dim3(tb), 0, s, d_msg_off, nm,
                       (const uint64_t *)d_msg_seg_off, (const uint64_t *)mwords,
                       (const int32_t *)d_seg_status, d_msg_status);
  }
  return hip_ok(hipGetLastError());
}

int cpk_decode_stream_host(cpk_ctx ctx, const void *h_packed, uint64_t avail,
                           const uint64_t *h_swo, uint32_t n, void *h_out, uint64_t *h_in_off,
                           int32_t *h_status) {
  if (!ctx || !h_swo || !h_in_off || !h_status) return CPK_EINVAL;
  if (n == 0) {
    h_in_off[0] = 0;
    return CPK_OK;
  }
  DeviceGuard g(ctx->device);
  uint64_t words = h_swo[n] - h_swo[0];
  void *d_pk = nullptr, *d_out = nullptr;
  uint64_t *d_swo = nullptr, *d_io = nullptr;
  int32_t *d_st = nullptr;
  int rc = CPK_OK;
  std::vector<uint64_t> rs;
  if (hipMalloc(&d_pk, avail + 64) != hipSuccess || hipMalloc(&d_out, words * 8 + 8) != hipSuccess ||
      hipMalloc(&d_swo, (n + 1) * 8ull) != hipSuccess ||
      hipMalloc(&d_io, (n + 1) * 8ull) != hipSuccess || hipMalloc(&d_st, n * 4ull) != hipSuccess) {
    rc = CPK_ENOMEM;
    goto done;
  }
  rs.resize(n + 1);
  for (uint32_t i = 0; i <= n; ++i) rs[i] = h_swo[i] - h_swo[0];
  if (hipMemset(d_pk, 0, avail + 64) ||
      (avail && hipMemcpy(d_pk, h_packed, avail, hipMemcpyHostToDevice)) ||
      hipMemcpy(d_swo, rs.data(), (n + 1) * 8ull, hipMemcpyHostToDevice)) {
    rc = CPK_EDEVICE;
    goto done;
  }
  rc = cpk_decode_stream(ctx, d_pk, avail, d_swo, n, d_out, d_io, d_st, nullptr);
  if (rc) goto done;
  if (hipMemcpy(h_status, d_st, n * 4ull, hipMemcpyDeviceToHost) ||
      hipMemcpy(h_in_off, d_io, (n + 1) * 8ull, hipMemcpyDeviceToHost) ||
      (words && hipMemcpy((uint8_t *)h_out + 8 * h_swo[0], d_out, words * 8, hipMemcpyDeviceToHost))) {
    rc = CPK_EDEVICE;
    goto done;
  }
  for (uint32_t i = 0; i < n; ++i)
    if (h_status[i] != CPK_OK) {
      rc = h_status[i];
      break;
    }
done:
  if (d_pk) hipFree(d_pk);
  if (d_out) hipFree(d_out);
  if (d_swo) hipFree(d_swo);
  if (d_io) hipFree(d_io);
  if (d_st) hipFree(d_st);
  return rc;
}

int cpk_generate(cpk_ctx ctx, const cpk_gen_params *params, const uint64_t *d_swo, uint32_t n,
                 void *d_out, void *stream) {
  if (!ctx || !params) return CPK_EINVAL;
  if (n == 0) return CPK_OK;
  DeviceGuard g(ctx->device);
  unsigned grid = (n + 255) / 256;
  hipLaunchKernelGGL(cpk::generate_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, *params,
                     d_swo, n, (uint64_t *)d_out);
  return hip_ok(hipGetLastError());
}

int cpk_count_mismatch(cpk_ctx ctx, const void *d_a, const void *d_b, uint64_t words,
                       uint64_t *d_mismatch, void *stream) {
  if (!ctx) return CPK_EINVAL;
  if (words == 0) return CPK_OK;
  DeviceGuard g(ctx->device);
  unsigned grid = (unsigned)(8 * ctx->cus);
  hipLaunchKernelGGL(cpk::mismatch_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (const uint64_t *)d_a, (const uint64_t *)d_b, words,
                     (unsigned long long *)d_mismatch);
  return hip_ok(hipGetLastError());
}

}  // extern "C"
