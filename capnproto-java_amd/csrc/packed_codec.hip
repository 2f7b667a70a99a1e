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
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

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

// ---------------------------------------------------------------- LDS maps
// Encoder: staging for the packed bytes of one piece (bound 9*8192 = 73,728)
// plus 16 bytes of alignment pad and slack; then LUT, bitmaps, scratch.
constexpr uint32_t kEncStage = 9 * kTileWords + 64;
constexpr uint32_t kEncLut = kEncStage;                 // u64[256]
constexpr uint32_t kEncDbits = kEncLut + 2048;          // u32[256]
constexpr uint32_t kEncHbits = kEncDbits + 1024;        // u32[256]
constexpr uint32_t kEncScr = kEncHbits + 1024;          // int[128]
constexpr uint32_t kEncLds = kEncScr + 512;             // 78,400 B -> 2 WG / CU

// Decoder: LUT, resolve/blk region, scratch, packed bytes.
constexpr uint32_t kDecPkCap = 9 * kTileWords;          // canonical bound
constexpr uint32_t kDecLut = 0;                         // u64[256]
constexpr uint32_t kDecReg = 2048;                      // 4736 B union
constexpr uint32_t kDecScr = kDecReg + 4736;            // int[128]
constexpr uint32_t kDecPk = kDecScr + 512;              // 7296, 16-aligned
constexpr uint32_t kDecLds = kDecPk + 32 + kDecPkCap + 32;  // 81,088 B
constexpr int kMaxChunks = 512;
constexpr uint32_t kWarm = 16;                          // warm-up bytes per walk

static_assert(kDecPk % 16 == 0, "packed region must be 16-aligned");
static_assert(kEncLut % 16 == 0, "lut must be aligned");
static_assert(kDecLds <= 81920 && kEncLds <= 81920, "2 workgroups per CU");

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
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

// Called by all 64 lanes of one wave.  Returns the exclusive prefix.
__device__ uint64_t lookback(uint64_t *status, uint32_t tile, uint64_t agg) {
  const int lane = lane_id();
  if (tile == 0) {
    if (lane == 0) st_status(&status[0], kFlagInc | agg);
    return 0;
  }
  if (lane == 0) st_status(&status[tile], kFlagAgg | agg);
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

// Append string (d2:d1:d0, len bytes) to a chunk byte stream in LDS.
struct Emitter {
  uint32_t *stage32;
  int dw, fill, first_dw, last_dw;
  uint32_t a0;
  __device__ __forceinline__ void put(int d, uint32_t v) {
    if (d == first_dw || d == last_dw) atomicOr(&stage32[d], v);
    else stage32[d] = v;
  }
  __device__ __forceinline__ void append(uint32_t d0, uint32_t d1, uint32_t d2, int len) {
    if (len == 0) return;
    uint32_t sh = 8u * (uint32_t)fill;
    uint64_t s01 = (uint64_t)d0 | ((uint64_t)d1 << 32);
    uint64_t lo64 = s01 << sh;
    uint64_t hi64 = ((uint64_t)d2 << sh) | (sh ? (s01 >> (64 - sh)) : 0ull);
    uint32_t t0 = (uint32_t)lo64 | a0, t1 = (uint32_t)(lo64 >> 32);
    uint32_t t2 = (uint32_t)hi64, t3 = (uint32_t)(hi64 >> 32);
    int nf = fill + len;
    int k = nf >> 2;
    if (k >= 1) put(dw, t0);
    if (k >= 2) put(dw + 1, t1);
    if (k >= 3) put(dw + 2, t2);
    a0 = k == 0 ? t0 : k == 1 ? t1 : k == 2 ? t2 : t3;
    dw += k;
    fill = nf & 3;
  }
  __device__ __forceinline__ void finish() {
    if (fill) put(dw, a0);
  }
};

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

template <bool kUnused = false>
__global__ __launch_bounds__(kThreads, 4) void encode_kernel(
    const uint64_t *__restrict__ in, const uint64_t *__restrict__ swo, uint32_t n,
    uint8_t *__restrict__ out, uint64_t *__restrict__ out_off, uint64_t *status,
    uint32_t *ticket) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t *stage = smem;
  uint32_t *stage32 = reinterpret_cast<uint32_t *>(smem);
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem + kEncLut);
  uint32_t *dbits = reinterpret_cast<uint32_t *>(smem + kEncDbits);
  uint32_t *hbits = reinterpret_cast<uint32_t *>(smem + kEncHbits);
  int *scr = reinterpret_cast<int *>(smem + kEncScr);
  // scr[0..15] F1 wave totals, scr[16..23] B1, scr[32..39] F2,
  // scr[64..65] ticket (alternating), scr[66..67] piece base (u64)

  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  fill_luts(lut, false);

  for (uint32_t it = 0;; ++it) {
    // ticket slot alternates: a wave still reading this piece's slot can
    // never see the next piece's ticket (one barrier per iteration)
    if (tid == 0) scr[64 + (it & 1)] = (int)atomicAdd(ticket, 1u);
    __syncthreads();  // also orders the previous piece's LDS use
    const uint32_t seg = (uint32_t)scr[64 + (it & 1)];
    if (seg >= n) break;
    const uint64_t w0 = swo[seg];
    const int W = (int)(swo[seg + 1] - w0);  // <= kTileWords (host-checked)
    // opaque per piece: stops the compiler hoisting per-lane address math
    // out of the persistent loop (it spilled it all to scratch)
    int kbase = w * kWaveWords + lane * kChunk;
    asm volatile("" : "+v"(kbase));
#define KW(j, i) (kbase + (j) * 256 + (i))
#define BIT(j, i) (1u << ((j) * kChunk + (i)))

    // ---- load + classify ----------------------------------------------------
    // vbits: bit (j*4+i) set iff word (j,i) is inside the piece.  Loads are
    // clamped to the last word instead of predicated (no per-word branches).
    uint32_t vbits = 0;
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      int nv = min(max(W - (kbase + j * 256), 0), kChunk);
      vbits |= ((1u << nv) - 1) << (j * kChunk);
    }
    uint32_t lo[kJ][kChunk], hi[kJ][kChunk];
    uint32_t msk4[kJ];  // nonzero-byte mask of word i in byte i
    const uint64_t *src = in + w0;
    const int wlast = max(W - 1, 0);
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
#pragma unroll
      for (int i = 0; i < kChunk; ++i) {
        uint64_t v = W ? src[min(KW(j, i), wlast)] : 0ull;
        v = (vbits & BIT(j, i)) ? v : 0ull;
        lo[j][i] = (uint32_t)v;
        hi[j][i] = (uint32_t)(v >> 32);
      }
      uint32_t m4 = 0;
#pragma unroll
      for (int i = 0; i < kChunk; ++i) m4 |= word_mask(lo[j][i], hi[j][i]) << (8 * i);
      msk4[j] = m4;
    }
#define MSK(j, i) ((msk4[j] >> (8 * (i))) & 0xffu)
#define VALID(j, i) ((vbits & BIT(j, i)) != 0)
    // group of the word just before this wave's first word
    int gprev = 3;
    if (w > 0 && lane == 0) {
      int k = w * kWaveWords - 1;
      if (k < W) {
        uint64_t v = in[w0 + k];
        gprev = grp_of(word_mask((uint32_t)v, (uint32_t)(v >> 32)));
      }
    }
    gprev = readlane(gprev, 0);

    // run starts: word k < W starts a run if k == 0 or its group differs
    uint32_t sbits = 0;
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const int glast = VALID(j, kChunk - 1) ? grp_of(MSK(j, kChunk - 1)) : 3;
      int pg = wave_shr1(glast, gprev);
      int gp = pg;
#pragma unroll
      for (int i = 0; i < kChunk; ++i) {
        const int k = KW(j, i);
        const int g = VALID(j, i) ? grp_of(MSK(j, i)) : 3;
        if (g != 3 && (k == 0 || g != gp)) sbits |= BIT(j, i);
        gp = g;
      }
      gprev = readlane(glast, 63);
    }

    // ---- B1: run end e(k) = next run start after k (or W) ----------------
    CPK_OPAQUE(sbits);
    CPK_OPAQUE(vbits);
    // erel[j]: e - k of words (j,0),(j,1) in halves of erel[j][0], etc.
    uint32_t erel[kJ][2];
    {
      int cE = kBig;
      int pE[kJ];
#pragma unroll
      for (int j = kJ - 1; j >= 0; --j) {
        int aE = kBig;
#pragma unroll
        for (int i = kChunk - 1; i >= 0; --i)
          if (sbits & BIT(j, i)) aE = KW(j, i);
        int iE = wave_sufx_min(aE);
        int xE = __shfl(iE, min(lane + 1, 63), 64);
        if (lane == 63) xE = kBig;
        pE[j] = min(cE, xE);
        cE = min(cE, readlane(iE, 0));
      }
      if (lane == 0) scr[16 + w] = cE;
      __syncthreads();
      int wE = kBig;
      for (int q = w + 1; q < kWaves; ++q) wE = min(wE, scr[16 + q]);
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        int r = min(wE, pE[j]);
        uint32_t e3, e2, e1, e0;
        e3 = (uint32_t)max(min(r, W) - KW(j, 3), 0);
        if (sbits & BIT(j, 3)) r = KW(j, 3);
        e2 = (uint32_t)max(min(r, W) - KW(j, 2), 0);
        if (sbits & BIT(j, 2)) r = KW(j, 2);
        e1 = (uint32_t)max(min(r, W) - KW(j, 1), 0);
        if (sbits & BIT(j, 1)) r = KW(j, 1);
        e0 = (uint32_t)max(min(r, W) - KW(j, 0), 0);
        erel[j][0] = e0 | (e1 << 16);
        erel[j][1] = e2 | (e3 << 16);
      }
    }
#define EREL(j, i) ((erel[j][(i) >> 1] >> (16 * ((i) & 1))) & 0xffffu)

    // ---- F1: run start s(k), last D before k -> roles ---------------------
    // zhead : Z word that emits a 0x00 tag (every 256th word of its run,
    //         PackedOutputStream.java:125-131)
    // member: D/L word copied verbatim inside a 0xFF literal run (:133-193)
    // lng   : D/L word of a stretch longer than 256 words (chain below)
    // cnt4  : run count byte of Z / D heads, min(255, e - k - 1)
    uint32_t zhead = 0, member = 0, lng = 0;
    uint32_t cnt4[kJ];
    CPK_OPAQUE(sbits);
    CPK_OPAQUE(vbits);
#pragma unroll
    for (int j = 0; j < kJ; ++j) CPK_OPAQUE(msk4[j]);
    {
      int cS = -1, cD = -1;
      int pS[kJ], pD[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        int aS = -1, aD = -1;
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
          if (sbits & BIT(j, i)) aS = KW(j, i);
          if (MSK(j, i) == 0xffu) aD = KW(j, i);
        }
        int iS = wave_incl_max(aS), iD = wave_incl_max(aD);
        pS[j] = max(cS, wave_shr1(iS, -1));
        pD[j] = max(cD, wave_shr1(iD, -1));
        cS = max(cS, readlane(iS, 63));
        cD = max(cD, readlane(iD, 63));
      }
      if (lane == 0) {
        scr[2 * w] = cS;
        scr[2 * w + 1] = cD;
      }
      __syncthreads();
      int wS = -1, wD = -1;
      for (int q = 0; q < w; ++q) {
        wS = max(wS, scr[2 * q]);
        wD = max(wD, scr[2 * q + 1]);
      }
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        int rs = max(wS, pS[j]), rd = max(wD, pD[j]);
        uint32_t c4 = 0;
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
          const int k = KW(j, i);
          const uint32_t m = MSK(j, i);
          if (sbits & BIT(j, i)) rs = k;
          const int er = (int)EREL(j, i);
          c4 |= (uint32_t)min(255, max(er - 1, 0)) << (8 * i);
          if (VALID(j, i)) {
            const int g = grp_of(m);
            if (g == 0 && ((k - rs) & 255) == 0) zhead |= BIT(j, i);
            if (g == 1) {
              if (k + er - rs > 256) lng |= BIT(j, i);
              else if (rd >= rs) member |= BIT(j, i);
            }
          }
          if (m == 0xffu) rd = k;
        }
        cnt4[j] = c4;
      }
    }

    if (__syncthreads_or(lng != 0)) {
      // D/L stretch longer than 256 words: heads chain h1 = first D,
      // h' = first D at or after h + 256 (the 255-word cap of
      // PackedOutputStream.java:145-147).  Walked by the run's first word.
      // dbits = D words, hbits = run starts, then (after the walk) heads.
      if (tid < 256) dbits[tid] = 0;
      else hbits[tid - 256] = 0;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kJ; ++j)
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
          const int k = KW(j, i);
          if (MSK(j, i) == 0xffu && VALID(j, i)) atomicOr(&dbits[k >> 5], 1u << (k & 31));
          if (sbits & BIT(j, i)) atomicOr(&hbits[k >> 5], 1u << (k & 31));
        }
      __syncthreads();
      // run start of every long-stretch word (last start bit <= k)
      int sl[kJ][kChunk];
#pragma unroll
      for (int j = 0; j < kJ; ++j)
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
          sl[j][i] = 0;
          if (lng & BIT(j, i)) {
            int k = KW(j, i), d = k >> 5;
            uint32_t m = hbits[d] & ((k & 31) == 31 ? ~0u : ((2u << (k & 31)) - 1));
            while (!m) m = hbits[--d];
            sl[j][i] = d * 32 + 31 - __builtin_clz(m);
          }
        }
      __syncthreads();
      if (tid < 256) hbits[tid] = 0;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kJ; ++j)
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
          if ((lng & sbits & BIT(j, i)) == 0) continue;
          const int k = KW(j, i);
          const int e = k + (int)EREL(j, i);
          int h = bm_next(dbits, k, e);
          while (h < e) {
            atomicOr(&hbits[h >> 5], 1u << (h & 31));
            int p = h + 256;
            if (p >= e) break;
            h = bm_next(dbits, p, e);
          }
        }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kJ; ++j)
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
          if ((lng & BIT(j, i)) == 0) continue;
          const int k = KW(j, i);
          if (bm_any(hbits, max(sl[j][i], k - 255), k - 1)) member |= BIT(j, i);
        }
    }

    // bytes emitted by word (j, i)
#define NBYTES(j, i)                                                              \
  (!VALID(j, i) ? 0                                                               \
   : MSK(j, i) == 0 ? ((zhead & BIT(j, i)) ? 2 : 0)                               \
   : (member & BIT(j, i)) ? 8                                                     \
   : (MSK(j, i) == 0xffu ? 10 : 1 + __builtin_popcount(MSK(j, i))))

    // ---- F2: byte offsets (exclusive sum over the piece) ------------------
    CPK_OPAQUE(vbits);
    CPK_OPAQUE(zhead);
    CPK_OPAQUE(member);
#pragma unroll
    for (int j = 0; j < kJ; ++j) CPK_OPAQUE(msk4[j]);
    int choff[kJ], chlen[kJ];
    int total;
    {
      int c = 0;
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        int a = 0;
#pragma unroll
        for (int i = 0; i < kChunk; ++i) a += NBYTES(j, i);
        chlen[j] = a;
        int inc = wave_incl_add(a);
        choff[j] = c + inc - a;
        c += readlane(inc, 63);
      }
      if (lane == 0) scr[32 + w] = c;
      __syncthreads();
      int wb = 0;
      total = 0;
      for (int q = 0; q < kWaves; ++q) {
        int t = scr[32 + q];
        if (q < w) wb += t;
        total += t;
      }
#pragma unroll
      for (int j = 0; j < kJ; ++j) choff[j] += wb;
    }

    // ---- look-back for the piece's output offset ---------------------------
    if (w == 0) {
      uint64_t base = lookback(status, seg, (uint64_t)total);
      if (lane == 0) {
        *reinterpret_cast<uint64_t *>(&scr[66]) = base;
        out_off[seg] = base;
        if (seg == n - 1) out_off[n] = base + (uint64_t)total;
      }
    }
    __syncthreads();
    const uint64_t base = *reinterpret_cast<uint64_t *>(&scr[66]);
    const int pad = (int)(base & 15);

    // ---- compact the packed bytes into LDS ----------------------------------
    CPK_OPAQUE(vbits);
    CPK_OPAQUE(zhead);
    CPK_OPAQUE(member);
#pragma unroll
    for (int j = 0; j < kJ; ++j) CPK_OPAQUE(msk4[j]);
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      if (chlen[j] > 0) {
        int cs = pad + choff[j], ce = cs + chlen[j];
        stage32[cs >> 2] = 0;
        stage32[(ce - 1) >> 2] = 0;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      if (chlen[j] == 0) continue;
      const int cs = pad + choff[j], ce = cs + chlen[j];
      Emitter em;
      em.stage32 = stage32;
      em.dw = cs >> 2;
      em.fill = cs & 3;
      em.first_dw = cs >> 2;
      em.last_dw = (ce - 1) >> 2;
      em.a0 = 0;
#pragma unroll
      for (int i = 0; i < kChunk; ++i) {
        const int len = NBYTES(j, i);
        if (len == 0) continue;
        const uint32_t l = lo[j][i], h = hi[j][i], m = MSK(j, i);
        uint32_t d0, d1, d2;
        if (member & BIT(j, i)) {
          d0 = l;
          d1 = h;
          d2 = 0;
        } else {
          const uint64_t sel = lut[m];
          const uint32_t c0 = __builtin_amdgcn_perm(h, l, (uint32_t)sel);
          const uint32_t c1 = __builtin_amdgcn_perm(h, l, (uint32_t)(sel >> 32));
          d0 = m | (c0 << 8);
          d1 = (c0 >> 24) | (c1 << 8);
          d2 = c1 >> 24;
          // run count after the tag (and after the 8 bytes of a 0xFF word),
          // capped at 255 (PackedOutputStream.java:125-131, :145-164)
          const uint32_t cnt = (cnt4[j] >> (8 * i)) & 0xffu;
          if (m == 0) d0 |= cnt << 8;
          else if (m == 0xffu) d2 |= cnt << 8;
        }
        em.append(d0, d1, d2, len);
      }
      em.finish();
    }
    __syncthreads();

    // ---- store: 16-byte lines, byte stores at the two shared edges --------
    {
      const int tb = pad + total;
      uint8_t *gbase = out + (base - (uint64_t)pad);
      const int nl = (tb + 15) >> 4;
      for (int c = tid; c < nl; c += kThreads) {
        int lo16 = c * 16, hi16 = lo16 + 16;
        if (lo16 >= pad && hi16 <= tb) {
          *reinterpret_cast<uint4 *>(gbase + lo16) = *reinterpret_cast<const uint4 *>(stage + lo16);
        } else {
          int b0 = max(lo16, pad), b1 = min(hi16, tb);
          for (int b = b0; b < b1; ++b) gbase[b] = stage[b];
        }
      }
    }
#undef KW
#undef BIT
#undef MSK
#undef VALID
#undef EREL
#undef NBYTES
  }
}

// ------------------------------------------------------------ decoder
__device__ __forceinline__ void bm_set(uint32_t (&bm)[5], int idx) {
#pragma unroll
  for (int q = 0; q < 5; ++q)
    if ((idx >> 5) == q) bm[q] |= 1u << (idx & 31);
}
__device__ __forceinline__ bool bm_test(const uint32_t (&bm)[5], int idx) {
  uint32_t r = 0;
#pragma unroll
  for (int q = 0; q < 5; ++q)
    if ((idx >> 5) == q) r = bm[q];
  return (r >> (idx & 31)) & 1;
}

// record length in bytes of the record whose tag is at pk[q]
__device__ __forceinline__ uint32_t rec_len(const uint8_t *pk, uint32_t q) {
  uint32_t tag = pk[q];
  if (tag == 0) return 2;
  if (tag == 0xffu) return 10 + 8u * pk[q + 9];
  return 1 + __builtin_popcount(tag);
}

// speculative walk from `start`; marks record starts in [cbeg, cend)
__device__ __forceinline__ uint32_t walk(const uint8_t *pk, uint32_t start, uint32_t cbeg,
                                         uint32_t cend, uint32_t (&bm)[5]) {
#pragma unroll
  for (int q = 0; q < 5; ++q) bm[q] = 0;
  uint32_t pos = start;
  while (pos < cend) {
    if (pos >= cbeg) bm_set(bm, (int)(pos - cbeg));
    pos += rec_len(pk, pos);
  }
  return pos;
}

// unaligned 8-byte read from LDS
__device__ __forceinline__ uint64_t lds_read8(const uint8_t *base, uint32_t p) {
  const uint32_t *a = reinterpret_cast<const uint32_t *>(base + (p & ~3u));
  uint32_t d0 = a[0], d1 = a[1], d2 = a[2];
  uint32_t sh = p & 3;
  uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
  uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

__global__ __launch_bounds__(kThreads, 4) void decode_kernel(
    const uint8_t *__restrict__ packed, const uint64_t *__restrict__ in_off,
    const uint64_t *__restrict__ swo, uint32_t n, uint64_t *__restrict__ out,
    int32_t *__restrict__ status, uint32_t *ticket) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem + kDecLut);
  uint16_t *J0 = reinterpret_cast<uint16_t *>(smem + kDecReg);          // [520]
  uint16_t *J1 = reinterpret_cast<uint16_t *>(smem + kDecReg + 1040);   // [520]
  uint8_t *onp = smem + kDecReg + 2080;                                 // [520]
  uint32_t *E = reinterpret_cast<uint32_t *>(smem + kDecReg + 2608);    // [520]
  uint32_t *blk = reinterpret_cast<uint32_t *>(smem + kDecReg);         // [1024]
  int *scr = reinterpret_cast<int *>(smem + kDecScr);
  uint8_t *pkr = smem + kDecPk;

  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  fill_luts(lut, true);

  for (uint32_t it = 0;; ++it) {
    // ticket slot alternates: a wave still reading this piece's slot can
    // never see the next piece's ticket (one barrier per iteration)
    if (tid == 0) scr[64 + (it & 1)] = (int)atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t seg = (uint32_t)scr[64 + (it & 1)];
    if (seg >= n) break;
    const uint64_t w0 = swo[seg];
    const int W = (int)(swo[seg + 1] - w0);
    const uint64_t a = in_off[seg];
    const uint32_t P = (uint32_t)(in_off[seg + 1] - a);
    if (W == 0 || P == 0 || W > kTileWords || P > kDecPkCap) {
      if (tid == 0) {
        int st;
        if (W == 0) st = P == 0 ? CPK_OK : CPK_ETRAILING;      // read() of 0 bytes
        else if (P == 0) st = CPK_ETRUNC;
        else st = CPK_EUNSUPPORTED;
        status[seg] = st;
      }
      continue;
    }
    // ---- stage packed bytes: LDS byte x <-> global (a & ~15) + x ---------
    const uint32_t pad = (uint32_t)(a & 15);
    {
      const uint8_t *g = packed + (a - pad);
      const uint32_t nl = (pad + P + 15) >> 4;
      for (uint32_t c = tid; c < nl; c += kThreads)
        *reinterpret_cast<uint4 *>(pkr + 16 * c) = *reinterpret_cast<const uint4 *>(g + 16 * c);
      if (tid == 0) {  // zero slack after the piece (walks peek up to +9)
        uint32_t z = pad + P;
        for (uint32_t b = z; b < ((z + 15) & ~15u) + 16; ++b) pkr[b] = 0;
      }
    }
    __syncthreads();
    const uint8_t *pk = pkr + pad;

    // ---- tag chain: speculative chunk walks + validation ------------------
    uint32_t C = (P + kMaxChunks - 1) / kMaxChunks;
    C = C < 16 ? 16 : (C + 7) & ~7u;
    const int nch = (int)((P + C - 1) / C);
    const int c = tid;
    const bool active = c < nch;
    const uint32_t cbeg = c * C;
    const uint32_t cend = min(cbeg + C, P);
    uint32_t bm[5] = {0, 0, 0, 0, 0};
    uint32_t X = 0;
    if (active) {
      uint32_t st = c == 0 ? 0 : (cbeg > kWarm ? cbeg - kWarm : 0);
      X = walk(pk, st, cbeg, cend, bm);
    }
    int rounds = 0;
    while ((1 << rounds) < nch + 1) ++rounds;
    bool onpath = false;
    for (int iter = 0;; ++iter) {
      const int t = active ? (X >= P ? nch : (int)(X / C)) : nch;
      if (active) {
        J0[c] = (uint16_t)t;
        onp[c] = c == 0;
      }
      if (tid == 0) {
        J0[nch] = (uint16_t)nch;
        J1[nch] = (uint16_t)nch;
        onp[nch] = 0;
        E[0] = 0;
      }
      __syncthreads();
      uint16_t *Jc = J0, *Jn = J1;
      for (int r = 0; r < rounds; ++r) {
        if (active) {
          int j = Jc[c];
          if (onp[c]) onp[j] = 1;
          Jn[c] = Jc[j];
        }
        __syncthreads();
        uint16_t *tmp = Jc;
        Jc = Jn;
        Jn = tmp;
      }
      onpath = active && onp[c];
      if (onpath && t < nch) E[t] = X;
      __syncthreads();
      bool bad = false;
      if (onpath && c > 0) {
        uint32_t e = E[c];
        if (!bm_test(bm, (int)(e - cbeg))) {
          bad = true;
          X = walk(pk, e, cbeg, cend, bm);
        }
      }
      if (!__syncthreads_or(bad)) break;
      if (iter > 2 * kMaxChunks + 8) break;  // unreachable: converges in <= nch
    }
    // keep only the true records: bits at or after the chunk's entry
    if (!onpath) {
#pragma unroll
      for (int q = 0; q < 5; ++q) bm[q] = 0;
    } else if (c > 0) {
      int e = (int)(E[c] - cbeg);
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        int lo = q * 32;
        if (e >= lo + 32) bm[q] = 0;
        else if (e > lo) bm[q] &= ~0u << (e - lo);
      }
    }
    __syncthreads();  // E/J region is reused as blk below

    // ---- output word offsets of the records --------------------------------
    int myw = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      uint32_t m = bm[q];
      while (m) {
        uint32_t qq = cbeg + 32 * q + __builtin_ctz(m);
        m &= m - 1;
        uint32_t tag = pk[qq];
        myw += (tag == 0) ? 1 + pk[qq + 1] : (tag == 0xffu) ? 1 + pk[qq + 9] : 1;
      }
    }
    int inc = wave_incl_add(myw);
    if (lane == 63) scr[w] = inc;
    if (tid == 0) scr[80] = 0x7fffffff;
    __syncthreads();
    int wb = 0, totw = 0;
    for (int q = 0; q < kWaves; ++q) {
      int tq = scr[q];
      if (q < w) wb += tq;
      totw += tq;
    }
    int o = wb + inc - myw;
    // first error in stream order (PackedInputStream.java:53-138 semantics)
    {
      int err = 0x7fffffff;
      int oo = o;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        uint32_t m = bm[q];
        while (m && err == 0x7fffffff) {
          uint32_t qq = cbeg + 32 * q + __builtin_ctz(m);
          m &= m - 1;
          if (oo >= W) break;
          uint32_t tag = pk[qq];
          int code = 0;
          uint32_t need = 1 + __builtin_popcount(tag);
          int nw = 1;
          uint32_t adv = need;
          if (qq + need > P) code = 2;                     // ETRUNC
          else if (tag == 0) {
            if (qq + 2 > P) code = 2;
            else {
              nw = 1 + pk[qq + 1];
              adv = 2;
              if (oo + nw > W) code = 3;                   // EOVERRUN
            }
          } else if (tag == 0xffu) {
            if (qq + 10 > P) code = 2;
            else {
              uint32_t rn = pk[qq + 9];
              nw = 1 + (int)rn;
              adv = 10 + 8 * rn;
              if (oo + nw > W) code = 3;
              else if (qq + adv > P) code = 2;
            }
          }
          if (!code && oo + nw == W && qq + adv < P) code = 4;  // ETRAILING
          if (code) err = (int)((qq << 3) | code);
          oo += nw;
        }
      }
      if (totw < W && err == 0x7fffffff && c == 0) err = (int)((P << 3) | 2);
      if (err != 0x7fffffff) atomicMin(&scr[80], err);
    }
    __syncthreads();
    const int err = scr[80];
    if (err != 0x7fffffff) {
      if (tid == 0) status[seg] = -(err & 7);
      continue;
    }
    if (totw != W) {  // cannot happen once the checks above pass
      if (tid == 0) status[seg] = CPK_ETRUNC;
      continue;
    }
    // ---- block starts: for every 8-word output block, covering record -----
    {
      int oo = o;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        uint32_t m = bm[q];
        while (m) {
          uint32_t qq = cbeg + 32 * q + __builtin_ctz(m);
          m &= m - 1;
          uint32_t tag = pk[qq];
          int nw = (tag == 0) ? 1 + pk[qq + 1] : (tag == 0xffu) ? 1 + pk[qq + 9] : 1;
          for (int bb = (oo + 7) >> 3; bb * 8 < oo + nw; ++bb)
            blk[bb] = qq | ((uint32_t)(bb * 8 - oo) << 17);
          oo += nw;
        }
      }
    }
    __syncthreads();
    // ---- gather-expand ------------------------------------------------------
    const int nblk = (W + 7) >> 3;
    uint64_t *dst = out + w0;
    for (int b = tid; b < nblk; b += kThreads) {
      uint32_t v = blk[b];
      uint32_t q = v & 0x1ffffu;
      int ofs = (int)(v >> 17);
      uint64_t words[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint32_t tag = pk[q];
        uint64_t x;
        int nw;
        uint32_t adv;
        if (tag == 0) {
          x = 0;
          nw = 1 + pk[q + 1];
          adv = 2;
        } else if (tag == 0xffu) {
          uint32_t rn = pk[q + 9];
          nw = 1 + (int)rn;
          adv = 10 + 8 * rn;
          x = lds_read8(pk, ofs == 0 ? q + 1 : q + 10 + 8 * (uint32_t)(ofs - 1));
        } else {
          uint64_t raw = lds_read8(pk, q + 1);
          uint64_t sel = lut[tag];
          uint32_t lo = (uint32_t)raw, hi = (uint32_t)(raw >> 32);
          uint32_t e0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
          uint32_t e1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
          x = (uint64_t)e0 | ((uint64_t)e1 << 32);
          nw = 1;
          adv = 1 + __builtin_popcount(tag);
        }
        words[i] = x;
        // past the end of the piece: stay on the last record (never stored)
        if (++ofs == nw && b * 8 + i + 1 < W) {
          q += adv;
          ofs = 0;
        }
      }
      const int kw = min(8, W - b * 8);
      uint64_t *d = dst + (uint64_t)b * 8;
      if (kw == 8 && (((uintptr_t)d) & 15) == 0) {
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          uint4 v4;
          v4.x = (uint32_t)words[i];
          v4.y = (uint32_t)(words[i] >> 32);
          v4.z = (uint32_t)words[i + 1];
          v4.w = (uint32_t)(words[i + 1] >> 32);
          *reinterpret_cast<uint4 *>(d + i) = v4;
        }
      } else {
        for (int i = 0; i < kw; ++i) d[i] = words[i];
      }
    }
    if (tid == 0) status[seg] = CPK_OK;
  }
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

}  // namespace cpk

// ================================================================ C ABI
struct cpk_ctx_s {
  int device;
  int cus;
  uint64_t *status;       // look-back words
  uint64_t status_cap;    // entries
  uint32_t *tickets;      // [0] encode, [1] decode  (16 B, memset block)
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
}  // namespace

extern "C" {

int cpk_abi_version(void) { return CPK_ABI_VERSION; }

const char *cpk_status_string(int s) {
  switch (s) {
    case CPK_OK: return "ok";
    case CPK_EINVAL: return "invalid argument / misaligned piece";
    case CPK_ETRUNC: return "premature end of packed input";
    case CPK_EOVERRUN: return "packed run past the end of the piece";
    case CPK_ETRAILING: return "piece filled before the end of its packed bytes";
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
  if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    c->cus = 256;
  if (hipMalloc(&c->tickets, 16) != hipSuccess) {
    free(c);
    return CPK_ENOMEM;
  }
  if (hipFuncSetAttribute((const void *)cpk::encode_kernel<false>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, cpk::kEncLds) != hipSuccess ||
      hipFuncSetAttribute((const void *)cpk::decode_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize, cpk::kDecLds) != hipSuccess) {
    hipFree(c->tickets);
    free(c);
    return CPK_EDEVICE;
  }
  *out = c;
  return CPK_OK;
}

void cpk_ctx_destroy(cpk_ctx ctx) {
  if (!ctx) return;
  DeviceGuard g(ctx->device);
  if (ctx->status) hipFree(ctx->status);
  if (ctx->tickets) hipFree(ctx->tickets);
  free(ctx);
}

int cpk_ctx_device(cpk_ctx ctx) { return ctx ? ctx->device : -1; }

int cpk_encode_batch(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t n,
                     uint64_t max_seg_words, void *d_out, uint64_t *d_out_off, void *stream) {
  if (!ctx || (!d_swo && n) || !d_out_off) return CPK_EINVAL;
  if (max_seg_words == 0 || max_seg_words > (uint64_t)cpk::kTileWords) return CPK_EUNSUPPORTED;
  if (((uintptr_t)d_out & 15) || ((uintptr_t)d_in & 7)) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return hip_ok(hipMemsetAsync(d_out_off, 0, 8, s));
  int rc = ensure_status(ctx, n);
  if (rc) return rc;
  if (hipMemsetAsync(ctx->status, 0, (size_t)n * 8, s) != hipSuccess) return CPK_EDEVICE;
  if (hipMemsetAsync(ctx->tickets, 0, 16, s) != hipSuccess) return CPK_EDEVICE;
  unsigned grid = (unsigned)(2 * ctx->cus);
  if (grid > n) grid = n;
  hipLaunchKernelGGL(cpk::encode_kernel<false>, dim3(grid), dim3(cpk::kThreads), cpk::kEncLds, s,
                     (const uint64_t *)d_in, d_swo, n, (uint8_t *)d_out, d_out_off, ctx->status,
                     ctx->tickets);
  return hip_ok(hipGetLastError());
}

int cpk_decode_batch(cpk_ctx ctx, const void *d_packed, const uint64_t *d_in_off,
                     const uint64_t *d_swo, uint32_t n, void *d_out, int32_t *d_status,
                     void *stream) {
  if (!ctx || (n && (!d_in_off || !d_swo || !d_status))) return CPK_EINVAL;
  if (((uintptr_t)d_packed & 15) || ((uintptr_t)d_out & 7)) return CPK_EINVAL;
  if (n == 0) return CPK_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(ctx->tickets + 1, 0, 4, s) != hipSuccess) return CPK_EDEVICE;
  unsigned grid = (unsigned)(2 * ctx->cus);
  if (grid > n) grid = n;
  hipLaunchKernelGGL(cpk::decode_kernel, dim3(grid), dim3(cpk::kThreads), cpk::kDecLds, s,
                     (const uint8_t *)d_packed, d_in_off, d_swo, n, (uint64_t *)d_out, d_status,
                     ctx->tickets + 1);
  return hip_ok(hipGetLastError());
}

int cpk_encode_host(cpk_ctx ctx, const void *h_in, const uint64_t *h_swo, uint32_t n,
                    void *h_out, uint64_t h_out_cap, uint64_t *h_out_off) {
  if (!ctx || !h_swo || !h_out_off) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  uint64_t words = h_swo[n] - h_swo[0];
  uint64_t maxw = 0;
  for (uint32_t i = 0; i < n; ++i) maxw = h_swo[i + 1] - h_swo[i] > maxw ? h_swo[i + 1] - h_swo[i] : maxw;
  uint64_t cap = cpk_batch_packed_capacity(h_swo, n);
  if (n == 0) {
    h_out_off[0] = 0;
    return CPK_OK;
  }
  if (maxw == 0) {  // only empty pieces: they pack to nothing (SerializePackedTest.java:21)
    for (uint32_t i = 0; i <= n; ++i) h_out_off[i] = 0;
    return CPK_OK;
  }
  void *d_in = nullptr, *d_out = nullptr;
  uint64_t *d_swo = nullptr, *d_off = nullptr;
  int rc = CPK_OK;
  std::vector<uint64_t> rel;
  if (hipMalloc(&d_in, words * 8 + 8) != hipSuccess || hipMalloc(&d_out, cap) != hipSuccess ||
      hipMalloc(&d_swo, (n + 1) * 8ull) != hipSuccess ||
      hipMalloc(&d_off, (n + 1) * 8ull) != hipSuccess) {
    rc = CPK_ENOMEM;
    goto done;
  }
  rel.resize(n + 1);
  for (uint32_t i = 0; i <= n; ++i) rel[i] = h_swo[i] - h_swo[0];
  if (hipMemcpy(d_in, (const uint8_t *)h_in + 8 * h_swo[0], words * 8, hipMemcpyHostToDevice) ||
      hipMemcpy(d_swo, rel.data(), (n + 1) * 8ull, hipMemcpyHostToDevice)) {
    rc = CPK_EDEVICE;
    goto done;
  }
  rc = cpk_encode_batch(ctx, d_in, d_swo, n, maxw, d_out, d_off, nullptr);
  if (rc) goto done;
  if (hipMemcpy(h_out_off, d_off, (n + 1) * 8ull, hipMemcpyDeviceToHost)) {
    rc = CPK_EDEVICE;
    goto done;
  }
  if (h_out_off[n] > h_out_cap) {
    rc = CPK_ENOMEM;
    goto done;
  }
  if (hipMemcpy(h_out, d_out, h_out_off[n], hipMemcpyDeviceToHost)) rc = CPK_EDEVICE;
done:
  if (d_in) hipFree(d_in);
  if (d_out) hipFree(d_out);
  if (d_swo) hipFree(d_swo);
  if (d_off) hipFree(d_off);
  return rc;
}

int cpk_decode_host(cpk_ctx ctx, const void *h_packed, const uint64_t *h_in_off,
                    const uint64_t *h_swo, uint32_t n, void *h_out, int32_t *h_status) {
  if (!ctx || !h_in_off || !h_swo || !h_status) return CPK_EINVAL;
  if (n == 0) return CPK_OK;
  DeviceGuard g(ctx->device);
  uint64_t words = h_swo[n] - h_swo[0];
  uint64_t pbytes = h_in_off[n] - h_in_off[0];
  void *d_pk = nullptr, *d_out = nullptr;
  uint64_t *d_swo = nullptr, *d_io = nullptr;
  int32_t *d_st = nullptr;
  int rc = CPK_OK;
  std::vector<uint64_t> rs, ri;
  if (hipMalloc(&d_pk, pbytes + 32) != hipSuccess || hipMalloc(&d_out, words * 8 + 8) != hipSuccess ||
      hipMalloc(&d_swo, (n + 1) * 8ull) != hipSuccess ||
      hipMalloc(&d_io, (n + 1) * 8ull) != hipSuccess || hipMalloc(&d_st, n * 4ull) != hipSuccess) {
    rc = CPK_ENOMEM;
    goto done;
  }
  rs.resize(n + 1);
  ri.resize(n + 1);
  for (uint32_t i = 0; i <= n; ++i) {
    rs[i] = h_swo[i] - h_swo[0];
    ri[i] = h_in_off[i] - h_in_off[0];
  }
  if (hipMemset(d_pk, 0, pbytes + 32) ||
      (pbytes && hipMemcpy(d_pk, (const uint8_t *)h_packed + h_in_off[0], pbytes, hipMemcpyHostToDevice)) ||
      hipMemcpy(d_swo, rs.data(), (n + 1) * 8ull, hipMemcpyHostToDevice) ||
      hipMemcpy(d_io, ri.data(), (n + 1) * 8ull, hipMemcpyHostToDevice)) {
    rc = CPK_EDEVICE;
    goto done;
  }
  rc = cpk_decode_batch(ctx, d_pk, d_io, d_swo, n, d_out, d_st, nullptr);
  if (rc) goto done;
  if (hipMemcpy(h_status, d_st, n * 4ull, hipMemcpyDeviceToHost) ||
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
