// packed_codec.hip -- MI355X (gfx950, CDNA4) batched codec for Cap'n Proto's
// packed stream encoding, and its C ABI (include/capnp_packed.h).
//
// Reference semantics: runtime/src/main/java/org/capnproto/
//   PackedOutputStream.java:35-205 (encoder), PackedInputStream.java:35-140
//   (decoder).  One "piece" = one write()/read() call; pieces are independent
//   (PackedOutputStream.java:36-43 re-initialises all run state per call).
//
// Design (DESIGN.md has the full derivation and the rooflines):
//   encoders       encode_sp.hip (single pass, the default for like-sized
//                  pieces of 4 Ki words or more and small message batches):
//                  a workgroup per 8192-word chunk, the chunk in VGPRs, roles
//                  by mask algebra, a decoupled look-back for the offsets,
//                  strings (tag + v_perm-compacted bytes + count) OR-ed into
//                  an LDS ring, 16-byte line stores; its sparse form
//                  (cpk_sparse, below: words re-read in B, twice the
//                  workgroups) for batches whose sampled words are >= 85 %
//                  zero; encode_v4.hip (two passes, mixed-size and small-
//                  piece batches): one wave per piece, a size pass, a scan,
//                  an emit pass.  The device chooses (e4_gate_kernel).
//   decoders       decode_kernel: one wave per piece, packed bytes staged in
//                  LDS window by window, the tag chain found by speculative
//                  per-lane walks with pointer-doubling validation, then a
//                  gather-expand of every 4-word output block from its
//                  covering record; decode_v2.hip (sparse batches): a record
//                  index per window instead of the block map;
//                  stream_split.hip: one long stream cut into blocks.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

#include "../../include/capnp_packed.h"
#include <initializer_list>

namespace cpk {

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
// bits of the error word (cpk_ctx_take_error): a piece over its size hint, a
// timed-out cross-workgroup wait, packed bytes past the caller's capacity
constexpr uint32_t kErrHint = 1u, kErrWait = 4u, kErrCap = 8u;
constexpr int kTkGate = 17 * kTkStride + 8;  // [0..1] min, max piece words, [2] encoder choice, [3] sampled zero
                                             // words, [6] single pass's form (1: sparse), [7] sampled words' packed
                                             // bytes, [8..10] decoder choice
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
// a wave-uniform 64-bit value into scalar registers
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}

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

// floor(r / C) for window positions (r < 2^13) by a full-rate 24-bit
// multiply and a shift (the compiler's division by a constant is a
// quarter-rate v_mul_hi_u32 + v_mad_u64_u32 pair, in the landing walk's loop)
template <uint32_t C>
__device__ __forceinline__ uint32_t chunk_div(uint32_t r) {
  constexpr uint32_t kM = ((1u << 20) + C - 1) / C;
  static_assert((kM * C - (1u << 20)) * (1u << 13) < (1u << 20), "exact for r < 2^13");
  return __umul24(r, kM) >> 20;
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

// ------------------------------------------------------------ streaming hints
// nontemporal (streaming) loads and stores: data read or written once
typedef unsigned int cpk_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint64_t ld_stream(const uint64_t *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ uint4 ld_stream16(const uint4 *p) {
  const cpk_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const cpk_u32x4 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_stream(uint4 w, void *p) {
  cpk_u32x4 v = {w.x, w.y, w.z, w.w};
  __builtin_nontemporal_store(v, reinterpret_cast<cpk_u32x4 *>(p));
}

// ------------------------------------------------------------ look-back
// One 8-byte relaxed agent-scope granule per status word: the data is the
// flag (cdna_hip_programming.md Guideline 16, form R2); the single-pass
// encoder's words (encode_sp.hip: sp_word) carry flag, epoch and value.
__device__ __forceinline__ void st_status(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_status(uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
//      records to check the reference's error conditions and mark, per
//      record, the 4-word output block its first word falls in (ds_max);
//      a prefix max hands every block its covering record; all 64 lanes then
//      gather-expand the blocks (PackedInputStream.java:82-134 per word).
// No barriers: up to 28 pieces in flight per CU.
constexpr int kDecThreads = 256;               // 4 independent waves
// workgroups per CU the register budget is sized for (= the LDS limit:
// 72 VGPRs; at 8 the stream form spilled, messages decode +10 %)
#ifndef CPK_DEC_WPE
#define CPK_DEC_WPE 7
#endif
constexpr int kDecWpe = CPK_DEC_WPE;
// Lane chunks C of 56 bytes (3.5 KiB windows, 7 workgroups per CU by LDS):
// measured against 40 / 48 / 60 / 64 at 131,072 pieces with the max-map
// block map, 56 is fastest on configs 2-4 (against 48: 4.29 -> 4.13 ms,
// 6.80 -> 6.51, 2.84 -> 2.80)
constexpr uint32_t kDecChunk = 56;
constexpr uint32_t kWin = 64 * kDecChunk;         // packed bytes resolved per window
// bytes loaded past the window (a literal run reaching past them is read from memory;
// 240: config 3 decode -4.5 % against 32, config 2 neutral; 368 costs occupancy)
constexpr uint32_t kDecLook = 240;
constexpr uint32_t kWinBuf = (kWin + 15 + kDecLook + 16 + 15) & ~15u;  // + pad, look-ahead, slack
// (8 workgroups per CU with 48-byte chunks; larger rounds cost occupancy)
#ifndef CPK_DEC_ROUND
#define CPK_DEC_ROUND 1280
#endif
constexpr int kRound = CPK_DEC_ROUND;  // output words expanded per round
// (4: 64 lanes cover a window's blocks in fewer, fuller passes; measured faster than 8)
#ifndef CPK_DEC_BLK
#define CPK_DEC_BLK 4
#endif
constexpr int kBlk = CPK_DEC_BLK;  // output words per expansion block
// a lane's visited positions: one bit per chunk byte (bit q mod 64 for
// position q: the walks index it by the position itself, so it is 64 bits
// whatever the chunk size)
typedef uint64_t VisMask;
static_assert(sizeof(VisMask) == 8, "visited bits are set at position mod 64");
static_assert(kDecChunk <= 64, "visited mask bits");
// the visited masks (phases 1-3) and the block map (phase 5) share LDS
constexpr uint32_t kDecWaveLds = kWinBuf + (4 * (kRound / kBlk) > 64 * sizeof(VisMask)
                                                ? 4 * (kRound / kBlk)
                                                : 64 * sizeof(VisMask));
// The block map: a record marks only the block whose span ends at or after
// its first word (ds_max of an entry ordered by output position), and a
// prefix max over the blocks hands every block the last record starting at
// or before its first word: one LDS op per record, no per-block loop
constexpr int kMapPer = kRound / kBlk / 64;  // map entries per lane in the fill
static_assert((kRound / kBlk == 64 * kMapPer && kWin <= 4096 && kRound + 256 < (1 << 19)),
              "max-map entry: 12-bit window position, 19-bit output position");
constexpr uint32_t kDecChkReach = (kWin + 2064);
// Dense windows (few, long records: 0xFF runs) are walked by one lane
// (decode_body<.., kSerial>, the form picked for dense batches): taken when
// the previous window looked dense (over 5.3 packed bytes per word); a serial
// walk passing kDecSerMax records gives the window back to the parallel
// walks, which then keep the next kDecSerCool windows.
#ifndef CPK_DEC_SER_MAX
#define CPK_DEC_SER_MAX 128
#endif
constexpr uint32_t kDecSerMax = CPK_DEC_SER_MAX, kDecSerCool = 32;
static_assert(kDecChkReach >= kWin + 2050, "a window's last record must fall inside the checked reach");
constexpr int kWinLinesPerLane = (int)((kWin + 15 + kDecLook + 15) / 16 + 63) / 64;
// LUT | 4 waves' windows and block maps | 4 waves' dense-form counters
constexpr uint32_t kDecCntOff = 2048 + 4 * kDecWaveLds;
// The dense form's window counters (cpk_ctx_dense_windows): compiled into
// the diagnostics build only (libcapnp_packed_hip_diag.so, build_native.py).
// Any code in the serial path changes the dense forms' register allocation
// (spills): with the counters, config-3 message decode +2 % (round 6,
// profiles/r6f_*).
#ifndef CPK_DEC_CNT
#define CPK_DEC_CNT 0
#endif
constexpr bool kDecCnt = CPK_DEC_CNT != 0;
constexpr uint32_t kDecLds = kDecCntOff + 32;  // 22,624 at 56-byte chunks

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

// The tag at piece position q and both possible count bytes (c1 after a
// 0x00 tag, c9 after 0xFF), read together: one LDS round trip per record on
// the walks.  (Round 5: reading a count byte only for the tags that have one
// cut the decoder's LDS cycles 22 % and made it 6 % slower -- the dependent
// second read and its exec-mask branches, docs/tuning_log.md.)
template <bool k32 = true>
__device__ __forceinline__ void rec_bytes(const uint8_t *pkw, uint32_t q, uint32_t &tag, uint32_t &c1, uint32_t &c9) {
  tag = pkw[q];
  c1 = pkw[q + 1];
  c9 = pkw[q + 9];
  // k32: the tag kept a 32-bit value (hipcc otherwise narrows it to 16-bit
  // ops: a mask and a separate +1 around every popcount; round 5: config 2
  // decode -1.0 %, the stream forms +5 %: not there)
  if constexpr (k32) asm("" : "+v"(tag));
}

// The record whose tag is at piece position q: its byte length and output
// words (PackedInputStream.java:82-134).
struct DecRec {
  uint32_t len, nw;
};
template <bool k32 = true>
__device__ __forceinline__ DecRec rec_at(const uint8_t *pkw, uint32_t q) {
  uint32_t tag, c1, c9;
  rec_bytes<k32>(pkw, q, tag, c1, c9);
  // masks, not nested selects (hipcc turns those into exec-mask branches)
  const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
  DecRec r;
  r.len = 1u + __builtin_popcount(tag) + (zm & 1u) + (fm & (8u * c9 + 1u));
  r.nw = 1u + (zm & c1) + (fm & c9);
  return r;
}

// 8 bytes at piece position x: from the LDS window when loaded, otherwise
// (tail of a literal run reaching past the window) straight from memory
// (kAllIn: the caller knows x + 12 <= lend -- every record of the window
// lies in the loaded bytes -- so no check and no memory path)
template <bool kAllIn = false, bool kLa = true>
__device__ __forceinline__ uint64_t read8(const uint8_t *pkw, uint32_t x, uint32_t lend,
                                         const uint8_t *gpiece, uint32_t glim, uint32_t ph,
                                         uint32_t e) {
  // The LDS read is unconditional (position clamped to the window start e,
  // which has 12 buffer bytes after it whatever the window's size): with
  // both reads under one branch hipcc merged them into flat loads.
  // LDS-aligned dwords: piece position x sits at byte phase (x + ph) & 3 of
  // the 16-byte aligned window buffer.
  const bool inw = kAllIn || x + 12 <= lend;
  const uint32_t xl = inw ? x : e;
  uint32_t sh, d0, d1, d2;
  if constexpr (kLa) {
    // from the LDS byte address itself: its low bits are the phase, its
    // aligned part the first dword (add, and, and; round 5: config-3
    // messages decode -1.2 %, the dense piece form +1.8 %: not there)
    typedef __attribute__((address_space(3))) const uint8_t lds_cu8;
    typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
    const uint32_t la = (uint32_t)(uintptr_t)((lds_cu8 *)pkw) + xl;
    sh = la & 3;
    lds_cu32 *pl = (lds_cu32 *)(uintptr_t)(la & ~3u);
    d0 = pl[0], d1 = pl[1], d2 = pl[2];
  } else {
    sh = (xl + ph) & 3;
    const uint32_t *pl = reinterpret_cast<const uint32_t *>(pkw + ((int64_t)xl - sh));  // (signed: xl < sh)
    d0 = pl[0], d1 = pl[1], d2 = pl[2];
  }
  if (!kAllIn && !inw) {
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

// (stats build: the window phases' clock sums live in the caller)
#ifdef CPK_PHASE_STATS
#define DEC_PH_PARAMS , unsigned long long &wph_last, unsigned long long *wph_acc
#define DEC_PH_ARGS , wph_last, wph_acc
#else
#define DEC_PH_PARAMS
#define DEC_PH_ARGS
#endif
// ---- 1-3 of a window [e, wend) (decode_body; decode_piece_mw): lane l
// walks its chunk [cb, cb + kDecChunk) from cb as if a tag stood there (the
// visited positions into visa[l], its words wt, its exit X), then on until it
// lands on a position some lane visited -- from there the two walks coincide,
// the chain being a function of the position -- (S, its words lw); R: the
// lanes reachable from l under "lane -> owner of its landing point" (always a
// later lane), by pointer doubling (6 rounds cover a chain of 64).  Nothing
// here depends on where the window's true records start.
struct WinWalk {
  uint32_t cb, S, wt, lw;
  uint64_t R;
};
template <bool k32 = true>
__device__ __forceinline__ WinWalk win_walks(const uint8_t *pkw, VisMask *visa, int lane, uint32_t e,
                                             uint32_t wend DEC_PH_PARAMS) {
  // ---- 1: speculative chunk walks --------------------------------------
  const uint32_t cb = e + kDecChunk * lane;
  const uint32_t ce = min(cb + kDecChunk, wend);
  VisMask vis = 0;
  uint32_t X = cb, wt = 0;  // wt: output words of the walk
  if (cb < wend) {
    uint32_t pos = cb;
    while (pos < ce) {
      // (the bit of piece position pos mod 64 -- a rotation of the chunk
      // offsets, distinct for a 56-byte chunk: the shift takes pos itself,
      // no subtraction per record; round 5: config 2 decode -0.5 %)
      vis |= (VisMask)1 << (pos & 63u);
      const DecRec r = rec_at<k32>(pkw, pos);
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
      const uint32_t ow_ = chunk_div<kDecChunk>(r);
      if ((visa[ow_] >> (S & 63u)) & 1) break;  // (bit S mod 64, as above)
      const DecRec rr = rec_at<k32>(pkw, S);
      lw += rr.nw;
      S += rr.len;
    }
  }
  WPH(2)
  // ---- 3: reachability over lanes --------------------------------------
  int nx = (cb < wend && S < wend) ? (int)chunk_div<kDecChunk>(S - e) : 64;
  uint64_t R = 1ull << lane;
  {
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
  }
  WinWalk ww;
  ww.cb = cb;
  ww.S = S;
  ww.wt = wt;
  ww.lw = lw;
  ww.R = R;
  return ww;
}

// ---- 5: error checks, block map, expansion (rounds of kRound words) of a
// window whose true records are known: an on-path lane holds the records
// [entry, S), the first at window word o0 (myw words); T words in all, the
// window's first record at piece position e, ow piece words before it
// (decode_body; decode_piece_mw).  Returns false when a record fails (st
// set); fin: the end of the record that fills the piece, else 0.
template <bool kStream, bool kLean = true>
__device__ __forceinline__ bool win_emit(const uint8_t *pkw, const uint64_t *lut, uint32_t *blk, int lane,
                                         uint32_t e, int ow, int W, uint32_t P, int T, bool on,
                                         uint32_t entry, uint32_t S, uint64_t onmask, int o0, int myw,
                                         uint32_t enext, uint32_t lend, const uint8_t *gp, uint32_t glim,
                                         uint32_t ph, uint64_t *dst, int &st, uint32_t &fin,
                                         bool premapped DEC_PH_PARAMS) {
  bool failed = false;
  fin = 0;
  // errors and the filling record can only occur in a window reaching the
  // piece's last word or within one window plus one record of its end
  // (the window's records start before e + kWin; the longest record, a
  // 0xFF tag with its word, count and 255 words, is 2,050 bytes)
  const bool chk = (ow + T >= W) || (P - e < kDecChkReach);
  for (int rb = 0; rb < T; rb += kRound) {
    int err = 0x7fffffff;
    // (premapped: the serial walk filled round 0's map, decode_body)
    if (!(premapped && rb == 0)) {
    wave_lds_order();  // (the visited masks / last round's map reads are done)
#pragma unroll
    for (int i = 0; i < kMapPer; ++i) blk[lane * kMapPer + i] = 0u;
    wave_lds_order();
    // after the first round only the lanes whose output meets this round
    if (!(chk && rb == 0)) {
      // no record here can fail or fill the piece: the map alone
      if (rb == 0) {
        // round 0 (usually the window's only one): every record's output
        // is at or past the round's start, so it always marks a block
        if (on) {
          uint32_t ro = (uint32_t)o0;
          for (uint32_t q = entry; q < S && ro <= (uint32_t)(kRound - kBlk);) {
            uint32_t tag, c1, c9;
            rec_bytes<!kStream>(pkw, q, tag, c1, c9);
            const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
            atomicMax(&blk[(ro + kBlk - 1) / kBlk], ((ro + 256u) << 12) | (q - e));
            ro += 1u + (zm & c1) + (fm & c9);
            q += 1 + __builtin_popcount(tag) + (zm & 1u) + (fm & (8u * c9 + 1u));
          }
        }
      } else
      if (on && (rb == 0 || (o0 < rb + kRound && o0 + myw > rb))) {
        int ro = o0 - rb;  // round-relative output of the record (> -256 when live)
        // (records past the round's last block start mark nothing, nor
        // do the ones after them)
        for (uint32_t q = entry; q < S && ro <= kRound - kBlk;) {
          uint32_t tag, c1, c9;
          rec_bytes<!kStream>(pkw, q, tag, c1, c9);
          const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
          const int nw = 1 + (int)((zm & c1) + (fm & c9));
          if (ro + nw > 0)
            atomicMax(&blk[(max(ro, 0) + kBlk - 1) / kBlk], ((uint32_t)(ro + 256) << 12) | (q - e));
          ro += nw;
          q += 1 + __builtin_popcount(tag) + (zm & 1u) + (fm & (8u * c9 + 1u));
        }
      }
    } else
    {
      // round 0 of a window near the piece's end.  Only two records can
      // fail or fill the piece: the one whose words reach word W (when the
      // window gets there; the reference stops reading after it), else the
      // window's last record (the only one whose bytes can pass P: every
      // other record ends where the next begins, before wend <= P).  The
      // map walk notes them; one lane then runs the reference's checks
      // on its record (PackedInputStream.java:53-138).
      uint32_t qc = 0xffffffffu;
      int oc = 0;
      if (on) {
        const int wr = W - ow;  // words left in the piece (> 0)
        uint32_t ql = entry;
        int o = o0, ol = o0;
        for (uint32_t q = entry; q < S;) {
          const uint32_t tag = pkw[q], c1 = pkw[q + 1], c9 = pkw[q + 9];
          const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
          const int nw = 1 + (int)((zm & c1) + (fm & c9));
          const int idx = (o + kBlk - 1) / kBlk;  // (round 0: o >= 0)
          if (idx < kRound / kBlk) atomicMax(&blk[idx], ((uint32_t)(o + 256) << 12) | (q - e));
          if (o < wr && o + nw >= wr) {
            qc = q;
            oc = o;
          }
          ql = q;
          ol = o;
          o += nw;
          q += 1 + __builtin_popcount(tag) + (zm & 1u) + (fm & (8u * c9 + 1u));
        }
        if (ow + T < W && lane == 63 - __builtin_clzll(onmask)) {
          qc = ql;
          oc = ol;
        }
      }
      if (qc != 0xffffffffu) {
        const uint32_t q = qc;
        const uint32_t tag = pkw[q], c1 = pkw[q + 1], c9 = pkw[q + 9];
        const uint32_t ntag = 1 + __builtin_popcount(tag);
        const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
        const int nw = 1 + (int)((zm & c1) + (fm & c9));
        const uint32_t adv = ntag + (zm & 1u) + (fm & (8u * c9 + 1u));
        const int oo = ow + oc;
        // truncated tag bytes / count / literal run -> EOF DecodeException;
        // run past the piece -> DecodeException / BufferOverflowException
        int code = 0;
        if (q + ntag > P) code = 2;
        else if (tag == 0 || tag == 0xffu) {
          if (q + (tag ? 10u : 2u) > P) code = 2;
          else if (oo + nw > W) code = 3;
          else if (q + adv > P) code = 2;
        }
        if (!kStream && !code && oo + nw == W && q + adv < P) code = 4;
        if (code) err = (int)(((q - e) << 3) | (uint32_t)code);
        if (oo + nw == W) fin = q + adv;
      }
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
    {
      // prefix max: lane l holds blocks [kMapPer * l, kMapPer * (l + 1))
      uint32_t m[kMapPer];
      int run = 0;
#pragma unroll
      for (int i = 0; i < kMapPer; ++i) {
        run = max(run, (int)blk[lane * kMapPer + i]);
        m[i] = (uint32_t)run;
      }
      const uint32_t pre = (uint32_t)wave_shr1(wave_incl_max(run), 0);
#pragma unroll
      for (int i = 0; i < kMapPer; ++i) blk[lane * kMapPer + i] = max(m[i], pre);
    }
    wave_lds_order();
    WPH(5)
    const int nb = (min(min(kRound, T - rb), W - ow - rb) + kBlk - 1) / kBlk;
    // two copies of the expansion: one for windows whose records all lie
    // in the loaded bytes (enext + 12 <= lend: the usual case), whose
    // reads need no bound check and no memory path
    auto expand = [&](auto allin) __attribute__((always_inline)) {
    constexpr bool kAllIn = decltype(allin)::value;
    for (int b = lane; b < nb; b += 64) {
      const uint32_t v = blk[b];
      uint32_t q = e + (v & 0xfffu);
      int ofs = kBlk * b + 256 - (int)(v >> 12);
      const int wbase = ow + rb + kBlk * b;  // piece word of the block's first word
      const int wleft = ow + T - wbase - 1;   // words of the window after the block's first
      uint64_t words[kBlk];
      // (the record's tag and count bytes are read once per record, not per
      // word: a literal run's words then need only their own reads, all in
      // flight together)
      uint32_t tag, c1, c9;
      rec_bytes<!kStream>(pkw, q, tag, c1, c9);
      if constexpr (!kStream) {
      // one path for every tag: a zero run's word reads its (unused) bytes
      // and lut[0] selects none; lut[0xff] is the identity for a literal
      // run's words (no divergent branches per word)
      uint64_t sel = lut[tag];
#pragma unroll
      for (int i = 0; i < kBlk; ++i) {
        // PackedInputStream.java:84-134 per word: zero run, 0xFF literal
        // run (tag word, then the counted words), or a tagged word
        const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
        const int nw = 1 + (int)((zm & c1) + (fm & c9));
        const uint32_t rp = (fm && ofs) ? q + 2 + 8u * (uint32_t)ofs : q + 1;
        const uint64_t raw = read8<kAllIn, kLean>(pkw, rp, lend, gp, glim, ph, e);
        const uint32_t rl = (uint32_t)raw, rh = (uint32_t)(raw >> 32);
        const uint32_t x0 = __builtin_amdgcn_perm(rh, rl, (uint32_t)sel);
        const uint32_t x1 = __builtin_amdgcn_perm(rh, rl, (uint32_t)(sel >> 32));
        words[i] = (uint64_t)x0 | ((uint64_t)x1 << 32);
        // past the window's last word: stay put (never stored)
        if (++ofs == nw && i < wleft) {
          q += 1 + __builtin_popcount(tag) + (zm & 1u) + (fm & (8u * c9 + 1u));
          ofs = 0;
          if (i + 1 < kBlk) {
            rec_bytes<!kStream>(pkw, q, tag, c1, c9);
            sel = lut[tag];
          }
        }
      }
      } else {
      // (the stream form keeps the branches: its register budget is tighter,
      // and the one-path form measured 3 % slower there, docs/tuning_log.md r5W)
#pragma unroll
      for (int i = 0; i < kBlk; ++i) {
        // PackedInputStream.java:84-134 per word: zero run, 0xFF literal
        // run (tag word, then the counted words), or a tagged word
        // (the count bytes are read with the tag: one LDS round trip)
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
          x = read8<kAllIn, kLean>(pkw, ofs == 0 ? q + 1 : q + 10 + 8 * (uint32_t)(ofs - 1), lend, gp, glim, ph, e);
        } else {
          const uint64_t raw = read8<kAllIn, kLean>(pkw, q + 1, lend, gp, glim, ph, e);
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
        if (++ofs == nw && i < wleft) {
          q += adv;
          ofs = 0;
          if (i + 1 < kBlk) rec_bytes<!kStream>(pkw, q, tag, c1, c9);
        }
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
          st_stream(v4, d + i);  // (nontemporal: plain stores cut writes 3 % and cost 1.8 % time)
        }
      }
      else if (kLean && kw == kBlk && kBlk == 4) {
        // a full block at an odd word: word 0, words 1-2 as one 16-byte
        // store, word 3 (no per-word branches; round 5: config 2 decode
        // -0.6 %, the dense piece form +2.2 %: not there)
        d[0] = words[0];  // (plain: nontemporal 8-byte stores left partial lines, +6 % HBM writes)
        uint4 v4;
        v4.x = (uint32_t)words[1];
        v4.y = (uint32_t)(words[1] >> 32);
        v4.z = (uint32_t)words[2];
        v4.w = (uint32_t)(words[2] >> 32);
        st_stream(v4, d + 1);
        d[kBlk - 1] = words[kBlk - 1];
      } else {
#pragma unroll
        for (int i = 0; i < kBlk; ++i)
          if (i < kw) d[i] = words[i];
      }
    }
    };
    if (enext + 12 <= lend) expand(std::true_type{});
    else
      expand(std::false_type{});
    wave_lds_order();  // blk reused by the next round
    WPH(6)
  }
  return !failed;
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
  const uint32_t *skip;   // (batch form: nonzero = the other decoder took the batch)
  const uint32_t *order;  // (stream form: ticket -> stream, largest first; null: in order)
};
template <bool kStream, bool kSerial = false>
__device__ __forceinline__ void decode_body(uint8_t *smem, const uint8_t *__restrict__ packed,
                                            uint64_t *__restrict__ in_off, const uint64_t *__restrict__ swo,
                                            uint32_t n, uint64_t *__restrict__ out, int32_t *__restrict__ status,
                                            uint32_t *ticket, uint64_t avail, DecStreams sd) {
  // the expansion's lean forms (reads from LDS byte addresses, read8; odd
  // blocks' stores without branches), but in the dense piece form, where
  // they measured slower
  constexpr bool kDecLean = kStream || !kSerial;
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem);
  const int lane = lane_id(), w = wave_id();
  uint8_t *wl = smem + 2048 + w * kDecWaveLds;
  uint8_t *wbuf = wl;                                            // window bytes
  uint32_t *blk = reinterpret_cast<uint32_t *>(wl + kWinBuf);    // [256]
  VisMask *visa = reinterpret_cast<VisMask *>(blk);  // [64], over the block map
  if (sd.skip && __builtin_amdgcn_readfirstlane(*sd.skip)) return;
  fill_luts(lut, true);
  if (kSerial && kDecCnt && threadIdx.x == 0)  // (the dense form's counters, below)
    reinterpret_cast<uint64_t *>(smem + kDecCntOff)[0] = 0ull;
  __syncthreads();  // the only block-wide barrier: LUT ready
  // (one stream: its one ticket is item 0 of counter 0 -- start there, and
  // a wave that does not get it leaves at once instead of trying the other
  // seven counters one dependent atomic after another)
  int xq = (kStream && sd.ns == 1) ? 0 : xcc_id(), dry = 0;
  WPH_INIT
  uint64_t scur = 0;      // stream mode: start of the next piece
  uint64_t slim = avail;  //   end of the stream's bytes
  int sfail = CPK_OK;     //   a failed piece stops the stream
  uint32_t snext = 0, sende = 0, sj = 0;  // next piece, end of the stream's pieces, stream
  bool ser = false;   // the next window is walked by one lane (the last one looked dense)
  uint32_t cool = 0;  // windows before the next serial attempt after one gave up
  int tprev = 0;      // the last window's words (a window near the piece's end stays parallel:
                      // in a stream the bytes do not say where the piece ends)
  // (dense form: windows walked serially / serial walks given back, counted
  // per workgroup at a fixed LDS address -- anything live across the window
  // loop costs the dense forms spills -- and added to ticket[1] / [2] at the
  // end: cpk_ctx_dense_windows)
  uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + kDecCntOff);

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
          if (j < sd.ns || ++dry >= 8 || sd.ns == 1) break;
          xq = (xq + 1) & 7;
        }
        if (j >= sd.ns) {
          more = false;
          break;
        }
        // (the stream's values are wave-uniform: kept in scalar registers,
        // which leaves the stream form's VGPRs to the windows)
        if (sd.order) j = (uint32_t)__builtin_amdgcn_readfirstlane((int)sd.order[j]);
        sj = j;
        snext = sd.sbeg ? (uint32_t)__builtin_amdgcn_readfirstlane((int)sd.spc[j]) : 0u;
        sende = sd.sbeg ? (uint32_t)__builtin_amdgcn_readfirstlane((int)sd.spc[j + 1]) : n;
        scur = sd.sbeg ? rfl64(sd.sbeg[j]) : 0;
        slim = sd.sbeg ? rfl64(sd.send[j]) : avail;
        sfail = CPK_OK;
        if (snext >= sende) sd.send_out[j] = scur;
      }
      if (!more) break;
      seg = snext++;
    }
    if (seg >= n) break;
    const uint64_t w0 = rfl64(swo[seg]);
    const int W = __builtin_amdgcn_readfirstlane((int)(swo[seg + 1] - w0));
    const uint64_t a = rfl64(kStream ? scur : in_off[seg]);
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
      // the window's start and the words so far are wave-uniform: say so
      // (the loop's exits made the compiler keep them in VGPRs and run the
      // window's uniform branches under exec masks)
      e = (uint32_t)__builtin_amdgcn_readfirstlane((int)e);
      ow = __builtin_amdgcn_readfirstlane(ow);
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
      const uint32_t need = min(e + kWin + kDecLook, P) - ebase;  // <= kWin + kDecLook + 15 bytes
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
      if constexpr (kSerial) {
        // ---- a dense window: its true records walked by one lane -----------
        // In a window of few, long records (the 0xFF runs of dense data) the
        // 64 speculative chunk walks mostly walk verbatim run bytes, and the
        // chain, count and map walks follow; one lane walking the true chain
        // from e visits only the ~30 true records
        // (PackedInputStream.java:82-134) and fills round 0's block map in
        // order with plain stores (a later record marking the same block is
        // the larger entry, as ds_max keeps it).  Only for windows that can
        // neither fail nor fill the piece and whose words fit one round: a
        // walk that meets the piece's last word, the round's end or
        // kDecSerMax records gives the window to the parallel path.  (The
        // decode_kernel<.., true> form, picked for dense batches: its extra
        // state costs the parallel path ~2 % on config-2 data.)
        if (ser && P - e >= kDecChkReach && W - ow > 2 * tprev) {
          wave_lds_order();
#pragma unroll
          for (int i = 0; i < kMapPer; ++i) blk[lane * kMapPer + i] = 0u;
          wave_lds_order();
          uint32_t q = e, nrec = 0;
          int o = 0, ok = 1;
          if (lane == 0) {
            const int wr = W - ow;  // words left in the piece
            while (q < wend) {
              const DecRec r = rec_at<!kStream>(pkw, q);
              if (o + (int)r.nw >= wr || o + (int)r.nw > kRound || ++nrec > kDecSerMax) {
                ok = 0;
                break;
              }
              if (o <= kRound - kBlk) blk[(o + kBlk - 1) / kBlk] = ((uint32_t)(o + 256) << 12) | (q - e);
              o += (int)r.nw;
              q += r.len;
            }
          }
          if (readlane(ok, 0)) {
            const int T = readlane(o, 0);
            const uint32_t enext = (uint32_t)readlane((int)q, 0);
            uint32_t fin = 0;
            const bool failed = !win_emit<kStream, kDecLean>(pkw, lut, blk, lane, e, ow, W, P, T, false, e, e, 0ull, 0,
                                                   0, enext, lend, gp, glim, ph, dst, st, fin, true DEC_PH_ARGS);
            if (failed) break;  // (cannot happen: no record here is checked)
            ow += T;
            e = enext;
            tprev = T;
            if (kDecCnt && lane == 0) atomicAdd(&cnt[0], 1u);
            continue;
          }
          // too many records (dense but tagged words, e.g. one zero byte per
          // word): the parallel path, and no serial walk for a while
          ser = false;
          cool = kDecSerCool;
          if (kDecCnt && lane == 0) atomicAdd(&cnt[1], 1u);
        }
      }

      WPH(1)
      // ---- 1-3: speculative walks, chain reachability ------------------------
      const WinWalk ww = win_walks<!kStream>(pkw, visa, lane, e, wend DEC_PH_ARGS);
      const uint32_t cb = ww.cb, wt = ww.wt, lw = ww.lw, S = ww.S;
      const uint64_t R = ww.R;
      const uint64_t onmask = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)R, 0)) |
                              ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(R >> 32), 0) << 32);
      const uint32_t enext =
          (uint32_t)__builtin_amdgcn_readlane((int)S, 63 - __builtin_clzll(onmask));
      // each on-path lane hands its landing point to its successor
      wave_lds_order();  // (phase 2's reads of visa are done)
      if (((onmask >> lane) & 1) && S < wend) visa[chunk_div<kDecChunk>(S - e)] = (VisMask)S;
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
          const DecRec r = rec_at<!kStream>(pkw, q);
          pre += r.nw;
          q += r.len;
        }
        myw = (int)(wt - pre + lw);
      }
      const int inc = wave_incl_add(myw);
      const int T = readlane(inc, 63);
      const int o0 = inc - myw;  // window-relative output of this lane's first record
      WPH(4)
      // ---- 5: error checks, block map, expansion ------------------------------
      uint32_t fin = 0;  // end of the record that fills the piece (if any)
      const bool failed = !win_emit<kStream, kDecLean>(pkw, lut, blk, lane, e, ow, W, P, T, on, entry, S, onmask, o0, myw,
                                             enext, lend, gp, glim, ph, dst, st, fin, false DEC_PH_ARGS);
      if (failed) break;
      if (ow + T >= W && fin) {  // the piece is full: next piece starts at fin
        ow = W;
        e = fin;
        break;
      }
      if constexpr (kSerial) {
        // dense data: ~8 packed bytes per word (0xFF runs); config-2-like
        // windows take ~3.8 (their ~550 records would be a long serial walk)
        // (wave-uniform values: kept in scalar registers)
        if (cool) --cool;
        else ser = __builtin_amdgcn_readfirstlane((int)(16u * (uint32_t)T < 3u * (enext - e))) != 0;
        tprev = __builtin_amdgcn_readfirstlane(T);
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
  if constexpr (kSerial && kDecCnt) {
    // (each wave hands on what the workgroup has counted so far, its own
    // counts included: every count is taken by its own wave's exchange)
    if (lane == 0) {
      const uint32_t a = atomicExch(&cnt[0], 0u), b = atomicExch(&cnt[1], 0u);
      if (a) atomicAdd(&ticket[1], a);
      if (b) atomicAdd(&ticket[2], b);
    }
  }
  WPH_FLUSH(16)
}
template <bool kStream, bool kSerial = false>
__global__ __launch_bounds__(kDecThreads, kDecWpe) void decode_kernel(
    const uint8_t *__restrict__ packed, uint64_t *__restrict__ in_off,
    const uint64_t *__restrict__ swo, uint32_t n, uint64_t *__restrict__ out,
    int32_t *__restrict__ status, uint32_t *ticket, uint64_t avail, DecStreams sd) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  decode_body<kStream, kSerial>(smem, packed, in_off, swo, n, out, status, ticket, avail, sd);
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
struct NoWords {
  __device__ void operator()(uint32_t, uint64_t) const {}
};
// (word(i, w): the table's words as read, i = 0 the first)
template <class F, class G = NoWords>
__device__ int read_table(const uint8_t *p, uint64_t n, uint64_t limit, uint64_t &ip,
                          uint32_t &count, uint64_t &total, F emit, G word = G()) {
  uint64_t first = 0;
  int st = serial_read(p, n, ip, 1, [&](uint32_t, uint64_t w) {
    first = w;
    word(0u, w);
  });
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
      word(1u + i, w);
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

// ---- stream tickets, largest first --------------------------------------
// A wave decodes a message's stream whole, so a large message taken last
// leaves the other waves idle while it finishes (config 3: 1 MiB messages
// among 16 KiB ones; taken largest first the decode is 3.8 % shorter).  A
// counting sort by the bit length of the word count: order[t] = the t-th
// message to take, larger classes first (within a class in any order -- the
// output does not depend on it).  (The two-pass encoder's segments taken
// the same way: 51.3 -> 57.0 ms on config 3 -- the passes stream the words
// in memory order, and lose that locality.)
constexpr int kOrdClasses = 64;
__device__ __forceinline__ uint32_t ord_class(uint64_t w) {
  return (uint32_t)(kOrdClasses - 1) - (w ? 64u - (uint32_t)__builtin_clzll(w) : 0u);
}
// (item i's words: words[i], or swo[i + 1] - swo[i] when swo is given)
__device__ __forceinline__ uint64_t ord_words(const uint64_t *words, const uint64_t *swo, uint32_t i) {
  return swo ? swo[i + 1] - swo[i] : words[i];
}
__global__ void ord_hist_kernel(const uint64_t *__restrict__ words, uint32_t n, uint32_t *hist,
                                const uint64_t *__restrict__ swo) {
  __shared__ uint32_t h[kOrdClasses];
  if (threadIdx.x < kOrdClasses) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&h[ord_class(ord_words(words, swo, i))], 1u);
  __syncthreads();
  if (threadIdx.x < kOrdClasses && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
__global__ void ord_scan_kernel(uint32_t *hist) {
  if (threadIdx.x != 0) return;
  uint32_t run = 0;
  for (int c = 0; c < kOrdClasses; ++c) {
    const uint32_t k = hist[c];
    hist[c] = run;
    run += k;
  }
}
// (a block reserves its range in each class with one global atomic: with a
// few classes and 256 Ki messages, one atomic per message took 1.5 ms)
__global__ void ord_scatter_kernel(const uint64_t *__restrict__ words, uint32_t n, uint32_t *cursor,
                                   uint32_t *__restrict__ order, const uint64_t *__restrict__ swo) {
  __shared__ uint32_t cnt[kOrdClasses], base[kOrdClasses];
  if (threadIdx.x < kOrdClasses) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = i < n ? ord_class(ord_words(words, swo, i)) : 0u;
  const uint32_t r = i < n ? atomicAdd(&cnt[c], 1u) : 0u;
  __syncthreads();
  if (threadIdx.x < kOrdClasses && cnt[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], cnt[threadIdx.x]);
  __syncthreads();
  if (i < n) order[base[c] + r] = i;
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

// The one-launch small paths' completion flag: once every wave's writes
// (pinned host memory included) are complete at system scope, seq goes to
// *flag -- host memory the caller spins on instead of a stream
// synchronisation (small_wait)
__device__ __forceinline__ void small_done(uint64_t *flag, uint64_t seq) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// ... and its start: with no stream synchronisation between two calls the
// launch's own acquire may stop at device scope, so lines of the pinned
// input an earlier call read could still sit in L2: dropped here
__device__ __forceinline__ void small_begin() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

// ---- one message from the front of a stream (cpk_read_message) -------------
// Serialize.read over PackedInputStream (Serialize.java:119-178) when the
// message's packed length is unknown: the table is read here, laid out as the
// stream's pieces -- [first word] [rest of the table] [segment 0] ... -- and
// padded with empty pieces (a read() of nothing consumes nothing,
// PackedInputStream.java:38) to kRmPieces, so the stream decoder's launch
// needs nothing from the host.  A failed table (or segments over the
// caller's capacity) leaves every piece empty: nothing is decoded.
constexpr uint32_t kRmHead = 257;              // table words at most (512 segments)
constexpr uint32_t kRmPieces = 2 + 512;        // first word, rest of the table, segments
constexpr uint32_t kRmInfo = 4 + 513;          // status, consumed, count, words, offsets

// sdesc: the one-wave decoder's stream descriptor (DecStreams with one
// stream): [0] its first byte, [1] its end, [2..3] its pieces (the table's
// two and the segments only: the padding is the parallel path's); [5] the
// parallel path's piece count
// (dec_tk: the batch decoder's ticket counters, zeroed here for the one-wave
// decode launched next -- one command fewer than a memset)
// (out, when set -- the one-launch path: the parse's own table words are
// written there and the stream descriptor starts at the first segment, so
// the decoder walks the segments only; otherwise the swo of the padding
// pieces is filled by all threads)
constexpr uint32_t kRmTableBytes = 2576;  // a table's packed bytes at most (257 words: 2,570)
struct RmScratch {
  uint32_t size[512];  // the segments' sizes as the parse reads them
  uint64_t fill[2];    // swo padding: first index, value
};
static_assert(kRmTableBytes % 16 == 0 && kRmTableBytes + sizeof(RmScratch) <= kDecLds, "rm_small_kernel LDS");
__device__ void rm_table_parse(const uint8_t *tb, uint64_t nt, uint64_t avail, uint64_t limit, uint64_t cap_words,
                               uint64_t *__restrict__ swo, uint64_t *__restrict__ info,
                               uint64_t *__restrict__ sdesc, uint64_t *__restrict__ out, RmScratch &rs);
__device__ __forceinline__ void rm_table_body(const uint8_t *__restrict__ packed, uint64_t avail, uint64_t limit,
                                              uint64_t cap_words, uint64_t *__restrict__ swo,
                                              uint64_t *__restrict__ info, uint64_t *__restrict__ sdesc,
                                              uint32_t *__restrict__ dec_tk, uint8_t *tb, RmScratch &rs,
                                              uint64_t *__restrict__ out) {
  if (dec_tk)
    for (uint32_t i = threadIdx.x; i < 8 * kTkStride; i += blockDim.x) dec_tk[i] = 0;
  // the bytes a table can reach staged in LDS (tb) by whole 16-byte lines
  // (readable up to round_up(avail, 16)), so the byte-serial parse below
  // makes no dependent memory round trips -- the packed bytes may be pinned
  // host memory
  const uint64_t nt = min(avail, (uint64_t)kRmTableBytes);
  for (uint32_t i = threadIdx.x; i < (uint32_t)((nt + 15) / 16); i += blockDim.x)
    reinterpret_cast<uint4 *>(tb)[i] = reinterpret_cast<const uint4 *>(packed)[i];
  __syncthreads();
  if (threadIdx.x == 0) rm_table_parse(tb, nt, avail, limit, cap_words, swo, info, sdesc, out, rs);
  if (out) return;
  __syncthreads();
  const uint32_t f0 = (uint32_t)rs.fill[0];
  const uint64_t fv = rs.fill[1];
  for (uint32_t i = f0 + threadIdx.x; i <= kRmPieces; i += blockDim.x) swo[i] = fv;
}
__global__ void rm_table_kernel(const uint8_t *__restrict__ packed, uint64_t avail, uint64_t limit,
                                uint64_t cap_words, uint64_t *__restrict__ swo, uint64_t *__restrict__ info,
                                uint64_t *__restrict__ sdesc, uint32_t *__restrict__ dec_tk) {
  __shared__ __attribute__((aligned(16))) uint8_t tb[kRmTableBytes];
  __shared__ RmScratch rs;
  rm_table_body(packed, avail, limit, cap_words, swo, info, sdesc, dec_tk, tb, rs, nullptr);
}
// (one thread) the table read and checked as doRead does, the message laid
// out as the stream's pieces
__device__ void rm_table_parse(const uint8_t *tb, uint64_t nt, uint64_t avail, uint64_t limit, uint64_t cap_words,
                               uint64_t *__restrict__ swo, uint64_t *__restrict__ info,
                               uint64_t *__restrict__ sdesc, uint64_t *__restrict__ out, RmScratch &rs) {
  uint64_t ip = 0, total = 0;
  uint32_t count = 0;
  int st = read_table(
      tb, nt, limit, ip, count, total, [&](uint32_t i, uint32_t sz) { rs.size[i] = sz; },
      [&](uint32_t i, uint64_t w) {
        if (out) out[i] = w;
      });
  if (st == CPK_OK && total > cap_words) st = CPK_ENOMEM;
  info[0] = (uint64_t)(int64_t)st;
  info[1] = 0;
  info[2] = st == CPK_OK || st == CPK_ENOMEM ? count : 0;
  info[3] = st == CPK_OK || st == CPK_ENOMEM ? total : 0;
  uint64_t w = 0;
  swo[0] = 0;
  if (st == CPK_OK) {
    swo[1] = w = 1;
    swo[2] = w += (count & ~1u) / 2;
    for (uint32_t i = 0; i < count; ++i) {
      info[4 + i] = w;
      swo[3 + i] = w += rs.size[i];
    }
    info[4 + count] = w;
  } else {
    swo[1] = swo[2] = 0;
  }
  rs.fill[0] = (st == CPK_OK ? count : 0) + 3;
  rs.fill[1] = w;
  const bool go = st == CPK_OK;
  // (out: the segments' stream starts where the table's bytes end)
  sdesc[0] = out && go ? ip : 0;
  sdesc[1] = avail;
  sdesc[2] = out && go ? 2 : 0;
  sdesc[3] = go ? count + 2 : 0;
  sdesc[5] = kRmPieces;  // (the parallel path decodes every piece)
}

// the message's status: its table's, else the stream's (a failed piece
// stops the stream: the last piece carries it); the bytes consumed
// (end: where the stream's pieces ended; npieces: how many were decoded)
// (mirror: a host-visible copy of the finished row, or null)
__device__ __forceinline__ void rm_final_body(const uint64_t *__restrict__ end, const int32_t *__restrict__ pstatus,
                                              const uint64_t *__restrict__ npieces, uint64_t *__restrict__ info,
                                              uint64_t *__restrict__ mirror);
__global__ void rm_final_kernel(const uint64_t *__restrict__ end, const int32_t *__restrict__ pstatus,
                                const uint64_t *__restrict__ npieces, uint64_t *__restrict__ info,
                                uint64_t *__restrict__ mirror) {
  rm_final_body(end, pstatus, npieces, info, mirror);
}
__device__ __forceinline__ void rm_final_body(const uint64_t *__restrict__ end, const int32_t *__restrict__ pstatus,
                                              const uint64_t *__restrict__ npieces, uint64_t *__restrict__ info,
                                              uint64_t *__restrict__ mirror) {
  if (threadIdx.x == 0 && (int64_t)info[0] == CPK_OK) {
    const int32_t st = pstatus[*npieces - 1];
    info[0] = (uint64_t)(int64_t)st;
    info[1] = st == CPK_OK ? *end : 0;
  }
  if (!mirror) return;
  __syncthreads();
  const uint32_t rows = 4 + (uint32_t)min(info[2], (uint64_t)512) + 1;  // (status, consumed, count, words, offsets)
  for (uint32_t i = threadIdx.x; i < rows; i += blockDim.x) mirror[i] = info[i];
}

// cpk_read_message whole in ONE launch when the one-wave decoder takes the
// message: the table (rm_table_body, which also writes the table's words),
// the stream of its segments from where the table's bytes end
// (decode_body<true>: one of the four waves finds the stream's ticket) and
// the info row (rm_final_body), separated by workgroup barriers -- three
// launches' dispatch latency saved on the small-message path
// (dcopy, when set: the packed bytes -- pinned host memory -- are first
// copied there by all threads at once, one PCIe round trip instead of one
// per window of the one-wave walk; round_up(avail, 16) + 64 bytes)
__global__ __launch_bounds__(kDecThreads, 1) void rm_small_kernel(
    const uint8_t *__restrict__ packed, uint64_t avail, uint64_t limit, uint64_t cap_words,
    uint64_t *__restrict__ swo, uint64_t *__restrict__ info, uint64_t *__restrict__ sdesc, uint32_t *tk,
    uint64_t *__restrict__ out, uint64_t *__restrict__ in_off, int32_t *__restrict__ pst,
    uint64_t *__restrict__ send_out, uint64_t *__restrict__ mirror, uint8_t *__restrict__ dcopy, uint64_t seq) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  if (mirror) small_begin();
  if (dcopy) {
    const uint32_t lines = (uint32_t)((avail + 15) / 16) + 4;
    for (uint32_t i = threadIdx.x; i < lines; i += blockDim.x)
      reinterpret_cast<uint4 *>(dcopy)[i] = reinterpret_cast<const uint4 *>(packed)[i];
    __syncthreads();
    packed = dcopy;
  }
  rm_table_body(packed, avail, limit, cap_words, swo, info, sdesc, tk, smem,
                *reinterpret_cast<RmScratch *>(smem + kRmTableBytes), out);
  __syncthreads();  // (the layout and the zeroed tickets before the decode)
  decode_body<true>(smem, packed, in_off, swo, kRmPieces, out, pst, tk, avail,
                    DecStreams{sdesc, sdesc + 1, sdesc + 2, 1, send_out, nullptr});
  __syncthreads();  // (the stream's end and statuses before the fold)
  rm_final_body(send_out, pst, sdesc + 3, info, mirror);
  if (mirror) small_done(mirror + kRmInfo, seq);
}

#include "decode_mw.hip"

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
                                      uint8_t *__restrict__ out, const uint64_t *__restrict__ tsize,
                                      uint64_t ocap, uint32_t *err) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const uint64_t s0 = mseg[m], s1 = mseg[m + 1];
  const uint64_t *c = poff + s0 + m;
  for (uint64_t s = s0; s < s1; ++s) soff[s] = c[1 + s - s0];
  // (the caller's output capacity: a table that would pass it is not
  // written, ArrayOutputStream.java:40-42)
  if (c[0] + tsize[m] > ocap) {
    atomicOr(err, kErrCap);
    return;
  }
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

// up to 8 device words gathered into pinned host memory, for the host's
// read-backs of a few sizes (read_words): one launch and one sync instead
// of a copy into pageable memory per word (~15-20 us each)
struct Gather8 {
  const uint64_t *p[8];
};
__global__ void gather8_kernel(Gather8 g, uint32_t k, uint64_t *out) {
  if (threadIdx.x < k) out[threadIdx.x] = *g.p[threadIdx.x];
}

#include "encode_v4.hip"
// the dense form's ring: 11 KiB per wave, the most three workgroups per CU
// leave room for (round 4: config 2's ~7.7 KiB of output per wave overflowed
// 8 KiB rings often enough that waves waited for their offset a third of
// the time; 11 KiB: encode -11 %)
#ifndef CPK_SP_RING_DENSE
#define CPK_SP_RING_DENSE 11264
#endif
#define CPK_SP_RING CPK_SP_RING_DENSE
#define CPK_SP_HCALL 1
#include "encode_sp.hip"
#undef CPK_SP_HCALL
#undef CPK_SP_RING
#include "encode_sp3.hip"
#include "decode_v2.hip"
#include "stream_split.hip"

}  // namespace cpk

// The single pass's sparse form: encode_sp.hip compiled again with B
// reading its words a second time (from L2) instead of holding them in 64
// VGPRs, 4 KiB rings and 6 workgroups per CU.  Mostly-zero batches emit
// little, so each wave's output fits its smaller ring and the extra
// occupancy pays (config 4 encode 3.12 -> 2.89 ms per 131,072 pieces); on
// config 2 a wave's ~6 KiB of output overflows the ring and it is 36 %
// slower, so the device gate takes it only for batches whose sampled words
// are >= 85 % zero (e4_gate_kernel).
#pragma push_macro("CPK_SP_RELOAD")
#pragma push_macro("CPK_SP_RING")
#pragma push_macro("CPK_SP_WPE")
#pragma push_macro("CPK_SP_A1G")
#pragma push_macro("CPK_SP_DEFER")
#pragma push_macro("CPK_SP_WAVES")
#undef CPK_SP_WAVES
#undef CPK_SP_RELOAD
#undef CPK_SP_RING
#undef CPK_SP_WPE
#undef CPK_SP_A1G
#undef CPK_SP_DEFER
#define CPK_SP_RELOAD 1
// (CPK_SPARSE_RING / _WPE / _A1G: A/B knobs for the form's ring, workgroups
// per CU and A1 load groups)
#ifdef CPK_SPARSE_RING
#define CPK_SP_RING CPK_SPARSE_RING
#else
#define CPK_SP_RING 4096
#endif
#ifdef CPK_SPARSE_WPE
#define CPK_SP_WPE CPK_SPARSE_WPE
#else
#define CPK_SP_WPE 6
#endif
#ifdef CPK_SPARSE_A1G
#define CPK_SP_A1G CPK_SPARSE_A1G
#else
#define CPK_SP_A1G 4
#endif
#define CPK_SP_OWN_ROLES 1
// (a step of zero words and no head builds no strings, a pair of them is
// skipped whole: round 6, config 4 encode -1.1 %; the dense form's steps
// are rarely empty)
#define CPK_SP_SKIP 1
#ifdef CPK_SPARSE_HCALL
#define CPK_SP_HCALL 1
#endif
namespace cpk_sparse {
using namespace cpk;
#include "encode_sp.hip"
}  // namespace cpk_sparse
#undef CPK_SP_HCALL
#undef CPK_SP_OWN_ROLES
#undef CPK_SP_DEFER
#undef CPK_SP_SKIP
#pragma pop_macro("CPK_SP_RELOAD")
#pragma pop_macro("CPK_SP_RING")
#pragma pop_macro("CPK_SP_WPE")
#pragma pop_macro("CPK_SP_A1G")
#pragma pop_macro("CPK_SP_DEFER")
#pragma pop_macro("CPK_SP_WAVES")

// ================================================================ C ABI
struct HostPipe;  // host_pipe.hip: staging of the host-memory forms

struct cpk_ctx_s {
  int device;
  int cus;
  uint64_t *status;       // look-back words
  uint64_t status_cap;    // entries
  uint32_t *tickets;      // cpk::kTkWords words: per-XCD counters, plan ticket, error bits
  int encoder;            // 0: single pass (encode_sp.hip); 4: size + emit passes; 5: by piece size
  int sp_form;            // the single pass's form: 0 by density, 1 dense, 2 sparse (CPK_SP_FORM)
  int decoder;            // 2: record index (decode_v2.hip); 1: block map (decode_kernel); 3: by density
  uint64_t *sp_status;    // single pass: look-back word per piece
  uint64_t sp_cap;        //   entries
  uint32_t sp_epoch;      //   launch epoch tagging the look-back words, 1..65535
  uint64_t *sp_desc;      //   message batches: piece descriptors | segment tables
  uint64_t sp_desc_cap;   //   u64 entries
  uint64_t *e4_bv;        // encoder v4: per 64-word step its run boundaries, members, heads
  uint64_t e4_bv_cap;     //   steps (kE4RowBytes each)
  HostPipe *pipe;         // cpk_encode_host / cpk_decode_host staging (lazy)
  uint64_t *ss_buf;       // parallel stream decode scratch (stream_split.hip)
  uint64_t ss_cap;        //   u64 entries
  uint64_t *rm_buf;       // cpk_read_message: piece word offsets | piece ends | statuses (lazy)
  uint64_t *fl_buf;       // cpk_decode_batch of a few large pieces: boundaries found [33] (lazy)
  uint64_t *probe_pin;    // host read-backs of a few device words (read_words): pinned [8] (lazy)
  uint8_t *rm_copy;       // cpk_read_message_host, one-wave path: the packed bytes on the device (lazy)
  uint64_t small_seq;     // the one-launch host paths' completion flag values (small_wait)
  uint64_t small_fallbacks;  // small_wait calls whose flag was unset even after a stream sync (lost flags)
  uint64_t small_timeouts;   // small_wait calls that waited past 5 ms (late launches included)
  uint64_t *sp_units;     // single pass, pieces over one chunk: unit counts | starts | block sums | unit table
  uint64_t sp_units_cap;  //   u64 entries
  // CPK_HOST_TRACE=1 (read at creation): host wall time of the one-message
  // host paths (cpk_encode_host[_gather], cpk_read_message_host) by phase,
  // summed per context and printed to stderr by cpk_ctx_destroy
  uint64_t rm_mw_max;     // cpk_read_message[_host]: streams under it by one workgroup (<= kRmMwMax)
  int e4_order;           // cpk_encode_messages' two passes, segments largest first: 1 both passes,
                          // 2 the emit pass only, 0 neither (CPK_E4_ORDER)
  bool trace;
  double tr_us[8];
  uint64_t tr_n[8];
};
// the phases (write: staging in, enqueues, waits, staging out; read: same)
enum { kTrWIn, kTrWLaunch, kTrWWait, kTrWOut, kTrRIn, kTrRLaunch, kTrRWait, kTrROut };
struct TrClock {
  cpk_ctx c;
  std::chrono::steady_clock::time_point t;
  explicit TrClock(cpk_ctx ctx) : c(ctx) {
    if (c->trace) t = std::chrono::steady_clock::now();
  }
  void mark(int k) {
    if (!c->trace) return;
    const auto n = std::chrono::steady_clock::now();
    c->tr_us[k] += std::chrono::duration<double, std::micro>(n - t).count();
    ++c->tr_n[k];
    t = n;
  }
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

// order[0..n) = 0..n-1 by size class, largest first (cpk::ord_*); hist:
// kOrdClasses u32 of scratch
void ord_launch(const uint64_t *words, uint32_t n, uint32_t *hist, uint32_t *order, hipStream_t s,
                const uint64_t *swo = nullptr) {
  const unsigned tb = 256, tg = (n + tb - 1) / tb;
  (void)hipMemsetAsync(hist, 0, 4 * cpk::kOrdClasses, s);
  hipLaunchKernelGGL(cpk::ord_hist_kernel, dim3(tg), dim3(tb), 0, s, words, n, hist, swo);
  hipLaunchKernelGGL(cpk::ord_scan_kernel, dim3(1), dim3(64), 0, s, hist);
  hipLaunchKernelGGL(cpk::ord_scatter_kernel, dim3(tg), dim3(tb), 0, s, words, n, hist, order, swo);
}

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

static int decode_batch_impl(cpk_ctx ctx, const void *d_packed, const uint64_t *d_in_off, const uint64_t *d_swo,
                             uint32_t n, void *d_out, int32_t *d_status, void *stream, bool probe);

// The end of a one-launch small path (rm_small_kernel, sp_small_kernel):
// its kernel writes seq to *flag (pinned host memory) after all its other
// writes, so the host reads its results once the flag turns -- without the
// stream synchronisation's wait for the kernel's completion signal.  Past a
// bound (the kernel is slow or faulted) the stream synchronisation decides.
// Returns 0 or nonzero like hipStreamSynchronize.
// The flag word is cleared by small_arm before the launch (it is pinned
// memory other calls use for other data) and its values carry a tag no
// offset or size the slot held can equal.
constexpr uint64_t kSmallTag = 0x5ea1ull << 48;
static uint64_t small_arm(cpk_ctx ctx, uint64_t *flag) {
  __atomic_store_n(flag, 0ull, __ATOMIC_RELEASE);
  return kSmallTag | (++ctx->small_seq & ((1ull << 48) - 1));
}
static int small_wait(cpk_ctx ctx, hipStream_t s, const uint64_t *flag, uint64_t seq) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1;; ++i) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return 0;
    __builtin_ia32_pause();
    if ((i & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5)) break;
  }
  // A late launch (a busy GPU, queueing behind other streams, the first
  // module load) also gets here: the stream synchronisation decides.  Only a
  // flag still unset after it -- a kernel that completed without writing it,
  // a device-side bug -- is counted (cpk_ctx_small_fallbacks); a lost flag
  // would otherwise only cost 5 ms per call and pass every test.
  ++ctx->small_timeouts;
  if (hipStreamSynchronize(s) != hipSuccess) return 1;
  if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return 0;
  ++ctx->small_fallbacks;
  return 1;
}
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
    // Encoders: the single pass (encode_sp.hip) for batches of like-sized
    // pieces of 4 Ki words and more (3.65 against 5.06 ms per 131,072
    // config-2 pieces of 8 Ki words; 3.96 against 5.50 ms for 16,384 of
    // 64 Ki words), the two passes (encode_v4.hip) for mixed sizes and
    // message batches; chosen on the device (e4_gate_kernel) among the
    // batches sp_takes admits.  CPK_ENCODER=0 / 4 force one of them.
    const char *e = getenv("CPK_ENCODER");
    c->encoder = (e && e[0] == '4') ? 4 : (e && e[0] == '0') ? 0 : 5;
    // CPK_SP_FORM=dense / sparse forces the single pass's form where the
    // gate picks the single pass (A/B of the density threshold)
    const char *f = getenv("CPK_SP_FORM");
    c->sp_form = (f && f[0] == 'd') ? 1 : (f && f[0] == 's') ? 2 : 0;
    // CPK_DECODER=1 selects the block-map decoder, 2 the record-index one
    const char *d = getenv("CPK_DECODER");
    c->decoder = (d && d[0] == '2') ? 2 : (d && d[0] == '1') ? 1 : 3;
    const char *t = getenv("CPK_HOST_TRACE");
    c->trace = t && t[0] == '1';
    // (CPK_RM_MW_MAX_KB: A/B of the one-workgroup reader's upper bound)
    const char *m = getenv("CPK_RM_MW_MAX_KB");
    c->rm_mw_max = m ? (uint64_t)atoll(m) << 10 : 0;
    const char *o = getenv("CPK_E4_ORDER");
    c->e4_order = o ? atoi(o) : 1;
  }
  if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    c->cus = 256;
  if (hipMalloc(&c->tickets, cpk::kTkWords * 4) != hipSuccess ||
      hipMemset(c->tickets, 0, cpk::kTkWords * 4) != hipSuccess) {
    free(c);
    return CPK_ENOMEM;
  }
  // the kernels' dynamic LDS, above the 64 KiB default for some: set here,
  // with the context's device current (the attribute is per device).  The
  // library is built for gfx950 only (160 KiB of LDS per CU): each request
  // is checked against that at compile time, so a refused attribute is a
  // runtime/driver failure, reported as CPK_EDEVICE
  constexpr uint32_t kGfx950Lds = 160 * 1024;
  static_assert(cpk::kDecLds <= kGfx950Lds && cpk::kSpLds <= kGfx950Lds && cpk::kSpSmallLds <= kGfx950Lds &&
                    cpk::kMwLds <= kGfx950Lds && cpk::kSsLds <= kGfx950Lds,
                "a kernel's dynamic LDS exceeds gfx950's 160 KiB");
  const struct {
    const void *f;
    uint32_t bytes;
  } lds[] = {{(const void *)cpk::decode_kernel<false>, cpk::kDecLds},
             {(const void *)cpk::decode_kernel<true>, cpk::kDecLds},
             {(const void *)cpk::decode_kernel<false, true>, cpk::kDecLds},
             {(const void *)cpk::decode_kernel<true, true>, cpk::kDecLds},
             {(const void *)cpk::sp_encode_kernel<true>, cpk::kSpLds},
             {(const void *)cpk::sp_encode_kernel<false>, cpk::kSpLds},
             {(const void *)cpk::sp_small_kernel, cpk::kSpSmallLds},
             {(const void *)cpk::rm_mw_kernel, cpk::kMwLds},
             {(const void *)cpk::stream_mw_kernel, cpk::kMwLds},
             {(const void *)cpk::ss_scan_kernel, cpk::kSsLds}};
  for (const auto &k : lds)
    if (hipFuncSetAttribute(k.f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)k.bytes) != hipSuccess) {
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
  if (ctx->trace) {
    static const char *nm[8] = {"write staging in", "write enqueue", "write wait", "write staging out",
                                "read staging in", "read enqueue", "read wait", "read staging out"};
    for (int k = 0; k < 8; ++k)
      if (ctx->tr_n[k])
        fprintf(stderr, "cpk host trace: %-18s %8llu marks %12.1f us total\n", nm[k],
                (unsigned long long)ctx->tr_n[k], ctx->tr_us[k]);
  }
  if (ctx->status) hipFree(ctx->status);
  if (ctx->tickets) hipFree(ctx->tickets);
  if (ctx->e4_bv) hipFree(ctx->e4_bv);
  if (ctx->sp_status) hipFree(ctx->sp_status);
  if (ctx->sp_desc) hipFree(ctx->sp_desc);
  if (ctx->ss_buf) hipFree(ctx->ss_buf);
  if (ctx->rm_buf) hipFree(ctx->rm_buf);
  if (ctx->fl_buf) hipFree(ctx->fl_buf);
  if (ctx->probe_pin) hipHostFree(ctx->probe_pin);
  if (ctx->rm_copy) hipFree(ctx->rm_copy);
  if (ctx->sp_units) hipFree(ctx->sp_units);
  pipe_destroy(ctx->pipe);
  free(ctx);
}

int cpk_ctx_device(cpk_ctx ctx) { return ctx ? ctx->device : -1; }
uint64_t cpk_ctx_small_fallbacks(cpk_ctx ctx) { return ctx ? ctx->small_fallbacks : 0; }
int cpk_ctx_dense_windows(cpk_ctx ctx, void *stream, uint64_t *serial, uint64_t *given_back) {
  if (!ctx || !serial || !given_back) return CPK_EINVAL;
  if (!cpk::kDecCnt) return CPK_EUNSUPPORTED;  // (counted by the diagnostics build only)
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  uint32_t c[2] = {0, 0};
  if (hipMemcpyAsync(c, ctx->tickets + cpk::kTkDec + 1, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CPK_EDEVICE;
  *serial = c[0];
  *given_back = c[1];
  return CPK_OK;
}

// The device words at src[0..k) (k <= 8) on the host, after the work already
// on stream s: one small kernel writes them to the context's pinned words.
static int read_words(cpk_ctx ctx, hipStream_t s, std::initializer_list<const uint64_t *> src, uint64_t *dst) {
  if (!ctx->probe_pin && hipHostMalloc((void **)&ctx->probe_pin, 8 * 8, hipHostMallocDefault) != hipSuccess) {
    ctx->probe_pin = nullptr;
    return CPK_ENOMEM;
  }
  cpk::Gather8 g = {};
  uint32_t k = 0;
  for (const uint64_t *p : src) g.p[k++] = p;
  hipLaunchKernelGGL(cpk::gather8_kernel, dim3(1), dim3(64), 0, s, g, k, ctx->probe_pin);
  if (hipStreamSynchronize(s) != hipSuccess) return CPK_EDEVICE;
  for (uint32_t i = 0; i < k; ++i) dst[i] = ctx->probe_pin[i];
  return CPK_OK;
}

// Single-pass encoder (encode_sp.hip): one launch, the look-back words
// epoch-tagged (cleared only when the epoch wraps or the array grows).  Work
// is ticketed per 8192-word chunk of a piece (a unit); a batch whose pieces
// may be larger than one chunk (the hint) first gets its unit table (three
// small kernels and the e4 scan, no host sync: the unit count stays on the
// device).  sp_takes screens which batches it takes; cpk_encode_batch lets
// the device choose by the piece sizes (e4_gate_kernel).
static uint64_t sp_unit_bound(uint64_t n, uint64_t hint);
// whether the single pass is enqueued at all (for the device to choose): a
// size hint, and a unit table of bounded size for pieces over one chunk (a
// loose hint would otherwise size it for nothing)
static bool sp_takes(cpk_ctx ctx, uint32_t n, uint64_t max_seg_words) {
  if (ctx->encoder == 0) return true;  // (CPK_ENCODER=0: single pass for every batch)
  return ctx->encoder != 4 && max_seg_words != 0 && sp_unit_bound(n, max_seg_words) <= (1ull << 25);
}

// `units`: a bound on the batch's units when its pieces may exceed one
// chunk (0: every piece is one unit)
int sp_launch(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, const uint64_t *pdesc,
              const uint64_t *tin, uint32_t n, uint64_t hint, void *d_out, uint64_t *d_out_off,
              hipStream_t s, bool gated = false, uint64_t units = 0, uint64_t out_cap = ~0ull) {
  const uint64_t ucap = units ? units : n;  // look-back words (+ as many run-state words)
  bool fresh = false;
  if (2 * ucap > ctx->sp_cap) {
    if (ctx->sp_status) hipFree(ctx->sp_status);
    ctx->sp_status = nullptr;
    ctx->sp_cap = 0;
    const uint64_t cap = 2 * ucap < 8192 ? 8192 : 2 * ucap + ucap / 2;
    if (hipMalloc(&ctx->sp_status, cap * 8) != hipSuccess) return CPK_ENOMEM;
    ctx->sp_cap = cap;
    fresh = true;
  }
  if (++ctx->sp_epoch > 0xffffu) {
    ctx->sp_epoch = 1;
    fresh = true;
  }
  if (fresh && hipMemsetAsync(ctx->sp_status, 0, ctx->sp_cap * 8, s) != hipSuccess) return CPK_EDEVICE;
  uint64_t *ustate = ctx->sp_status + ucap;
  const uint64_t *utab = nullptr, *nunits = nullptr;
  if (units) {
    // unit counts -> starts (e4 scan) -> unit table
    const uint32_t nb = (uint32_t)((n + cpk::kE4ScanBlock - 1) / cpk::kE4ScanBlock);
    const uint64_t need = (uint64_t)n + (n + 1) + nb + 1 + units;
    if (need > ctx->sp_units_cap) {
      if (ctx->sp_units) hipFree(ctx->sp_units);
      ctx->sp_units = nullptr;
      ctx->sp_units_cap = 0;
      const uint64_t cap = need + need / 4;
      if (hipMalloc(&ctx->sp_units, cap * 8) != hipSuccess) return CPK_ENOMEM;
      ctx->sp_units_cap = cap;
    }
    uint64_t *ucnt = ctx->sp_units, *ustart = ucnt + n, *bsum = ustart + (n + 1), *tab = bsum + nb + 1;
    const unsigned tb = 256, tg = (n + tb - 1) / tb;
    hipLaunchKernelGGL(cpk::sp_units_count_kernel, dim3(tg), dim3(tb), 0, s, d_swo, pdesc, n, hint, ucnt);
    hipLaunchKernelGGL(cpk::e4_scan_reduce, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s, (const uint64_t *)ucnt, n,
                       bsum);
    hipLaunchKernelGGL(cpk::e4_scan_top, dim3(1), dim3(cpk::kE4ScanThreads), 0, s, bsum, nb);
    hipLaunchKernelGGL(cpk::e4_scan_down, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s, (const uint64_t *)ucnt, n,
                       (const uint64_t *)bsum, ustart);
    hipLaunchKernelGGL(cpk::sp_units_fill_kernel, dim3(tg), dim3(tb), 0, s, (const uint64_t *)ustart, n, tab);
    utab = tab;
    nunits = ustart + n;
  }
  // (gated: the ticket was set by e4_gate_kernel -- exhausted unless the
  // batch is the single pass's)
  if (!gated && hipMemsetAsync(ctx->tickets + cpk::kTkPlan, 0, 4, s) != hipSuccess) return CPK_EDEVICE;
  // (gated: both forms enqueued, the one the gate did not pick returns at once)
  const uint32_t *pick = gated ? ctx->tickets + cpk::kTkGate + 6 : nullptr;
  unsigned grid = (unsigned)(cpk::kSpWpe * ctx->cus);
  if (grid > ucap) grid = (unsigned)ucap;
  if (pdesc)
    hipLaunchKernelGGL(cpk::sp_encode_kernel<true>, dim3(grid), dim3(cpk::kSpThreads), cpk::kSpLds, s,
                       (const uint64_t *)d_in, d_swo, pdesc, tin, n, (uint8_t *)d_out, d_out_off,
                       ctx->sp_status, ctx->sp_epoch, ctx->tickets + cpk::kTkPlan, utab, nunits, ustate, hint,
                       ctx->tickets + cpk::kTkErr, tin ? tin - 1 : (const uint64_t *)nullptr, pick, 0u, out_cap);
  else
    hipLaunchKernelGGL(cpk::sp_encode_kernel<false>, dim3(grid), dim3(cpk::kSpThreads), cpk::kSpLds, s,
                       (const uint64_t *)d_in, d_swo, pdesc, tin, n, (uint8_t *)d_out, d_out_off,
                       ctx->sp_status, ctx->sp_epoch, ctx->tickets + cpk::kTkPlan, utab, nunits, ustate, hint,
                       ctx->tickets + cpk::kTkErr, tin ? tin - 1 : (const uint64_t *)nullptr, pick, 0u, out_cap);
  if (gated && !pdesc) {
    unsigned g2 = (unsigned)(cpk_sparse::kSpWpe * ctx->cus);
    if (g2 > ucap) g2 = (unsigned)ucap;
    hipLaunchKernelGGL(cpk_sparse::sp_encode_kernel<false>, dim3(g2), dim3(cpk_sparse::kSpThreads),
                       cpk_sparse::kSpLds, s, (const uint64_t *)d_in, d_swo, pdesc, tin, n, (uint8_t *)d_out,
                       d_out_off, ctx->sp_status, ctx->sp_epoch, ctx->tickets + cpk::kTkPlan, utab, nunits, ustate,
                       hint, ctx->tickets + cpk::kTkErr, (const uint64_t *)nullptr, pick, 1u, out_cap);
  }
  return hip_ok(hipGetLastError());
}

// a bound on the units of n pieces of at most `hint` words (0: every piece
// one unit); over 2^32 units: unsupported
static uint64_t sp_unit_bound(uint64_t n, uint64_t hint) {
  if (hint <= 64ull * cpk::kSpCS) return 0;
  const uint64_t per = (hint + 64ull * cpk::kSpCS - 1) / (64ull * cpk::kSpCS);
  return n * per;
}

// The size pass's rows for the emit pass (kE4RowBytes per 64-word step):
// `stride` rows per piece from the hint when they fit in 4 GiB, else packed
// by word offset (stride 0: the batch's word count is read back, synchronising
// the stream)
static int e4_rows(cpk_ctx ctx, const uint64_t *d_swo, uint32_t n, uint64_t hint, hipStream_t s,
                   uint64_t &stride) {
  stride = hint ? (hint + 63) / 64 : 0;
  if (stride && stride > cpk::kE4MaxRows / (n ? n : 1)) stride = 0;  // (no overflow)
  uint64_t rows;
  if (stride) {
    rows = (uint64_t)(n ? n : 1) * stride;
  } else {
    uint64_t ends[2];
    int rc = read_words(ctx, s, {d_swo, d_swo + n}, ends);
    if (rc) return rc;
    rows = (ends[1] - ends[0]) / 64 + n + 1;
  }
  if (rows > ctx->e4_bv_cap) {
    if (ctx->e4_bv) hipFree(ctx->e4_bv);
    ctx->e4_bv = nullptr;
    ctx->e4_bv_cap = 0;
    const uint64_t cap = rows + rows / 4;
    if (hipMalloc(&ctx->e4_bv, cap * cpk::kE4RowBytes) != hipSuccess) return CPK_ENOMEM;
    ctx->e4_bv_cap = cap;
  }
  return CPK_OK;
}

// Encoder v4 (encode_v4.hip): size pass, scan, emit pass.  Pieces of any
// size; a piece over the hint is reported (output undefined).  The size pass
// leaves each 64-word step's run boundaries for the emit pass: `stride` rows
// per piece from the hint, or packed by word offset when there is no hint (the
// batch's word count is then read back, synchronising the stream).
int e4_encode(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t n, uint64_t hint,
              void *d_out, uint64_t *d_out_off, hipStream_t s, bool gate = false, uint64_t out_cap = ~0ull) {
  const uint32_t nb = (uint32_t)((n + cpk::kE4ScanBlock - 1) / cpk::kE4ScanBlock);
  int rc = ensure_status(ctx, (uint64_t)n + nb + 1);
  if (rc) return rc;
  uint64_t stride;
  rc = e4_rows(ctx, d_swo, n, hint, s, stride);
  if (rc) return rc;
  uint64_t *sizes = ctx->status, *bsum = ctx->status + n;
  if (hipMemsetAsync(ctx->tickets, 0, cpk::kTkErr * 4, s) != hipSuccess) return CPK_EDEVICE;
  if (gate) {
    // which encoder takes the batch, decided on the device from the piece
    // sizes (no host sync): the other's tickets are exhausted, so its
    // kernels return at once (the scans then write offsets the single pass
    // overwrites)
    uint32_t *mm = ctx->tickets + cpk::kTkGate;
    if (hipMemsetAsync(mm, 0xff, 4, s) != hipSuccess || hipMemsetAsync(mm + 1, 0, 4, s) != hipSuccess ||
        hipMemsetAsync(mm + 3, 0, 4, s) != hipSuccess || hipMemsetAsync(mm + 7, 0, 4, s) != hipSuccess)
      return CPK_EDEVICE;
    const unsigned mg = n < 256u * 256u ? (unsigned)((n + 255) / 256) : 256u;
    hipLaunchKernelGGL(cpk::e4_minmax_kernel, dim3(mg), dim3(256), 0, s, d_swo, n, mm, (const uint64_t *)d_in);
    hipLaunchKernelGGL(cpk::e4_gate_kernel, dim3(1), dim3(64), 0, s, ctx->tickets, mg * 256u, (uint32_t)ctx->sp_form,
                       d_swo, n);
  }
  unsigned grid = (unsigned)(8 * ctx->cus);
  if (grid > (n + cpk::kE4Waves - 1) / cpk::kE4Waves) grid = (n + cpk::kE4Waves - 1) / cpk::kE4Waves;
  hipLaunchKernelGGL(cpk::e4_size_kernel, dim3(grid), dim3(cpk::kE4Threads), 0, s,
                     (const uint64_t *)d_in, d_swo, n, sizes, ctx->tickets + cpk::kTkEnc, hint,
                     ctx->tickets + cpk::kTkErr, ctx->e4_bv, stride,
                     gate ? (const uint32_t *)(ctx->tickets + cpk::kTkGate + 2) : (const uint32_t *)nullptr,
                     (const uint32_t *)nullptr);
  hipLaunchKernelGGL(cpk::e4_scan_reduce, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)sizes, n, bsum);
  hipLaunchKernelGGL(cpk::e4_scan_top, dim3(1), dim3(cpk::kE4ScanThreads), 0, s, bsum, nb);
  hipLaunchKernelGGL(cpk::e4_scan_down, dim3(nb), dim3(cpk::kE4ScanThreads), 0, s,
                     (const uint64_t *)sizes, n, (const uint64_t *)bsum, d_out_off);
  hipLaunchKernelGGL(cpk::e4_emit_kernel, dim3(grid), dim3(cpk::kE4Threads), cpk::kE4Lds, s,
                     (const uint64_t *)d_in, d_swo, n, (const uint64_t *)d_out_off,
                     (uint8_t *)d_out, ctx->tickets + cpk::kTkDec, (const uint64_t *)ctx->e4_bv,
                     stride, gate ? (const uint32_t *)(ctx->tickets + cpk::kTkGate + 2) : (const uint32_t *)nullptr,
                     (const uint64_t *)sizes, out_cap, ctx->tickets + cpk::kTkErr, (const uint32_t *)nullptr);
  return hip_ok(hipGetLastError());
}

int cpk_encode_messages(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t nseg,
                        const uint64_t *d_msg_seg_off, uint32_t nm, uint64_t max_seg_words,
                        void *d_out, uint64_t *d_out_off, void *stream) {
  return cpk_encode_messages_cap(ctx, d_in, d_swo, nseg, d_msg_seg_off, nm, max_seg_words, d_out, ~0ull,
                                 d_out_off, stream);
}
int cpk_encode_messages_cap(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t nseg,
                            const uint64_t *d_msg_seg_off, uint32_t nm, uint64_t max_seg_words,
                            void *d_out, uint64_t out_cap, uint64_t *d_out_off, void *stream) {
  if (!ctx || !d_out_off || (nm && !d_msg_seg_off) || (nseg && !d_swo)) return CPK_EINVAL;
  if (((uintptr_t)d_out & 15) || ((uintptr_t)d_in & 7)) return CPK_EINVAL;
  if (max_seg_words == 0) return CPK_EINVAL;  // (a bound is needed for the step rows)
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (nm == 0) return hip_ok(hipMemsetAsync(d_out_off, 0, 8, s));
  const uint64_t np = (uint64_t)nm + nseg;  // pieces: a table per message + the segments
  if (np > 0xffffffffull) return CPK_EINVAL;
  if (ctx->encoder == 0 || (ctx->encoder != 4 && np <= 1024)) {
    // single pass (forced, or a small batch -- one SerializePacked.write:
    // two launches instead of the two passes' nine; a large batch of mixed
    // sizes takes the two passes, faster there): piece descriptors in
    // message order + the tables' words
    const uint64_t need = 2 * np + (uint64_t)nseg / 2 + nm + 2;
    if (need > ctx->sp_desc_cap) {
      if (ctx->sp_desc) hipFree(ctx->sp_desc);
      ctx->sp_desc = nullptr;
      ctx->sp_desc_cap = 0;
      const uint64_t cap = need + need / 4;
      if (hipMalloc(&ctx->sp_desc, cap * 8) != hipSuccess) return CPK_ENOMEM;
      ctx->sp_desc_cap = cap;
    }
    // pdesc[2 np] | output bound | tables
    uint64_t *pdesc = ctx->sp_desc, *tbuf = ctx->sp_desc + 2 * np + 1;
    const unsigned tb = 256, tg = (nm + tb - 1) / tb;
    hipLaunchKernelGGL(cpk::sp_msg_prep_kernel, dim3(tg), dim3(tb), 0, s, d_swo, d_msg_seg_off, nm, pdesc,
                       tbuf, tbuf - 1);
    // (tables are at most 257 words: the segments' hint bounds the units)
    const uint64_t ub = sp_unit_bound(np, max_seg_words);
    if (ub > 0xffffffffull) return CPK_EUNSUPPORTED;
    return sp_launch(ctx, d_in, nullptr, pdesc, tbuf, (uint32_t)np, max_seg_words, d_out, d_out_off, s, false, ub,
                     out_cap);
  }
  const uint32_t nb = (uint32_t)((np + cpk::kE4ScanBlock - 1) / cpk::kE4ScanBlock);
  // scratch: segment sizes | table sizes | message-order sizes | segment offsets | block sums |
  // the segments largest first (u32) | their class counts (u32)
  int rc = ensure_status(ctx, (uint64_t)nseg + nm + np + nseg + nb + 1 + nseg / 2 + 1 + cpk::kOrdClasses / 2);
  if (rc) return rc;
  uint64_t *ssize = ctx->status, *tsize = ssize + nseg, *comb = tsize + nm, *soff = comb + np;
  uint64_t *bsum = soff + nseg;
  uint32_t *sord = reinterpret_cast<uint32_t *>(bsum + nb + 1), *shist = sord + nseg + (nseg & 1);
  uint64_t stride;
  rc = e4_rows(ctx, d_swo, nseg, max_seg_words, s, stride);
  if (rc) return rc;
  if (hipMemsetAsync(ctx->tickets, 0, cpk::kTkErr * 4, s) != hipSuccess) return CPK_EDEVICE;
  const unsigned tb = 256, tg = (nm + tb - 1) / tb;
  unsigned grid = (unsigned)(8 * ctx->cus);
  if (grid > (nseg + cpk::kE4Waves - 1) / cpk::kE4Waves) grid = (nseg + cpk::kE4Waves - 1) / cpk::kE4Waves;
  // (segments largest first, both passes: a wave takes a whole segment, and a
  // 256 KiB one taken last kept the rest of the chip idle behind it)
  const uint32_t *order = nullptr;
  if (nseg && ctx->e4_order) {
    ord_launch(nullptr, nseg, shist, sord, s, d_swo);
    order = sord;
  }
  const uint32_t *size_order = ctx->e4_order == 1 ? order : nullptr;
  if (nseg)
    hipLaunchKernelGGL(cpk::e4_size_kernel, dim3(grid), dim3(cpk::kE4Threads), 0, s,
                       (const uint64_t *)d_in, d_swo, nseg, ssize, ctx->tickets + cpk::kTkEnc,
                       max_seg_words, ctx->tickets + cpk::kTkErr, ctx->e4_bv, stride, (const uint32_t *)nullptr,
                       size_order);
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
                     (const uint64_t *)d_out_off, soff, (uint8_t *)d_out, (const uint64_t *)tsize, out_cap,
                     ctx->tickets + cpk::kTkErr);
  if (nseg)
    hipLaunchKernelGGL(cpk::e4_emit_kernel, dim3(grid), dim3(cpk::kE4Threads), cpk::kE4Lds, s,
                       (const uint64_t *)d_in, d_swo, nseg, (const uint64_t *)soff, (uint8_t *)d_out,
                       ctx->tickets + cpk::kTkDec, (const uint64_t *)ctx->e4_bv, stride, (const uint32_t *)nullptr,
                       (const uint64_t *)ssize, out_cap, ctx->tickets + cpk::kTkErr, order);
  return hip_ok(hipGetLastError());
}

int cpk_encode_batch(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t n,
                     uint64_t max_seg_words, void *d_out, uint64_t *d_out_off, void *stream) {
  return cpk_encode_batch_cap(ctx, d_in, d_swo, n, max_seg_words, d_out, ~0ull, d_out_off, stream);
}
int cpk_encode_batch_cap(cpk_ctx ctx, const void *d_in, const uint64_t *d_swo, uint32_t n,
                         uint64_t max_seg_words, void *d_out, uint64_t out_cap, uint64_t *d_out_off,
                         void *stream) {
  if (!ctx || (!d_swo && n) || !d_out_off) return CPK_EINVAL;
  if (((uintptr_t)d_out & 15) || ((uintptr_t)d_in & 7)) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return hip_ok(hipMemsetAsync(d_out_off, 0, 8, s));
  if (!sp_takes(ctx, n, max_seg_words))
    return e4_encode(ctx, d_in, d_swo, n, max_seg_words, d_out, d_out_off, s, false, out_cap);
  if (ctx->encoder == 0) {
    // (forced single pass: pieces of any size, several units for a large one)
    uint64_t hint = max_seg_words;
    if (!hint) {  // (no bound given: the batch's words bound every piece)
      uint64_t ends[2];
      int rc = read_words(ctx, s, {d_swo, d_swo + n}, ends);
      if (rc) return rc;
      hint = ends[1] - ends[0];
    }
    uint64_t ub = sp_unit_bound(n, hint);
    if (hint > 64ull * cpk::kSpCS && !max_seg_words) ub = n + hint / (64ull * cpk::kSpCS) + 1;
    if (ub > 0xffffffffull) return CPK_EUNSUPPORTED;
    return sp_launch(ctx, d_in, d_swo, nullptr, nullptr, n, max_seg_words, d_out, d_out_off, s, false, ub,
                     out_cap);
  }
  // by piece size: both enqueued, the device picks one (e4_gate_kernel);
  // pieces over one chunk go to the single pass as several units
  int rc = e4_encode(ctx, d_in, d_swo, n, max_seg_words, d_out, d_out_off, s, true, out_cap);
  if (rc) return rc;
  return sp_launch(ctx, d_in, d_swo, nullptr, nullptr, n, max_seg_words, d_out, d_out_off, s, true,
                   sp_unit_bound(n, max_seg_words), out_cap);
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
  // kErrHint: a piece over its size hint; kErrWait: a cross-workgroup wait
  // timed out (cannot happen by design: every wave it waits on is resident);
  // kErrCap: packed bytes would have passed the caller's output capacity
  // (nothing was written there: ArrayOutputStream.java:40-42 -> IOException)
  if (!e) return CPK_OK;
  return (e & cpk::kErrWait) ? CPK_EDEVICE : (e & cpk::kErrCap) ? CPK_ENOMEM : CPK_EINVAL;
}

// one launch of the configured decoder (grid: as many workgroups per CU as
// its LDS allows, at most 8; never more than the work needs)
namespace {
// which decoder a single-decoder call uses (the record-index one only when
// forced: the by-density choice is made for batches, cpk_decode_batch)
bool dec_v2(cpk_ctx ctx) { return ctx->decoder == 2; }

void dec_launch(cpk_ctx ctx, bool stream, unsigned want, const uint8_t *packed, uint64_t *in_off,
                const uint64_t *swo, uint32_t n, uint64_t *out, int32_t *status, uint64_t avail,
                cpk::DecStreams sd, hipStream_t s, int which = 0) {
  // which: 0 the context's choice, 1 the block map, 2 the record index, 3
  // the block map's dense form (decode_kernel<.., true>)
  const bool v2 = which ? which == 2 : dec_v2(ctx);
  const bool dense = which == 3;
  const uint32_t lds = v2 ? cpk::kD2Lds : cpk::kDecLds;
  const unsigned per_cu = (unsigned)min(8u, 160u * 1024u / lds);
  unsigned grid = per_cu * (unsigned)ctx->cus;
  if (grid > want) grid = want;
  if (grid == 0) grid = 1;
  uint32_t *tk = ctx->tickets + cpk::kTkDec;
  if (v2 && stream)
    hipLaunchKernelGGL(cpk::decode2_kernel<true>, dim3(grid), dim3(cpk::kD2Threads), lds, s, packed, in_off, swo, n,
                       out, status, tk, avail, sd);
  else if (v2)
    hipLaunchKernelGGL(cpk::decode2_kernel<false>, dim3(grid), dim3(cpk::kD2Threads), lds, s, packed, in_off, swo, n,
                       out, status, tk, avail, sd);
  else if (stream && dense)
    hipLaunchKernelGGL((cpk::decode_kernel<true, true>), dim3(grid), dim3(cpk::kDecThreads), lds, s, packed, in_off,
                       swo, n, out, status, tk, avail, sd);
  else if (stream)
    hipLaunchKernelGGL(cpk::decode_kernel<true>, dim3(grid), dim3(cpk::kDecThreads), lds, s, packed, in_off, swo, n,
                       out, status, tk, avail, sd);
  else if (dense)
    hipLaunchKernelGGL((cpk::decode_kernel<false, true>), dim3(grid), dim3(cpk::kDecThreads), lds, s, packed, in_off,
                       swo, n, out, status, tk, avail, sd);
  else
    hipLaunchKernelGGL(cpk::decode_kernel<false>, dim3(grid), dim3(cpk::kDecThreads), lds, s, packed, in_off, swo, n,
                       out, status, tk, avail, sd);
}
}  // namespace

// probe: a batch of <= 32 pieces may read its extent back (one sync) to
// decode a few large pieces as one stream.  The host forms pass false: they
// know the sizes and take that path themselves (cpk_decode_host), so their
// two-slot pipeline never blocks on it; nor does a stream being captured.

int cpk_decode_batch(cpk_ctx ctx, const void *d_packed, const uint64_t *d_in_off,
                     const uint64_t *d_swo, uint32_t n, void *d_out, int32_t *d_status,
                     void *stream) {
  bool probe = n <= 32;
  if (probe && ctx) {
    DeviceGuard g(ctx->device);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
      probe = false;
  }
  return decode_batch_impl(ctx, d_packed, d_in_off, d_swo, n, d_out, d_status, stream, probe);
}

static int decode_batch_impl(cpk_ctx ctx, const void *d_packed, const uint64_t *d_in_off, const uint64_t *d_swo,
                             uint32_t n, void *d_out, int32_t *d_status, void *stream, bool probe) {
  if (!ctx || (n && (!d_in_off || !d_swo || !d_status))) return CPK_EINVAL;
  if (((uintptr_t)d_packed & 15) || ((uintptr_t)d_out & 7)) return CPK_EINVAL;
  if (n == 0) return CPK_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(ctx->tickets + cpk::kTkDec, 0, 8 * cpk::kTkStride * 4, s) != hipSuccess)
    return CPK_EDEVICE;
  // persistent: blocks of 4 independent waves, as many per CU as the LDS holds
  uint64_t *in_off = const_cast<uint64_t *>(d_in_off);
  if (ctx->decoder != 3) {
    dec_launch(ctx, false, (n + 3) / 4, (const uint8_t *)d_packed, in_off, d_swo, n, (uint64_t *)d_out,
               d_status, 0, cpk::DecStreams{nullptr, nullptr, nullptr, 0, nullptr, nullptr}, s);
    return hip_ok(hipGetLastError());
  }
  // by density, decided on the device (dec_gate_kernel): both enqueued, the
  // one not chosen returns at its first instruction
  uint32_t *skip = ctx->tickets + cpk::kTkGate + 8;  // [3]: block map, record index, dense block map
  hipLaunchKernelGGL(cpk::dec_gate_kernel, dim3(1), dim3(64), 0, s, (const uint64_t *)d_in_off, d_swo, n, skip);
  if (probe && n <= 32) {
    // A few pieces: read their extent back (one sync).  With >= 8 MiB of
    // words each on average the batch decoders would give a piece one wave
    // (one 64 MiB piece: ~100 ms), so decode them as one stream, 256-byte
    // blocks in parallel, and let the batch decoders skip when every piece
    // ended exactly at its packed range's end (dec_stream_check_kernel);
    // otherwise they run after it and report the batch form's statuses.
    // (through pinned memory: four copies into pageable memory cost ~75 us
    // per call, ADVICE r5, profiles/r6b_small_decode_launch_overhead.txt)
    uint64_t e[4];
    int rc0 = read_words(ctx, s, {d_in_off, d_in_off + n, d_swo, d_swo + n}, e);
    if (rc0) return rc0;
    if (e[3] - e[2] >= ((uint64_t)n << 20) && (e[0] & 15) == 0 && e[1] >= e[0]) {
      if (!ctx->fl_buf && hipMalloc(&ctx->fl_buf, 33 * 8) != hipSuccess) return CPK_ENOMEM;
      int rc = cpk_decode_stream(ctx, (const uint8_t *)d_packed + e[0], e[1] - e[0], d_swo, n, d_out, ctx->fl_buf,
                                 d_status, s);
      if (rc) return rc;
      hipLaunchKernelGGL(cpk::dec_stream_check_kernel, dim3(1), dim3(64), 0, s, (const uint64_t *)ctx->fl_buf,
                         (const uint64_t *)d_in_off, (const int32_t *)d_status, n, skip);
      if (hipMemsetAsync(ctx->tickets + cpk::kTkDec, 0, 8 * cpk::kTkStride * 4, s) != hipSuccess)
        return CPK_EDEVICE;
    }
  }
  dec_launch(ctx, false, (n + 3) / 4, (const uint8_t *)d_packed, in_off, d_swo, n, (uint64_t *)d_out, d_status, 0,
             cpk::DecStreams{nullptr, nullptr, nullptr, 0, nullptr, skip}, s, 1);
  dec_launch(ctx, false, (n + 3) / 4, (const uint8_t *)d_packed, in_off, d_swo, n, (uint64_t *)d_out, d_status, 0,
             cpk::DecStreams{nullptr, nullptr, nullptr, 0, nullptr, skip + 1}, s, 2);
  dec_launch(ctx, false, (n + 3) / 4, (const uint8_t *)d_packed, in_off, d_swo, n, (uint64_t *)d_out, d_status, 0,
             cpk::DecStreams{nullptr, nullptr, nullptr, 0, nullptr, skip + 2}, s, 3);
  return hip_ok(hipGetLastError());
}

namespace {
// streams of at least this many bytes (after the bound below) are cut into
// blocks and decoded in parallel (stream_split.hip); shorter ones by one
// workgroup (decode_mw.hip; one wave under kRmMwMin).  Device-resident
// (tools/stream_bench.py, config-2 data, one piece): 0.32 MiB packed 0.17 ms
// by the workgroup against 0.23 ms by the block path, 0.65 MiB 0.31 / 0.23
constexpr uint64_t kSsMin = 384 * 1024;
constexpr uint64_t kRmSsMin = 64 * 1024;  // cpk_read_message
// cpk_read_message_host: streams under kRmMwMax bytes in one launch (pinned
// memory, no DMA), by one wave (rm_small_kernel) under kRmMwMin, else by a
// whole workgroup (rm_mw_kernel).  Measured (threshold_probe, config-2-like
// messages): one wave 36.7 / mw 42.9 us at 3.9 KB packed, 51.2 / 45.7 at
// 7.8 KB; mw 54 us at 64 KiB of words (one wave 151), 116 at 256 KiB (the
// parallel block path 206)
constexpr uint64_t kRmMwMin = 6 * 1024;
constexpr uint64_t kRmMwMax = 512 * 1024;
// From host memory the workgroup reads the packed bytes straight from pinned
// memory (PCIe round trips per window) and the block path stages them by
// DMA: the block path is ahead from 128 KiB there (passByBytes replay, 512
// KiB messages: 806 us per iteration against 940 at 256 KiB and 1,190 at
// 512 KiB, profiles/r6c_pass_by_bytes_mw*.txt)
constexpr uint64_t kRmMwMaxHost = 128 * 1024;
uint64_t rm_mw_max(cpk_ctx ctx, bool host) {
  const uint64_t d = host ? kRmMwMaxHost : kRmMwMax;
  return ctx->rm_mw_max && ctx->rm_mw_max < kRmMwMax ? ctx->rm_mw_max : d;
}

// the bytes a stream of `words` words may take: 10 per word at most
uint64_t ss_reach(uint64_t avail, uint64_t words) {
  const uint64_t b = words > (~0ull - 16) / 10 ? ~0ull : 10 * words + 16;
  return avail < b ? avail : b;
}

// parallel stream decode over at most `reach` bytes; enqueues the one-wave
// decoder after it, which runs only if the parallel path met anything
// irregular (it then decodes the whole stream, errors included)
int ss_decode(cpk_ctx ctx, const uint8_t *pk, uint64_t avail, uint64_t reach, const uint64_t *swo, uint32_t n,
              uint64_t *out, uint64_t *in_off, int32_t *status, hipStream_t s) {
  using namespace cpk;
  const uint64_t nb = (reach + kSsBlock - 1) / kSsBlock, ng = (nb + kSsGroup - 1) / kSsGroup;
  // scratch layout (u64 entries)
  const uint64_t need = 5 * nb + 3 * kSsCand * nb + (nb + 1) / 2 + 3 * kSsVar * ng + (kSsVar + 1) * nb +
                        ((kSsVar + 1) * nb + 1) / 2 + (ng + 1) / 2 + ng + 4 * (nb + 1) + (nb + 1) / 2 + 2 + 2;
  if (need > ctx->ss_cap) {
    if (ctx->ss_buf) hipFree(ctx->ss_buf);
    ctx->ss_buf = nullptr;
    ctx->ss_cap = 0;
    const uint64_t cap = need + need / 4;
    if (hipMalloc(&ctx->ss_buf, cap * 8) != hipSuccess) return CPK_ENOMEM;
    ctx->ss_cap = cap;
  }
  uint64_t *q = ctx->ss_buf;
  auto take = [&](uint64_t k) {
    uint64_t *r = q;
    q += k;
    return r;
  };
  SsBufs B;
  B.X = take(nb);
  B.W = take(nb);
  B.C1 = take(nb);
  B.L1 = take(nb);
  B.WL1 = take(nb);
  B.C2 = take(kSsCand * nb);
  B.L2 = take(kSsCand * nb);
  B.WL2 = take(kSsCand * nb);
  B.N2 = (uint32_t *)take((nb + 1) / 2);
  B.GE = take(kSsVar * ng);
  B.GX = take(kSsVar * ng);
  B.GW = take(kSsVar * ng);
  B.VE = take((kSsVar + 1) * nb);
  B.VW = (uint32_t *)take(((kSsVar + 1) * nb + 1) / 2);
  B.GC = (uint32_t *)take((ng + 1) / 2);
  B.GB = take(ng);
  B.E = take(nb + 1);
  B.WO = take(nb + 1);
  B.sin = take(nb + 1);
  B.sswo = take(nb + 1);
  B.sst = (int32_t *)take((nb + 1) / 2);
  B.flag = (uint32_t *)take(2);
  B.lim = take(2);
  if (hipMemsetAsync(B.N2, 0, 4 * nb, s) != hipSuccess || hipMemsetAsync(B.flag, 0, 8, s) != hipSuccess ||
      hipMemsetAsync(ctx->tickets + kTkDec, 0, 8 * kTkStride * 4, s) != hipSuccess)
    return CPK_EDEVICE;
  const unsigned tb = 256, gb = (unsigned)((nb + tb - 1) / tb);
  const uint64_t nsub = (nb + kSsSub - 1) / kSsSub;
  hipLaunchKernelGGL(ss_scan_kernel, dim3((unsigned)ng), dim3(kSsThreads), kSsLds, s, pk, reach, swo, n, nb, B);
  hipLaunchKernelGGL(ss_group_kernel, dim3((unsigned)ng), dim3(64), 0, s, pk, nb, B);
  hipLaunchKernelGGL(ss_top_kernel, dim3(1), dim3(64), 0, s, pk, nb, B);
  hipLaunchKernelGGL(ss_cut_kernel, dim3(gb), dim3(tb), 0, s, nb, B);
  hipLaunchKernelGGL(ss_bound_kernel, dim3((n + 1 + 63) / 64), dim3(64), 0, s, pk, swo, n, nb, in_off, B);
  hipLaunchKernelGGL(ss_sub_kernel, dim3((unsigned)((nsub + 1 + tb - 1) / tb)), dim3(tb), 0, s, swo, n, nb,
                     (const uint64_t *)in_off, B);
  dec_launch(ctx, false, (unsigned)((nsub + 3) / 4), pk, B.sin, B.sswo, (uint32_t)nsub, out, B.sst, 0,
             DecStreams{nullptr, nullptr, nullptr, 0, nullptr}, s);
  hipLaunchKernelGGL(ss_check_kernel, dim3((unsigned)((nsub + tb - 1) / tb)), dim3(tb), 0, s, nsub, B);
  hipLaunchKernelGGL(ss_final_kernel, dim3((n + tb - 1) / tb), dim3(tb), 0, s, n, status, ctx->tickets + kTkDec, B,
                     getenv("CPK_STREAM_NO_FALLBACK") ? 1 : 0);
  // the one-wave decoder: no ticket unless the parallel path gave up
  dec_launch(ctx, true, 1, pk, in_off, swo, n, out, status, avail,
             DecStreams{nullptr, nullptr, nullptr, 1, in_off + n}, s);
  return hip_ok(hipGetLastError());
}
}  // namespace

int cpk_decode_stream(cpk_ctx ctx, const void *d_packed, uint64_t avail,
                      const uint64_t *d_swo, uint32_t n, void *d_out, uint64_t *d_in_off,
                      int32_t *d_status, void *stream) {
  if (!ctx || (n && (!d_in_off || !d_swo || !d_status))) return CPK_EINVAL;
  if (((uintptr_t)d_packed & 15) || ((uintptr_t)d_out & 7)) return CPK_EINVAL;
  if (n == 0) return CPK_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (avail >= kSsMin && !getenv("CPK_STREAM_ONE_WAVE")) {
    // the stream's word count bounds the bytes worth cutting into blocks
    // (the rest of `avail` may be later messages): read it back
    uint64_t ends[2];
    int rc = read_words(ctx, s, {d_swo, d_swo + n}, ends);
    if (rc) return rc;
    const uint64_t reach = ss_reach(avail, ends[1] - ends[0]);
    if (reach >= kSsMin)
      return ss_decode(ctx, (const uint8_t *)d_packed, avail, reach, d_swo, n, (uint64_t *)d_out, d_in_off,
                       d_status, s);
  }
  if (avail >= kRmMwMin && !getenv("CPK_STREAM_ONE_WAVE")) {
    // a mid-size stream: one workgroup, its 16 waves sharing each piece's windows
    hipLaunchKernelGGL(cpk::stream_mw_kernel, dim3(1), dim3(cpk::kMwThreads), cpk::kMwLds, s,
                       (const uint8_t *)d_packed, avail, d_swo, n, (uint64_t *)d_out, d_in_off, d_status);
    return hip_ok(hipGetLastError());
  }
  if (hipMemsetAsync(ctx->tickets + cpk::kTkDec, 0, 8 * cpk::kTkStride * 4, s) != hipSuccess)
    return CPK_EDEVICE;
  // one stream: one wave works, the others find no ticket
  dec_launch(ctx, true, 1, (const uint8_t *)d_packed, d_in_off, d_swo, n, (uint64_t *)d_out, d_status, avail,
             cpk::DecStreams{nullptr, nullptr, nullptr, 1, d_in_off + n}, s);
  return hip_ok(hipGetLastError());
}

}  // extern "C"
static int read_message_impl(cpk_ctx ctx, const void *d_packed, uint64_t avail, uint64_t traversal_limit_words,
                             void *d_out, uint64_t out_cap_words, uint64_t *d_info, void *stream,
                             uint64_t *info_mirror, uint64_t seq = 0, bool *flagged = nullptr);
extern "C" {
int cpk_read_message(cpk_ctx ctx, const void *d_packed, uint64_t avail, uint64_t traversal_limit_words,
                     void *d_out, uint64_t out_cap_words, uint64_t *d_info, void *stream) {
  return read_message_impl(ctx, d_packed, avail, traversal_limit_words, d_out, out_cap_words, d_info, stream,
                           nullptr);
}
}  // extern "C"

// (info_mirror: where rm_final_kernel also copies the info row, e.g. pinned
// host memory read after one sync; d_info null: a device row in rm_buf;
// *flagged set: the one-launch kernel took it and writes seq to
// info_mirror[kRmInfo] when done)
static int read_message_impl(cpk_ctx ctx, const void *d_packed, uint64_t avail, uint64_t traversal_limit_words,
                             void *d_out, uint64_t out_cap_words, uint64_t *d_info, void *stream,
                             uint64_t *info_mirror, uint64_t seq, bool *flagged) {
  if (flagged) *flagged = false;
  using cpk::kRmPieces;
  if (!ctx || (!d_info && !info_mirror) || (avail && !d_packed) || !d_out) return CPK_EINVAL;
  if (((uintptr_t)d_packed & 15) || ((uintptr_t)d_out & 7)) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  // swo [515] | in_off [515] | statuses [514 x i32] | stream descriptor [4] | stream end [1] | pieces [1]
  // | spare [2] | info row [517]
  if (!ctx->rm_buf &&
      hipMalloc(&ctx->rm_buf, (2 * (kRmPieces + 1) + kRmPieces / 2 + 8 + cpk::kRmInfo) * 8ull) != hipSuccess)
    return CPK_ENOMEM;
  if (!d_info) d_info = ctx->rm_buf + 2 * (kRmPieces + 1) + kRmPieces / 2 + 8;
  uint64_t *swo = ctx->rm_buf, *in_off = swo + kRmPieces + 1;
  int32_t *pst = (int32_t *)(in_off + kRmPieces + 1);
  uint64_t *sdesc = in_off + kRmPieces + 1 + kRmPieces / 2, *send_out = sdesc + 4, *npad = sdesc + 5;
  // the pieces' sizes are on the device only: the stream decoder is sized by
  // the bytes the caller's capacity can reach (10 per word at most)
  const uint64_t reach = ss_reach(avail, out_cap_words + cpk::kRmHead);
  // (a lower bar than cpk_decode_stream's: a message's one-wave decode is
  //  ~0.5 GB/s, the parallel path ~250 us of fixed cost: even at 64 KiB)
  const bool one = getenv("CPK_STREAM_ONE_WAVE") != nullptr;
  if (!one && !dec_v2(ctx) && reach >= kRmMwMin && reach < rm_mw_max(ctx, info_mirror != nullptr)) {
    // (the host path: pinned bytes, copied to the device in the kernel)
    if (info_mirror && !ctx->rm_copy && hipMalloc(&ctx->rm_copy, kRmMwMax + 128) != hipSuccess)
      return CPK_ENOMEM;
    hipLaunchKernelGGL(cpk::rm_mw_kernel, dim3(1), dim3(cpk::kMwThreads), cpk::kMwLds, s,
                       (const uint8_t *)d_packed, avail, traversal_limit_words, out_cap_words, swo, d_info, sdesc,
                       (uint64_t *)d_out, in_off, pst, send_out, info_mirror,
                       info_mirror ? ctx->rm_copy : nullptr, seq);
    if (flagged) *flagged = info_mirror != nullptr;
    return hip_ok(hipGetLastError());
  }
  const bool par = reach >= kRmSsMin && !one;
  if (!par && !dec_v2(ctx)) {
    // (the host path's packed bytes are pinned host memory: copied to the
    // device once, in the kernel)
    uint8_t *dcopy = nullptr;
    if (info_mirror && reach + 96 <= kRmMwMax + 128) {
      if (!ctx->rm_copy && hipMalloc(&ctx->rm_copy, kRmMwMax + 128) != hipSuccess) return CPK_ENOMEM;
      dcopy = ctx->rm_copy;
    }
    hipLaunchKernelGGL(cpk::rm_small_kernel, dim3(1), dim3(cpk::kDecThreads), cpk::kDecLds, s,
                       (const uint8_t *)d_packed, avail, traversal_limit_words, out_cap_words, swo, d_info, sdesc,
                       ctx->tickets + cpk::kTkDec, (uint64_t *)d_out, in_off, pst, send_out, info_mirror, dcopy,
                       seq);
    if (flagged) *flagged = info_mirror != nullptr;
    return hip_ok(hipGetLastError());
  }
  hipLaunchKernelGGL(cpk::rm_table_kernel, dim3(1), dim3(64), 0, s, (const uint8_t *)d_packed, avail,
                     traversal_limit_words, out_cap_words, swo, d_info, sdesc,
                     par ? (uint32_t *)nullptr : ctx->tickets + cpk::kTkDec);
  int rc;
  if (par) {
    // every piece, the padding included, gets a status; the last carries the stream's
    rc = ss_decode(ctx, (const uint8_t *)d_packed, avail, reach, swo, kRmPieces, (uint64_t *)d_out, in_off, pst, s);
  } else {
    // one wave over the table's pieces and the segments (the piece count is
    // on the device: a one-stream descriptor), none of the padding; its
    // tickets were zeroed by rm_table_kernel
    dec_launch(ctx, true, 1, (const uint8_t *)d_packed, in_off, swo, kRmPieces, (uint64_t *)d_out, pst, avail,
               cpk::DecStreams{sdesc, sdesc + 1, sdesc + 2, 1, send_out}, s);
    rc = hip_ok(hipGetLastError());
  }
  if (rc) return rc;
  hipLaunchKernelGGL(cpk::rm_final_kernel, dim3(1), dim3(64), 0, s, par ? (const uint64_t *)(in_off + kRmPieces)
                                                                        : (const uint64_t *)send_out,
                     (const int32_t *)pst, par ? (const uint64_t *)npad : (const uint64_t *)(sdesc + 3), d_info,
                     info_mirror);
  return hip_ok(hipGetLastError());
}
extern "C" {

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
  // (+ the stream order: nm u32 and kOrdClasses u32)
  int rc = ensure_status(ctx, 3ull * nm + 1 + 2ull * nb + (nm + 1) / 2 + cpk::kOrdClasses / 2);
  if (rc) return rc;
  uint64_t *mwords = ctx->status, *mbeg = mwords + nm, *mwoff = mbeg + nm;
  uint64_t *bs0 = mwoff + nm + 1, *bs1 = bs0 + nb;
  uint32_t *ord = reinterpret_cast<uint32_t *>(bs1 + nb), *ohist = ord + ((nm + 1) & ~1u);
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
  uint64_t pk[2] = {0, 0};  // the messages' packed range (the decoder's density choice)
  if (hipGetLastError() != hipSuccess) return CPK_EDEVICE;
  {
    uint64_t w[4];
    const int rcw = read_words(ctx, s, {mwoff + nm, d_msg_seg_off + nm, d_msg_off, d_msg_off + nm}, w);
    if (rcw) return rcw;
    h_totals[0] = w[0];
    h_totals[1] = w[1];
    pk[0] = w[2];
    pk[1] = w[3];
  }
  if (h_totals[0] > out_cap_words || h_totals[1] > seg_cap) return CPK_ENOMEM;
  if (h_totals[1] && (!d_seg_word_off || !d_seg_in_off || !d_seg_status)) return CPK_EINVAL;
  if (!d_seg_word_off) return CPK_OK;  // (no segments: every table failed)
  hipLaunchKernelGGL(cpk::msg_swo_kernel, dim3(tg), dim3(tb), 0, s, (const uint8_t *)d_packed,
                     d_msg_off, nm, traversal_limit_words, (const uint64_t *)mwoff,
                     (const uint64_t *)d_msg_seg_off, (const int32_t *)d_msg_status, d_seg_word_off);
  if (h_totals[1]) {
    if (hipMemsetAsync(ctx->tickets + cpk::kTkDec, 0, 8 * cpk::kTkStride * 4, s) != hipSuccess)
      return CPK_EDEVICE;
    // the messages' streams largest first (ord_*: a counting sort by size class)
    ord_launch(mwords, nm, ohist, ord, s);
    // the stream ends overwrite the words array (no longer needed); dense
    // batches (packed bytes >= 80 % of the words') take the block map's
    // dense form, as dec_gate_kernel picks it for cpk_decode_batch (config 3:
    // 48.0 -> 44.4 ms once the stream form's uniform values sat in scalar
    // registers -- with 36 B/lane of spills it had been 49.9,
    // profiles/r5aa_stream_sgpr.txt)
    const bool dense = ctx->decoder == 3 && pk[1] >= pk[0] && 100 * (pk[1] - pk[0]) >= 80 * 8 * h_totals[0];
    dec_launch(ctx, true, (nm + 3) / 4, (const uint8_t *)d_packed, d_seg_in_off, (const uint64_t *)d_seg_word_off,
               (uint32_t)h_totals[1], (uint64_t *)d_out, d_seg_status, 0,
               cpk::DecStreams{mbeg, d_msg_off + 1, d_msg_seg_off, nm, mwords, nullptr,
                               ord},
               s, dense ? 3 : 0);
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
  for (uint32_t i = 0; i < n; ++i)
    if (h_swo[i + 1] < h_swo[i]) return CPK_EINVAL;
  const uint64_t words = h_swo[n] - h_swo[0];
  if ((!h_packed && avail) || (!h_out && words)) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  // only the bytes the stream can reach are staged (the rest of `avail` may
  // be later messages), through the context's pinned slot 0 (grow-only: no
  // allocation once it is large enough)
  const uint64_t R = ss_reach(avail, words);
  HostPipe *p = nullptr;
  // meta: swo | in_off | status (int32)
  int rc = pipe_get(ctx, R, words * 8, 2 * (n + 1ull) + n / 2 + 1, &p, 1);
  if (rc) return rc;
  HostSlot &sl = p->slot[0];
  uint64_t *m = sl.pin_meta, *dm = sl.d_meta;
  for (uint32_t i = 0; i <= n; ++i) m[i] = h_swo[i] - h_swo[0];
  memset((uint8_t *)sl.pin_in + R, 0, 64);  // (the decoder's read slack)
  if (hipMemcpyAsync(dm, m, (n + 1) * 8ull, hipMemcpyHostToDevice, p->sk) ||
      h2d_pipelined(sl.d_in, sl.pin_in, h_packed, R, p->sk) ||
      hipMemcpyAsync((uint8_t *)sl.d_in + R, (uint8_t *)sl.pin_in + R, 64, hipMemcpyHostToDevice, p->sk))
    return CPK_EDEVICE;
  rc = cpk_decode_stream(ctx, sl.d_in, R, dm, n, sl.d_out, dm + n + 1, (int32_t *)(dm + 2 * (n + 1ull)), p->sk);
  if (rc) {
    pipe_drain(p);
    return rc;
  }
  if (hipMemcpyAsync(m + n + 1, dm + n + 1, (n + 1) * 8ull + n * 4ull, hipMemcpyDeviceToHost, p->sk))
    return CPK_EDEVICE;
  if (words) {
    if (d2h_pipelined((uint8_t *)h_out + 8 * h_swo[0], sl.pin_out, sl.d_out, words * 8, p->sk, sl.eh, sl.ed))
      return CPK_EDEVICE;
  } else if (hipStreamSynchronize(p->sk)) {
    return CPK_EDEVICE;
  }
  memcpy(h_in_off, m + n + 1, (n + 1) * 8ull);
  memcpy(h_status, m + 2 * (n + 1ull), n * 4ull);
  for (uint32_t i = 0; i < n; ++i)
    if (h_status[i] != CPK_OK) return h_status[i];
  return CPK_OK;
}

int cpk_read_message_host(cpk_ctx ctx, const void *h_packed, uint64_t avail, uint64_t traversal_limit_words,
                          void *h_out, uint64_t out_cap_words, uint64_t *h_info) {
  using cpk::kRmInfo;
  if (!ctx || !h_info || (avail && !h_packed) || (out_cap_words && !h_out)) return CPK_EINVAL;
  DeviceGuard g(ctx->device);
  // only the bytes the caller's capacity can reach are staged (the rest of
  // `avail` may be later messages)
  const uint64_t R = ss_reach(avail, out_cap_words + cpk::kRmHead);
  HostPipe *p = nullptr;
  int rc = pipe_get(ctx, R, (out_cap_words + cpk::kRmHead) * 8, kRmInfo + 1, &p, 1);
  if (rc) return rc;
  HostSlot &sl = p->slot[0];
  uint64_t *info = sl.pin_meta;
  TrClock tc(ctx);
  if (R < rm_mw_max(ctx, true) && !getenv("CPK_NO_SMALL")) {
    // the one-wave range: the kernels read the packed bytes from the pinned
    // slot and write the words and the info row into pinned memory in place
    // -- no DMA either way, one sync
    memcpy(sl.pin_in, h_packed, R);
    memset((uint8_t *)sl.pin_in + R, 0, 64);
    tc.mark(kTrRIn);
    const uint64_t seq = small_arm(ctx, info + kRmInfo);
    bool flagged = false;
    rc = read_message_impl(ctx, sl.pin_in, R, traversal_limit_words, sl.pin_out, out_cap_words, nullptr, p->sk,
                           info, seq, &flagged);
    if (rc) {
      pipe_drain(p);
      return rc;
    }
    tc.mark(kTrRLaunch);
    if (flagged ? small_wait(ctx, p->sk, info + kRmInfo, seq) : hipStreamSynchronize(p->sk)) return CPK_EDEVICE;
    tc.mark(kTrRWait);
    const int st = (int)(int64_t)info[0];
    const uint32_t count = (uint32_t)info[2];
    for (int i = 0; i < 4; ++i) h_info[i] = info[i];
    if (st != CPK_OK) return st;
    const uint64_t w0 = info[4], words = info[4 + count] - w0;
    for (uint32_t i = 0; i <= count; ++i) h_info[4 + i] = info[4 + i] - w0;
    if (words) memcpy(h_out, (const uint64_t *)sl.pin_out + w0, words * 8);
    tc.mark(kTrROut);
    return CPK_OK;
  }
  // (the bytes chunk by chunk, DMA under the host copy; then the decoder's
  // 64 bytes of read slack)
  memset((uint8_t *)sl.pin_in + R, 0, 64);
  if (h2d_pipelined(sl.d_in, sl.pin_in, h_packed, R, p->sk) ||
      hipMemcpyAsync((uint8_t *)sl.d_in + R, (uint8_t *)sl.pin_in + R, 64, hipMemcpyHostToDevice, p->sk))
    return CPK_EDEVICE;
  tc.mark(kTrRIn);
  rc = cpk_read_message(ctx, sl.d_in, R, traversal_limit_words, sl.d_out, out_cap_words, sl.d_meta, p->sk);
  if (rc) {
    pipe_drain(p);
    return rc;
  }
  if (hipMemcpyAsync(info, sl.d_meta, kRmInfo * 8ull, hipMemcpyDeviceToHost, p->sk)) return CPK_EDEVICE;
  tc.mark(kTrRLaunch);
  if (hipStreamSynchronize(p->sk)) return CPK_EDEVICE;
  tc.mark(kTrRWait);
  const int st = (int)(int64_t)info[0];
  const uint32_t count = (uint32_t)info[2];
  h_info[0] = info[0];
  h_info[1] = info[1];
  h_info[2] = info[2];
  h_info[3] = info[3];
  if (st != CPK_OK) return st;
  // the segments only (the table's words lead the device buffer)
  const uint64_t w0 = info[4], words = info[4 + count] - w0;
  for (uint32_t i = 0; i <= count; ++i) h_info[4 + i] = info[4 + i] - w0;
  // (the words chunk by chunk: each chunk's copy-out under the next's DMA)
  if (words && d2h_pipelined(h_out, sl.pin_out, (uint64_t *)sl.d_out + w0, words * 8, p->sk, sl.eh, sl.ed))
    return CPK_EDEVICE;
  tc.mark(kTrROut);
  return CPK_OK;
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
