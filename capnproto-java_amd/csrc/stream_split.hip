// stream_split.hip -- parallel decode of ONE packed stream whose piece
// boundaries are not known (cpk_decode_stream: Serialize.read over
// PackedInputStream, Serialize.java:165-175, PackedInputStream.java:35-140).
// Included by packed_codec.hip.
//
// The stream is cut into 256-byte blocks.  A record (tag, its bytes, the run
// count, the literal words) has a length that depends on its own bytes only,
// so a walk from any true record start follows the true parse; the problem is
// to know, per block, where the first true record in it starts.
//   ss_scan   per group of 256 blocks (bytes staged in LDS, a thread per
//             block): a speculative walk from the block's first byte: exit
//             X_b (first record start at/after the block end) and the words
//             of the records it starts in the block, W_b; then a walk from
//             X_{b-1} (the guess of its true entry)
//             merged with the speculative walk: once the two meet they agree
//             to the end of the block, so the exit is X_b and the words
//             follow from W_b.  Non-meeting walks run to the block end.  A
//             landing that skips blocks or misses the guess (long literal
//             runs, non-convergence) registers its exit as a second guess of
//             the block it lands in, which is walked too.
//   ss_group  per group (one wave), the blocks resolved in order for each
//             guess of the group's entry, 64 at a time: runs of blocks whose
//             entry is their first guess are taken at once; a block whose
//             entry lies past its end is crossed by a record (no words), an
//             entry equal to a second guess takes that walk's result, any
//             other is walked here.
//   ss_top    one wave chains the groups (a group whose entry was not guessed
//             is resolved again with the true entry) and scans the words.
//   ss_cut    per block its first record and first word, clamped to the end
//             of the last piece; ss_bound finds each piece boundary (a word
//             offset) as a record start by a walk from the block holding it.
// The blocks are then decoded as independent pieces by the batch decoder.
// Anything irregular -- a record past the end of the bytes, a run across a
// piece boundary, a block the batch decoder rejects -- leaves the one-wave
// stream decoder (decode_kernel<true>) to decode the stream after all, which
// gives the reference's exact error behaviour; on the good path its tickets
// are taken away and it exits at once.

constexpr uint32_t kSsBlock = 256;    // bytes per block
constexpr uint32_t kSsGroup = 256;    // blocks per group (a workgroup's scan, a wave's resolution)
constexpr uint32_t kSsCand = 2;       // second guesses kept per block
constexpr uint32_t kSsVar = 1 + kSsCand;  // group variants: guess 1, second guesses
constexpr uint64_t kSsInf = ~0ull;    // a walk that ran past the end of the bytes

// per-call scratch (u64 arrays; nb blocks, ng groups)
struct SsBufs {
  uint64_t *X, *W;          // speculative exit / words [nb]
  uint64_t *C1, *L1, *WL1;  // landing from X_{b-1}: entry, exit, words [nb]
  uint64_t *C2, *L2, *WL2;  // second guesses [nb * kSsCand]
  uint32_t *N2;             // second guesses registered [nb]
  uint64_t *GE, *GX, *GW;   // group variants: entry, exit, words [ng * kSsVar]
  uint64_t *VE;             // per block entry [kSsVar + 1][nb] (last row: top's redo)
  uint32_t *VW;             // per block words before it in its group [kSsVar + 1][nb]
  uint32_t *GC;             // chosen variant per group [ng]
  uint64_t *GB;             // words before the group [ng]
  uint64_t *E, *WO;         // per block entry / first word [nb + 1]
  uint64_t *sin, *sswo;     // the blocks as batch pieces [nb + 1]
  int32_t *sst;             // their statuses [nb]
  uint32_t *flag;           // [0]: fast path failed; [1]: the end (bytes)
  uint64_t *lim;            // [0]: R, bytes the walks may read; [1]: words wanted
};

// byte sources for the walks: the stream in HBM, or a group's bytes staged
// in LDS ([s0, s1) of the stream; every walk of the group stays inside)
struct SsGlobal {
  const uint8_t *pk;
  uint64_t R;
  __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return pk[min(p, R - 1)]; }
};
struct SsLds {
  const uint8_t *lds;
  uint64_t s0, s1;
  __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return lds[min(p, s1 - 1) - s0]; }
};

// one record from p (< R): false if it runs past R
template <class Rd>
__device__ __forceinline__ bool ss_step(const Rd &rd, uint64_t R, uint64_t &p, uint64_t &w) {
  const uint32_t t = rd(p), c1 = rd(p + 1), c9 = rd(p + 9);
  uint64_t len = 1u + (uint32_t)__builtin_popcount(t), wd = 1;
  if (t == 0) {
    len = 2;
    wd = 1u + c1;
  } else if (t == 0xffu) {
    len = 10u + 8u * c9;
    wd = 1u + c9;
  }
  if (p + len > R) return false;
  p += len;
  w += wd;
  return true;
}

__device__ __forceinline__ uint64_t ss_end(uint64_t b, uint64_t R) { return min(b * kSsBlock + kSsBlock, R); }

// the block's exit and words for entry e (merged with its speculative walk)
template <class Rd>
__device__ __forceinline__ void ss_from(const Rd &rd, uint64_t R, uint64_t b, uint64_t e, uint64_t Xb,
                                        uint64_t Wb, uint64_t &exit, uint64_t &words) {
  const uint64_t end = ss_end(b, R);
  if (e >= end) {  // a record crosses the whole block (or the walk is dead)
    exit = e;
    words = 0;
    return;
  }
  uint64_t t = e, wt = 0, s = b * kSsBlock, ws = 0;
  while (t < end) {
    if (s == t) {  // on the speculative path from here to the end
      exit = Xb;
      words = wt + (Wb - ws);
      return;
    }
    if (s < t) {
      if (!ss_step(rd, R, s, ws)) s = kSsInf;
    } else if (!ss_step(rd, R, t, wt)) {
      exit = kSsInf;
      words = wt;
      return;
    }
  }
  exit = t;
  words = wt;
}

__device__ __forceinline__ uint64_t ss_R(const uint64_t *swo, uint32_t n, uint64_t avail) {
  // a word costs at most 10 bytes in any stream the reference decodes
  const uint64_t total = swo[n] - swo[0];
  return min(avail, 10 * total + 16);
}

// The walks on a group's staged bytes: positions relative to the staged
// start (u32), the three bytes a record may need read together, no branches.
struct SsLw {
  const uint8_t *lds;
  uint32_t last;  // staged bytes - 1
  uint32_t rlim;  // R - s0 (clamped): a record may not end past it
  __device__ __forceinline__ bool step(uint32_t &p, uint32_t &w) const {
    const uint32_t t = lds[min(p, last)], c1 = lds[min(p + 1, last)], c9 = lds[min(p + 9, last)];
    const uint32_t len = t == 0 ? 2u : (t == 0xffu ? 10u + 8u * c9 : 1u + (uint32_t)__builtin_popcount(t));
    const uint32_t wd = t == 0 ? 1u + c1 : (t == 0xffu ? 1u + c9 : 1u);
    if (p + len > rlim) return false;
    p += len;
    w += wd;
    return true;
  }
  // ss_from on the staged bytes: block start bs, end be (relative)
  __device__ __forceinline__ void from(uint32_t bs, uint32_t be, uint32_t e, uint32_t Xb, uint32_t Wb,
                                       uint32_t &exit, uint32_t &words) const {
    if (e >= be) {
      exit = e;
      words = 0;
      return;
    }
    uint32_t t = e, wt = 0, s = bs, ws = 0;
    while (t < be) {
      if (s == t) {
        exit = Xb;
        words = wt + (Wb - ws);
        return;
      }
      if (s < t) {
        if (!step(s, ws)) s = ~0u;
      } else if (!step(t, wt)) {
        exit = ~0u;
        words = wt;
        return;
      }
    }
    exit = t;
    words = wt;
  }
};

// A group's walks run on its bytes staged in LDS: its blocks, the block
// before (whose speculative exit is block b0's first guess) and the 9 after
// (a record is at most 2050 bytes, so a landing from the group's blocks ends
// at most 9 blocks further on), plus the longest record past those.
constexpr uint32_t kSsPre = 1, kSsPost = 9;
constexpr uint32_t kSsLocal = kSsPre + kSsGroup + kSsPost;                      // blocks walked
constexpr uint32_t kSsStage = ((kSsLocal * kSsBlock + 2064) + 15) & ~15u;      // bytes staged
constexpr uint32_t kSsoX = kSsStage, kSsoW = kSsoX + 4 * kSsLocal, kSsoN = kSsoW + 4 * kSsLocal;
constexpr uint32_t kSsoC = kSsoN + 4 * kSsLocal;
constexpr uint32_t kSsLds = kSsoC + 4 * kSsCand * kSsLocal;  // 75,480 B: two groups per CU
constexpr uint32_t kSsThreads = kSsGroup;  // a thread per block
constexpr uint32_t kSsStageLoads = (kSsStage / 16 + kSsThreads - 1) / kSsThreads;

// a workgroup per group: speculative walks, landing walks from the previous
// block's speculative exit, and walks from the landings' exits (the second
// guesses of the blocks they land in, published in global slots)
__global__ __launch_bounds__(kSsThreads) void ss_scan_kernel(const uint8_t *__restrict__ pk, uint64_t avail,
                                                     const uint64_t *__restrict__ swo, uint32_t n, uint64_t nbmax,
                                                     SsBufs B) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint64_t R = ss_R(swo, n, avail);
  const uint32_t t = threadIdx.x;
  if (blockIdx.x == 0 && t == 0) {
    B.lim[0] = R;
    B.lim[1] = swo[n] - swo[0];
  }
  const uint64_t nb = min(nbmax, (R + kSsBlock - 1) / kSsBlock);
  const uint64_t b0 = (uint64_t)blockIdx.x * kSsGroup;
  if (b0 >= nb) return;
  const uint64_t lb0 = b0 ? b0 - kSsPre : 0, lb1 = min(nb, b0 + kSsGroup + kSsPost);
  const uint32_t L = (uint32_t)(lb1 - lb0);
  const uint64_t s0 = lb0 * kSsBlock, s1 = min(R, lb1 * kSsBlock + 2064);
  uint32_t *lx = reinterpret_cast<uint32_t *>(smem + kSsoX);
  uint32_t *lw = reinterpret_cast<uint32_t *>(smem + kSsoW);
  uint32_t *lnc = reinterpret_cast<uint32_t *>(smem + kSsoN);
  uint32_t *lc = reinterpret_cast<uint32_t *>(smem + kSsoC);
  // stage [s0, s1) (16-byte loads: the stream is readable to a 16-byte
  // bound), all of a thread's loads in flight before its LDS writes
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(pk + s0);
    uint4 *dst = reinterpret_cast<uint4 *>(smem);
    const uint32_t lines = (uint32_t)((s1 - s0 + 15) / 16);
    uint4 v[kSsStageLoads];
#pragma unroll
    for (uint32_t k = 0; k < kSsStageLoads; ++k) v[k] = src[min(t + k * kSsThreads, lines - 1)];
#pragma unroll
    for (uint32_t k = 0; k < kSsStageLoads; ++k) {
      const uint32_t i = t + k * kSsThreads;
      if (i < lines) dst[i] = v[k];
    }
    for (uint32_t i = t; i < kSsLocal; i += kSsThreads) lnc[i] = 0;
  }
  __syncthreads();
  const SsLw wk{smem, (uint32_t)(s1 - s0 - 1), (uint32_t)min(R - s0, (uint64_t)0xffffffffu)};
  const uint32_t rel_end = (uint32_t)(min(R, lb1 * kSsBlock) - s0);  // (relative end of the last local block)
  auto rel = [&](uint32_t v) -> uint64_t { return v == ~0u ? kSsInf : s0 + v; };
  // speculative walks of the local blocks (relative exits; ~0u: past R)
  for (uint32_t j = t; j < L; j += kSsThreads) {
    const uint32_t bs = j * kSsBlock, be = min(bs + kSsBlock, rel_end);
    uint32_t p = bs, w = 0;
    while (p < be)
      if (!wk.step(p, w)) {
        p = ~0u;
        break;
      }
    lx[j] = p;
    lw[j] = w;
    const uint64_t b = lb0 + j;
    if (b >= b0 && b < b0 + kSsGroup) {
      B.X[b] = rel(p);
      B.W[b] = w;
    }
  }
  __syncthreads();
  // landing walks of the group's blocks
  const uint64_t b = b0 + t;
  if (b < nb) {
    const uint32_t j = (uint32_t)(b - lb0);
    const uint32_t bs = j * kSsBlock, be = min(bs + kSsBlock, rel_end);
    const uint32_t e = b ? lx[j - 1] : 0u;
    uint32_t x, w;
    wk.from(bs, be, e, lx[j], lw[j], x, w);
    B.C1[b] = rel(e);
    B.L1[b] = rel(x);
    B.WL1[b] = w;
    // where the true parse goes next if e was right: a guess for that block
    if (x != ~0u && s0 + x < R) {
      const uint32_t c = x / kSsBlock;  // (local; j < c <= j + kSsPost)
      if (c < L && x != lx[c - 1]) {
        const uint32_t k = atomicAdd(&lnc[c], 1u);
        if (k < kSsCand) lc[c * kSsCand + k] = x;
      }
    }
  }
  __syncthreads();
  // the second guesses: blocks b0 + 1 .. lb1 - 1
  for (uint32_t j = (uint32_t)(b0 + 1 - lb0) + t; j < L; j += kSsThreads) {
    const uint32_t cnt = min(lnc[j], kSsCand);
    const uint64_t c = lb0 + j;
    const uint32_t bs = j * kSsBlock, be = min(bs + kSsBlock, rel_end);
    for (uint32_t k = 0; k < cnt; ++k) {
      const uint32_t e = lc[j * kSsCand + k];
      uint32_t x, w;
      wk.from(bs, be, e, lx[j], lw[j], x, w);
      const uint32_t slot = atomicAdd(&B.N2[c], 1u);
      if (slot < kSsCand) {
        B.C2[c * kSsCand + slot] = rel(e);
        B.L2[c * kSsCand + slot] = rel(x);
        B.WL2[c * kSsCand + slot] = w;
      }
    }
  }
}

__device__ __forceinline__ uint64_t ss_rl64(uint64_t v, int l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}

struct SsLane {
  uint64_t c1, l1, w1, c2[kSsCand], l2[kSsCand], w2[kSsCand], X, W;
  uint32_t n2;
};

__device__ __forceinline__ void ss_load_lane(const SsBufs &B, uint64_t b, bool ok, SsLane &L) {
  L.c1 = ok ? B.C1[b] : kSsInf - 1;
  L.l1 = ok ? B.L1[b] : 0;
  L.w1 = ok ? B.WL1[b] : 0;
  L.X = ok ? B.X[b] : 0;
  L.W = ok ? B.W[b] : 0;
  L.n2 = ok ? min(B.N2[b], kSsCand) : 0u;
#pragma unroll
  for (int k = 0; k < (int)kSsCand; ++k) {
    const bool h = ok && (uint32_t)k < L.n2;
    L.c2[k] = h ? B.C2[b * kSsCand + k] : 0;
    L.l2[k] = h ? B.L2[b * kSsCand + k] : 0;
    L.w2[k] = h ? B.WL2[b * kSsCand + k] : 0;
  }
}

__device__ __forceinline__ uint64_t ss_scan_add(uint64_t w, int lane) {  // inclusive, over the wave
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(w, d, 64);
    if (lane >= d) w += o;
  }
  return w;
}

// Resolves blocks [b0, b0 + cnt) in order from entry e (one wave, 64 blocks
// at a time): a run of blocks each entered at its first guess is taken at
// once (lane-parallel check); the block that breaks the run is crossed by a
// record, matches a second guess, or is walked.  Row `row` of VE / VW gets
// each block's entry and the words of the group's blocks before it.
__device__ void ss_chain(const uint8_t *__restrict__ pk, uint64_t R, const SsBufs &B, uint64_t nbmax, uint64_t b0,
                         uint32_t cnt, uint64_t e, uint32_t row, int lane, uint64_t &exit, uint64_t &words) {
  uint64_t acc = 0;
  for (uint32_t base = 0; base < cnt; base += 64) {
    const uint32_t m = min(64u, cnt - base);
    const bool ok = (uint32_t)lane < m;
    const uint64_t b = b0 + base + (uint64_t)lane;
    SsLane L;
    ss_load_lane(B, b, ok, L);
    const uint64_t px = __shfl_up(L.l1, 1, 64);
    uint64_t ve = 0, vw = 0;
    uint32_t k = 0;
    while (k < m) {
      // optimistic from lane k: lane k enters at e, a later lane at the
      // first-guess exit of the lane before it
      const uint64_t ent = (uint32_t)lane == k ? e : px;
      const uint64_t bad = __ballot(ok && (uint32_t)lane >= k && ent != L.c1);
      const uint32_t r = bad ? (uint32_t)__builtin_ctzll(bad) : m;
      const bool in = (uint32_t)lane >= k && (uint32_t)lane < r;
      const uint64_t w = ss_scan_add(in ? L.w1 : 0, lane);
      if (in) {
        ve = ent;
        vw = acc + w - L.w1;
      }
      if (r > k) {
        acc += ss_rl64(w, (int)r - 1);
        e = ss_rl64(L.l1, (int)r - 1);
      }
      if (r >= m) break;
      // lane r
      uint64_t x, wr;
      const uint64_t br = b0 + base + r;
      if (e >= ss_end(br, R)) {  // a record crosses the whole block
        x = e;
        wr = 0;
      } else {
        const uint32_t n2 = (uint32_t)__builtin_amdgcn_readlane((int)L.n2, (int)r);
        int hit = -1;
#pragma unroll
        for (int q = 0; q < (int)kSsCand; ++q)
          if (hit < 0 && (uint32_t)q < n2 && e == ss_rl64(L.c2[q], (int)r)) hit = q;
        if (hit >= 0) {
          x = 0;
          wr = 0;
#pragma unroll
          for (int q = 0; q < (int)kSsCand; ++q)
            if (q == hit) {
              x = ss_rl64(L.l2[q], (int)r);
              wr = ss_rl64(L.w2[q], (int)r);
            }
        } else {
          ss_from(SsGlobal{pk, R}, R, br, e, ss_rl64(L.X, (int)r), ss_rl64(L.W, (int)r), x, wr);
        }
      }
      if ((uint32_t)lane == r) {
        ve = e;
        vw = acc;
      }
      acc += wr;
      e = x;
      k = r + 1;
    }
    if (ok) {
      B.VE[row * nbmax + b] = ve;
      B.VW[row * nbmax + b] = (uint32_t)vw;
    }
  }
  exit = e;
  words = acc;
}

// one wave per group, each guess of the group's entry
__global__ __launch_bounds__(64) void ss_group_kernel(const uint8_t *__restrict__ pk, uint64_t nbmax, SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t nb = min(nbmax, (R + kSsBlock - 1) / kSsBlock);
  const uint64_t g = blockIdx.x;
  const uint64_t b0 = g * kSsGroup;
  if (b0 >= nb) return;
  const int lane = (int)threadIdx.x;
  const uint32_t cnt = (uint32_t)min((uint64_t)kSsGroup, nb - b0);
  const uint32_t n20 = min(B.N2[b0], kSsCand);
  for (uint32_t v = 0; v < kSsVar; ++v) {
    const bool have = v == 0 || v - 1 < n20;
    const uint64_t e = v == 0 ? B.C1[b0] : (have ? B.C2[b0 * kSsCand + v - 1] : 0);
    uint64_t x = kSsInf, w = 0;
    if (have) ss_chain(pk, R, B, nbmax, b0, cnt, e, v, lane, x, w);
    if (lane == 0) {
      B.GE[g * kSsVar + v] = have ? e : kSsInf - 1;  // (no guess: never matches)
      B.GX[g * kSsVar + v] = x;
      B.GW[g * kSsVar + v] = w;
    }
  }
}

// one wave: the groups chained from the stream's start; a group entered
// other than guessed is resolved again here (row kSsVar of VE / VW)
__global__ __launch_bounds__(64) void ss_top_kernel(const uint8_t *__restrict__ pk, uint64_t nbmax, SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t nb = min(nbmax, (R + kSsBlock - 1) / kSsBlock);
  const uint64_t ng = (nb + kSsGroup - 1) / kSsGroup;
  const int lane = (int)threadIdx.x;
  uint64_t e = 0, wsum = 0;
  for (uint64_t g0 = 0; g0 < ng; g0 += 64) {
    const uint64_t g = g0 + (uint64_t)lane;
    const bool ok = g < ng;
    uint64_t ge[kSsVar], gx[kSsVar], gw[kSsVar];
#pragma unroll
    for (int v = 0; v < (int)kSsVar; ++v) {
      ge[v] = ok ? B.GE[g * kSsVar + v] : kSsInf - 1;
      gx[v] = ok ? B.GX[g * kSsVar + v] : 0;
      gw[v] = ok ? B.GW[g * kSsVar + v] : 0;
    }
    const uint32_t cnt = (uint32_t)min((uint64_t)64, ng - g0);
    const uint64_t px = __shfl_up(gx[0], 1, 64);
    uint32_t ch = 0;
    uint64_t gb = 0;
    uint32_t i = 0;
    while (i < cnt) {
      // optimistic: from lane i on, every group entered by its first guess
      const uint64_t ent = (uint32_t)lane == i ? e : px;
      const uint64_t bad = __ballot((uint32_t)lane >= i && (uint32_t)lane < cnt && ent != ge[0]);
      const uint32_t k = bad ? (uint32_t)__builtin_ctzll(bad) : cnt;  // first group off the guess
      const bool in = (uint32_t)lane >= i && (uint32_t)lane < k;
      const uint64_t w = ss_scan_add(in ? gw[0] : 0, lane);
      if (in) {
        ch = 0;
        gb = wsum + w - gw[0];
      }
      if (k > i) {
        wsum += ss_rl64(w, (int)k - 1);
        e = ss_rl64(gx[0], (int)k - 1);
      }
      if (k >= cnt) break;
      // group k: another guess, or resolved again with the true entry
      int hit = -1;
#pragma unroll
      for (int v = 1; v < (int)kSsVar; ++v)
        if (hit < 0 && e == ss_rl64(ge[v], (int)k)) hit = v;
      uint64_t x = 0, wk = 0;
      if (hit >= 0) {
#pragma unroll
        for (int v = 1; v < (int)kSsVar; ++v)
          if (v == hit) {
            x = ss_rl64(gx[v], (int)k);
            wk = ss_rl64(gw[v], (int)k);
          }
      } else {
        const uint64_t b0 = (g0 + k) * kSsGroup;
        ss_chain(pk, R, B, nbmax, b0, (uint32_t)min((uint64_t)kSsGroup, nb - b0), e, kSsVar, lane, x, wk);
        hit = (int)kSsVar;
      }
      if ((uint32_t)lane == k) {
        ch = (uint32_t)hit;
        gb = wsum;
      }
      wsum += wk;
      e = x;
      i = k + 1;
    }
    if (ok) {
      B.GC[g] = ch;
      B.GB[g] = gb;
    }
  }
  if (lane == 0) {
    B.E[nb] = e;
    B.WO[nb] = wsum;
  }
}

// per block: its entry and first word under the chosen resolution
__global__ __launch_bounds__(256) void ss_cut_kernel(uint64_t nbmax, SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t nb = min(nbmax, (R + kSsBlock - 1) / kSsBlock);
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint64_t g = b / kSsGroup;
  const uint32_t v = B.GC[g];
  B.E[b] = B.VE[v * nbmax + b];
  B.WO[b] = B.GB[g] + B.VW[v * nbmax + b];
}

// piece boundary j (a word offset) as a record start: a walk from the last
// block whose first word is not past it
__global__ __launch_bounds__(64) void ss_bound_kernel(const uint8_t *__restrict__ pk, const uint64_t *__restrict__ swo,
                                                      uint32_t n, uint64_t nbmax, uint64_t *__restrict__ in_off,
                                                      SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t nb = min(nbmax, (R + kSsBlock - 1) / kSsBlock);
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j > n) return;
  const uint64_t T = swo[j] - swo[0];
  if (j == 0 || nb == 0) {
    if (j == 0) in_off[0] = 0;
    else atomicOr(&B.flag[0], 1u);
    return;
  }
  // last b in [0, nb] with WO[b] <= T (WO[0] = 0)
  uint64_t lo = 0, hi = nb;
  while (lo < hi) {
    const uint64_t mid = (lo + hi + 1) / 2;
    if (B.WO[mid] <= T) lo = mid;
    else hi = mid - 1;
  }
  uint64_t p = B.E[lo], w = B.WO[lo];
  bool good = p < kSsInf;
  while (good && w < T) {
    if (p >= R || !ss_step(SsGlobal{pk, R}, R, p, w)) good = false;
  }
  if (!good || w != T) {
    atomicOr(&B.flag[0], 1u);  // truncated / a run across the boundary
    return;
  }
  in_off[j] = p;
}

// the blocks, kSsSub at a time, as batch pieces, clamped to the last piece's
// end (a few large pieces keep the batch decoder's waves busy; one per block
// would spend them on per-piece setup)
constexpr uint32_t kSsSub = 32;
__global__ __launch_bounds__(256) void ss_sub_kernel(const uint64_t *__restrict__ swo, uint32_t n, uint64_t nbmax,
                                                     const uint64_t *__restrict__ in_off, SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t nb = min(nbmax, (R + kSsBlock - 1) / kSsBlock);
  const uint64_t nsub = (nbmax + kSsSub - 1) / kSsSub;
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > nsub) return;
  const uint64_t b = min(k * kSsSub, nb);
  const uint64_t T = B.lim[1];
  uint64_t e = 0, wo = 0;  // (a failed resolution: every piece empty)
  if (B.flag[0] == 0) {
    e = in_off[n];
    wo = T;
    if (B.WO[b] < T) {
      e = B.E[b];
      wo = B.WO[b];
    }
  }
  B.sin[k] = e;
  B.sswo[k] = swo[0] + wo;
}

__global__ __launch_bounds__(256) void ss_check_kernel(uint64_t nsub, SsBufs B) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (__ballot(k < nsub && B.sst[k] != CPK_OK) && (threadIdx.x & 63) == 0) atomicOr(&B.flag[0], 2u);
}

// good path: statuses, and the fallback decoder's tickets taken away
// (no_fallback: a diagnostic mode, CPK_STREAM_NO_FALLBACK=1, in which a
// stream the parallel path gives up on is reported as CPK_EUNSUPPORTED
// instead of being decoded by one wave -- tests use it to show that the
// parallel path itself decoded a stream)
__global__ __launch_bounds__(256) void ss_final_kernel(uint32_t n, int32_t *__restrict__ status, uint32_t *tickets,
                                                       SsBufs B, int no_fallback) {
  const bool bad = B.flag[0] != 0;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if ((!bad || no_fallback) && i < n) status[i] = bad ? CPK_EUNSUPPORTED : CPK_OK;
  if (blockIdx.x == 0 && threadIdx.x < 8) tickets[threadIdx.x * kTkStride] = (bad && !no_fallback) ? 0u : 0x40000000u;
}
