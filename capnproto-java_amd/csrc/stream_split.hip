// stream_split.hip -- parallel decode of ONE packed stream whose piece
// boundaries are not known (cpk_decode_stream: Serialize.read over
// PackedInputStream, Serialize.java:165-175, PackedInputStream.java:35-140).
// Included by packed_codec.hip.
//
// The stream is cut into 1 KiB blocks.  A record (tag, its bytes, the run
// count, the literal words) has a length that depends on its own bytes only,
// so a walk from any true record start follows the true parse; the problem is
// to know, per block, where the first true record in it starts.
//   ss_spec   per block, a speculative walk from the block's first byte:
//             exit X_b (first record start at/after the block end) and the
//             words of the records it starts in the block, W_b.
//   ss_land   per block, a walk from X_{b-1} (the guess of its true entry)
//             merged with the speculative walk: once the two meet they agree
//             to the end of the block, so the exit is X_b and the words
//             follow from W_b.  Non-meeting walks run to the block end.  A
//             landing that skips blocks or misses the guess (long literal
//             runs, non-convergence) registers its exit as a second guess of
//             the block it lands in; ss_land2 walks those.
//   ss_group  per 64 blocks (one wave), the blocks resolved one after another
//             for each guess of the group's entry: a block whose entry lies
//             past its end is crossed by a record (no words), an entry equal
//             to a guess takes that walk's result, any other is walked here.
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

constexpr uint32_t kSsBlock = 1024;   // bytes per block
constexpr uint32_t kSsGroup = 64;     // blocks per group (one wave)
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

// one record from p (< R): false if it runs past R
__device__ __forceinline__ bool ss_step(const uint8_t *__restrict__ pk, uint64_t R, uint64_t &p, uint64_t &w) {
  const uint32_t t = pk[p];
  const uint32_t c1 = pk[min(p + 1, R - 1)], c9 = pk[min(p + 9, R - 1)];
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
__device__ __forceinline__ void ss_from(const uint8_t *__restrict__ pk, uint64_t R, uint64_t b, uint64_t e,
                                        uint64_t Xb, uint64_t Wb, uint64_t &exit, uint64_t &words) {
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
      if (!ss_step(pk, R, s, ws)) s = kSsInf;
    } else if (!ss_step(pk, R, t, wt)) {
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

__global__ __launch_bounds__(256) void ss_spec_kernel(const uint8_t *__restrict__ pk, uint64_t avail,
                                                      const uint64_t *__restrict__ swo, uint32_t n, uint64_t nbmax,
                                                      SsBufs B) {
  const uint64_t R = ss_R(swo, n, avail);
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b == 0) {
    B.lim[0] = R;
    B.lim[1] = swo[n] - swo[0];
  }
  if (b >= nbmax || b * kSsBlock >= R) return;
  const uint64_t end = ss_end(b, R);
  uint64_t p = b * kSsBlock, w = 0;
  while (p < end)
    if (!ss_step(pk, R, p, w)) {
      p = kSsInf;
      break;
    }
  B.X[b] = p;
  B.W[b] = w;
}

__device__ __forceinline__ void ss_push(SsBufs &B, uint64_t R, uint64_t c, uint64_t e) {
  const uint32_t k = atomicAdd(&B.N2[c], 1u);
  if (k < kSsCand) B.C2[c * kSsCand + k] = e;
  (void)R;
}

__global__ __launch_bounds__(256) void ss_land_kernel(const uint8_t *__restrict__ pk, uint64_t nbmax, SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nb = (R + kSsBlock - 1) / kSsBlock;
  if (b >= nbmax || b >= nb) return;
  const uint64_t e = b ? B.X[b - 1] : 0;
  uint64_t x, w;
  ss_from(pk, R, b, e, B.X[b], B.W[b], x, w);
  B.C1[b] = e;
  B.L1[b] = x;
  B.WL1[b] = w;
  // where the true parse goes next if e was right: a guess for that block
  if (x < R) {
    const uint64_t c = x / kSsBlock;
    if (x != B.X[c - 1]) ss_push(B, R, c, x);
  }
}

__global__ __launch_bounds__(256) void ss_land2_kernel(const uint8_t *__restrict__ pk, uint64_t nbmax, SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nb = (R + kSsBlock - 1) / kSsBlock;
  const uint64_t b = i / kSsCand;
  const uint32_t k = (uint32_t)(i % kSsCand);
  if (b >= nbmax || b >= nb || k >= min(B.N2[b], kSsCand)) return;
  const uint64_t e = B.C2[i];
  uint64_t x, w;
  ss_from(pk, R, b, e, B.X[b], B.W[b], x, w);
  B.L2[i] = x;
  B.WL2[i] = w;
}

__device__ __forceinline__ uint64_t ss_rl64(uint64_t v, int l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}

// The group's blocks resolved in order from entry e (wave-uniform loop; the
// lanes hold the blocks' walk results).  Lane i receives block b0 + i's entry
// and the words of the blocks before it in the group; returns the exit and
// the group's words.
struct SsLane {
  uint64_t c1, l1, w1, c2[kSsCand], l2[kSsCand], w2[kSsCand], X, W;
  uint32_t n2;
};
__device__ __forceinline__ void ss_chain(const uint8_t *__restrict__ pk, uint64_t R, uint64_t b0, uint32_t cnt,
                                         const SsLane &L, uint64_t e, int lane, uint64_t &ve, uint32_t &vw,
                                         uint64_t &exit, uint64_t &words) {
  uint64_t acc = 0;
  ve = 0;
  vw = 0;
  for (uint32_t i = 0; i < cnt; ++i) {
    const uint64_t b = b0 + i;
    if ((uint32_t)lane == i) {
      ve = e;
      vw = (uint32_t)acc;
    }
    uint64_t x, w;
    if (e >= ss_end(b, R)) {
      x = e;
      w = 0;
    } else if (e == ss_rl64(L.c1, (int)i)) {
      x = ss_rl64(L.l1, (int)i);
      w = ss_rl64(L.w1, (int)i);
    } else {
      const uint32_t n2 = (uint32_t)__builtin_amdgcn_readlane((int)L.n2, (int)i);
      int hit = -1;
#pragma unroll
      for (int k = 0; k < (int)kSsCand; ++k)
        if (hit < 0 && (uint32_t)k < n2 && e == ss_rl64(L.c2[k], (int)i)) hit = k;
      if (hit >= 0) {
        uint64_t xs = 0, ws = 0;
#pragma unroll
        for (int k = 0; k < (int)kSsCand; ++k)
          if (k == hit) {
            xs = ss_rl64(L.l2[k], (int)i);
            ws = ss_rl64(L.w2[k], (int)i);
          }
        x = xs;
        w = ws;
      } else {
        ss_from(pk, R, b, e, ss_rl64(L.X, (int)i), ss_rl64(L.W, (int)i), x, w);
      }
    }
    acc += w;
    e = x;
  }
  exit = e;
  words = acc;
}

__device__ __forceinline__ void ss_load_lane(const SsBufs &B, uint64_t b, bool ok, SsLane &L) {
  L.c1 = ok ? B.C1[b] : 0;
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

// one wave per group, each guess of the group's entry
__global__ __launch_bounds__(64) void ss_group_kernel(const uint8_t *__restrict__ pk, uint64_t nbmax, SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t nb = min(nbmax, (R + kSsBlock - 1) / kSsBlock);
  const uint64_t g = blockIdx.x;
  const uint64_t b0 = g * kSsGroup;
  if (b0 >= nb) return;
  const int lane = (int)threadIdx.x;
  const uint32_t cnt = (uint32_t)min((uint64_t)kSsGroup, nb - b0);
  const uint64_t b = b0 + (uint64_t)lane;
  SsLane L;
  ss_load_lane(B, b, (uint32_t)lane < cnt, L);
  const uint32_t n20 = (uint32_t)__builtin_amdgcn_readlane((int)L.n2, 0);
  for (uint32_t v = 0; v < kSsVar; ++v) {
    uint64_t e;
    bool have = true;
    if (v == 0) {
      e = ss_rl64(L.c1, 0);
    } else {
      have = v - 1 < n20;
      e = 0;
#pragma unroll
      for (int k = 0; k < (int)kSsCand; ++k)
        if ((uint32_t)k == v - 1) e = ss_rl64(L.c2[k], 0);
    }
    uint64_t ve = 0, x = kSsInf, w = 0;
    uint32_t vw = 0;
    if (have) ss_chain(pk, R, b0, cnt, L, e, lane, ve, vw, x, w);
    if ((uint32_t)lane < cnt) {
      B.VE[v * nbmax + b] = ve;
      B.VW[v * nbmax + b] = vw;
    }
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
    uint32_t ch = 0;
    uint64_t gb = 0;
    uint32_t i = 0;
    while (i < cnt) {
      // optimistic: from lane i on, every group entered by its first guess
      const uint64_t px = __shfl_up(gx[0], 1, 64);
      const bool chain = (uint32_t)lane > i ? (px == ge[0]) : ((uint32_t)lane == i ? e == ge[0] : true);
      const uint64_t bad = __ballot((uint32_t)lane >= i && (uint32_t)lane < cnt && !chain);
      const uint32_t k = bad ? (uint32_t)__builtin_ctzll(bad) : cnt;  // first group off the guess
      // lanes [i, k): variant 0, words scanned
      {
        const bool in = (uint32_t)lane >= i && (uint32_t)lane < k;
        uint64_t w = in ? gw[0] : 0;
        // inclusive scan (u64 via two 32-bit halves would overflow-carry;
        // the group words fit 40 bits: scan with shuffles)
        for (int d = 1; d < 64; d <<= 1) {
          const uint64_t o = __shfl_up(w, d, 64);
          if (lane >= d) w += o;
        }
        const uint64_t own = in ? gw[0] : 0;
        if (in) {
          ch = 0;
          gb = wsum + w - own;
        }
        if (k > i) {
          wsum += ss_rl64(w, (int)k - 1);
          e = ss_rl64(gx[0], (int)k - 1);
        }
      }
      if (k >= cnt) break;
      // group k: another guess, or resolved again with the true entry
      int hit = -1;
#pragma unroll
      for (int v = 1; v < (int)kSsVar; ++v)
        if (hit < 0 && e == ss_rl64(ge[v], (int)k)) hit = v;
      uint64_t x, w;
      if (hit >= 0) {
        x = 0;
        w = 0;
#pragma unroll
        for (int v = 1; v < (int)kSsVar; ++v)
          if (v == hit) {
            x = ss_rl64(gx[v], (int)k);
            w = ss_rl64(gw[v], (int)k);
          }
      } else {
        const uint64_t gk = g0 + k, b0 = gk * kSsGroup;
        const uint32_t bc = (uint32_t)min((uint64_t)kSsGroup, nb - b0);
        SsLane L;
        ss_load_lane(B, b0 + (uint64_t)lane, (uint32_t)lane < bc, L);
        uint64_t ve;
        uint32_t vw;
        ss_chain(pk, R, b0, bc, L, e, lane, ve, vw, x, w);
        if ((uint32_t)lane < bc) {
          B.VE[kSsVar * nbmax + b0 + lane] = ve;
          B.VW[kSsVar * nbmax + b0 + lane] = vw;
        }
        hit = (int)kSsVar;
      }
      if ((uint32_t)lane == k) {
        ch = (uint32_t)hit;
        gb = wsum;
      }
      wsum += w;
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
    if (p >= R || !ss_step(pk, R, p, w)) good = false;
  }
  if (!good || w != T) {
    atomicOr(&B.flag[0], 1u);  // truncated / a run across the boundary
    return;
  }
  in_off[j] = p;
}

// the blocks as batch pieces, clamped to the last piece's end
__global__ __launch_bounds__(256) void ss_sub_kernel(const uint64_t *__restrict__ swo, uint32_t n, uint64_t nbmax,
                                                     const uint64_t *__restrict__ in_off, SsBufs B) {
  const uint64_t R = B.lim[0];
  const uint64_t nb = min(nbmax, (R + kSsBlock - 1) / kSsBlock);
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nbmax) return;
  const uint64_t T = B.lim[1], endp = in_off[n];
  uint64_t e = endp, wo = T;
  if (b <= nb && B.WO[b] < T) {
    e = B.E[b];
    wo = B.WO[b];
  }
  B.sin[b] = e;
  B.sswo[b] = swo[0] + wo;
}

// good path: statuses, and the fallback decoder's tickets taken away
// (no_fallback: a diagnostic mode, CPK_STREAM_NO_FALLBACK=1, in which a
// stream the parallel path gives up on is reported as CPK_EUNSUPPORTED
// instead of being decoded by one wave -- tests use it to show that the
// parallel path itself decoded a stream)
__global__ __launch_bounds__(256) void ss_final_kernel(uint32_t n, uint64_t nbmax, int32_t *__restrict__ status,
                                                       uint32_t *tickets, SsBufs B, int no_fallback) {
  __shared__ int bad;
  if (threadIdx.x == 0) bad = (int)B.flag[0];
  __syncthreads();
  for (uint64_t b = threadIdx.x; b < nbmax; b += blockDim.x)
    if (B.sst[b] != CPK_OK) bad = 1;
  __syncthreads();
  if (!bad || no_fallback)
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) status[i] = bad ? CPK_EUNSUPPORTED : CPK_OK;
  if (threadIdx.x < 8) tickets[threadIdx.x * kTkStride] = (bad && !no_fallback) ? 0u : 0x40000000u;
}
