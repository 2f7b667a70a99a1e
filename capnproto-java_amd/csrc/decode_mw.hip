// decode_mw.hip -- one packed stream decoded by all the waves of one
// workgroup: the one-launch path of cpk_read_message_host for messages up to
// kRmMwMax bytes (Serialize.read's pieces one after another, each piece's
// windows spread over the waves).  Included from packed_codec.hip (namespace
// cpk) after rm_small_kernel.
//
// decode_body starts each window at a known tag position (the previous
// window's exit), so one wave walks a piece window by window and a lone wave's
// latency adds up: ~13 us per 3.5 KiB window (tools/micro/small_phases.cpp).
// Here a piece's windows lie on a fixed grid, window t at piece position
// t * kWin, and wave w takes windows w, w + NW, ... .  The chunk walks,
// landing walks and pointer doubling (win_walks) do not depend on where a
// window's true records start, so all waves run them at once.  Then, in
// window order, each wave takes its entry e_t -- the first true record at or
// after its grid start, published by the wave of window t - 1 --, finds the
// lane whose chunk holds it, walks from e_t to the first position some lane
// visited (none when e_t was visited itself), takes the lanes reachable from
// there as the true chain and publishes its exit e_{t+1} at once: a few
// hundred cycles per window on the serial path.  The output offset follows
// the same chain; the block map and expansion (win_emit) run in parallel
// again.  Statuses, words and the stream's end are decode_body<true>'s
// (PackedInputStream.java:35-140 per piece).

constexpr int kMwWaves = 16;                      // waves of the workgroup
constexpr int kMwThreads = 64 * kMwWaves;
constexpr uint32_t kMwDone = 0xffffffffu;         // O-chain value: the piece has ended

// the chain between the waves (LDS): E[t % NW] / O[t % NW] = tag t << 32 |
// value, written by the wave of window t - 1 (its exit / the piece's words
// before window t) and read by the wave of window t
struct MwShared {
  uint64_t E[kMwWaves], O[kMwWaves];
  int32_t st;     // the ended piece's status ...
  uint32_t fin;   // ... and (CPK_OK) the end of its bytes
  uint32_t rounds;  // rounds the piece took (the most any wave ran)
  uint32_t tmo;     // a chain wait timed out (the piece reports CPK_EDEVICE)
};
constexpr uint32_t kMwLds = 2048 + kMwWaves * kDecWaveLds + sizeof(MwShared);

__device__ __forceinline__ void mw_put(uint64_t *slot, uint32_t tag, uint32_t v) {
  __hip_atomic_store(slot, ((uint64_t)tag << 32) | v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (bounded: a chain that never arrives -- cannot happen, every window of
// the round is held by a resident wave -- reads as 0xffffffff, which ends the
// piece: an entry past the bytes / the piece already over; the timeout is
// noted in *tmo and the piece reports CPK_EDEVICE, not a decode status)
__device__ __forceinline__ uint32_t mw_get(uint64_t *slot, uint32_t tag, uint32_t *tmo) {
  uint64_t v;
  uint32_t spins = 0;
  while (((v = __hip_atomic_load(slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 32) != tag) {
    if (++spins > (1u << 22)) {
      atomicOr(tmo, 1u);
      return 0xffffffffu;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
__device__ __forceinline__ uint64_t mw_rl64(uint64_t v, int l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}

// One wave's window t (grid start g) of the piece at packed offset a
// (P readable bytes of the stream from there, W words into dst).  Returns
// true once the piece is over (ended here or in an earlier window): the wave
// takes no more windows of it.
__device__ __forceinline__ bool mw_window(uint8_t *wl, const uint64_t *lut, MwShared &ms, int lane,
                                          const uint8_t *gp, uint64_t a, uint32_t P, int W, uint64_t *dst,
                                          uint64_t g64, uint32_t t) {
  uint8_t *wbuf = wl;
  uint32_t *blk = reinterpret_cast<uint32_t *>(wl + kWinBuf);
  VisMask *visa = reinterpret_cast<VisMask *>(blk);
  const uint32_t slot = t % kMwWaves, nslot = (t + 1) % kMwWaves;
  const bool live = g64 < P;  // (uniform) the window holds bytes of the stream
  const uint32_t g = live ? (uint32_t)g64 : 0u;
  const uint32_t wend = live ? min(g + kWin, P) : 0u;
  const uint8_t *pkw = wbuf;
  uint32_t lend = 0, ph = 0;
  WinWalk ww = {0u, 0u, 0u, 0u, 0ull};
#ifdef CPK_PHASE_STATS
  unsigned long long wph_last = 0, wph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  if (live) {
    // the window's bytes (as decode_body loads them)
    const uint32_t padw = (uint32_t)((a + g) & 15);
    const uint32_t ebase = g - padw;
    const uint32_t need = min(g + kWin + kDecLook, P) - ebase;
    const uint32_t lines = (need + 15) >> 4;
    const uint4 *gsrc = reinterpret_cast<const uint4 *>(gp - padw + g);
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
    lend = ebase + 16 * lines;
    pkw = wbuf + (int64_t)padw - (int64_t)g;
    ph = (padw - g) & 3;
    wave_lds_order();
    ww = win_walks<false>(pkw, visa, lane, g, wend DEC_PH_ARGS);
  }
  // ---- the entry (serial over the windows) ----------------------------------
  const uint32_t ein = mw_get(&ms.E[slot], t, &ms.tmo);
  uint64_t onmask = 0;
  uint32_t S = ww.S, enext = ein;
  int j = 0;
  uint32_t sw = 0, q = ein;
  int o = -1;
  if (live && ein < wend) {
    j = (int)chunk_div<kDecChunk>(ein - g);
    // lane j walks from the entry to the first position some lane visited
    // (the entry itself, usually) or out of the window
    if (lane == j) {
      while (q < wend) {
        const uint32_t r = q - g;
        const uint32_t oo = chunk_div<kDecChunk>(r);
        if ((visa[oo] >> (q & 63u)) & 1) {  // (win_walks: the bit of q mod 64)
          o = (int)oo;
          break;
        }
        const DecRec rr = rec_at<false>(pkw, q);
        sw += rr.nw;
        q += rr.len;
      }
    }
    q = (uint32_t)readlane((int)q, j);
    o = readlane(o, j);
    sw = (uint32_t)readlane((int)sw, j);
    if (o == j) onmask = mw_rl64(ww.R, j);  // into lane j's own walk
    else if (o > j) onmask = (1ull << j) | mw_rl64(ww.R, o);
    else onmask = 1ull << j;                // out of the window
    if (lane == j && o != j) S = q;
    enext = (uint32_t)readlane((int)S, 63 - __builtin_clzll(onmask));
  }
  if (lane == 0) mw_put(&ms.E[nslot], t + 1, enext);
  // ---- the window's records: entries, words --------------------------------
  const bool on = (onmask >> lane) & 1;
  uint32_t entry = ein;
  int myw = 0, T = 0, o0 = 0;
  if (onmask) {
    wave_lds_order();  // (the walks' reads of visa are done)
    if (on && S < wend) visa[chunk_div<kDecChunk>(S - g)] = (VisMask)S;
    wave_lds_order();
    if (lane != j) entry = (uint32_t)visa[lane];
    if (on) {
      if (lane == j && o != j) {
        myw = (int)sw;
      } else {
        // the walk's words from where the true records join it
        const uint32_t from = lane == j ? q : entry;
        uint32_t pre = 0;
        for (uint32_t x = ww.cb; x < from;) {
          const DecRec r = rec_at<false>(pkw, x);
          pre += r.nw;
          x += r.len;
        }
        myw = (int)(ww.wt - pre + ww.lw + (lane == j ? sw : 0u));
      }
    }
    const int inc = wave_incl_add(myw);
    T = readlane(inc, 63);
    o0 = inc - myw;
  }
  // ---- the output offset (serial), then the map and expansion ---------------
  const uint32_t owin = mw_get(&ms.O[slot], t, &ms.tmo);
  if (owin == kMwDone) {  // the piece ended in an earlier window
    if (lane == 0) mw_put(&ms.O[nslot], t + 1, kMwDone);
    return true;
  }
  const int ow = (int)owin;
  auto end_piece = [&](int st, uint32_t fin) {
    if (lane == 0) {
      ms.st = st;
      ms.fin = fin;
      mw_put(&ms.O[nslot], t + 1, kMwDone);
    }
  };
  if (ein >= P) {  // the bytes end before the piece's words: EOF DecodeException
    end_piece(CPK_ETRUNC, 0);
    return true;
  }
  if (!onmask) {  // a record from an earlier window covers this one
    if (lane == 0) mw_put(&ms.O[nslot], t + 1, owin);
    return false;
  }
  const bool fills = ow + T >= W;
  const bool chk = fills || (P - ein < kDecChkReach);
  if (!chk && lane == 0) mw_put(&ms.O[nslot], t + 1, (uint32_t)(ow + T));
  int st = CPK_OK;
  uint32_t fin = 0;
  const bool ok = win_emit<true>(pkw, lut, blk, lane, ein, ow, W, P, T, on, entry, S, onmask, o0, myw, enext,
                                 lend, gp, (uint32_t)(((a + P + 15) & ~15ull) - a), ph, dst, st,
                                 fin, false DEC_PH_ARGS);
  if (!ok) end_piece(st, 0);
  else if (fills && fin) end_piece(CPK_OK, fin);
  else if (chk && lane == 0) mw_put(&ms.O[nslot], t + 1, (uint32_t)(ow + T));
  return !ok || (fills && fin);
}

// Pieces [p0, p1) of the stream at packed[sbeg, slim), back to back, by all
// kMwWaves waves (every thread of the workgroup calls it).  status[piece],
// in_off[piece] (its first byte) and *send_out (the stream's end) as
// decode_body<true> writes them.
__device__ void decode_stream_mw(uint8_t *smem, const uint8_t *__restrict__ packed, uint64_t sbeg, uint64_t slim,
                                 const uint64_t *__restrict__ swo, uint32_t p0, uint32_t p1,
                                 uint64_t *__restrict__ out, int32_t *__restrict__ status,
                                 uint64_t *__restrict__ in_off, uint64_t *__restrict__ send_out) {
  const uint64_t *lut = reinterpret_cast<const uint64_t *>(smem);
  const int lane = lane_id(), w = __builtin_amdgcn_readfirstlane(wave_id());
  uint8_t *wl = smem + 2048 + w * kDecWaveLds;
  MwShared &ms = *reinterpret_cast<MwShared *>(smem + 2048 + kMwWaves * kDecWaveLds);
  fill_luts(reinterpret_cast<uint64_t *>(smem), true);
  // LDS keeps what an earlier kernel left there: no slot may hold a tag this
  // launch will wait for (tags count up from 0 in every launch)
  if (threadIdx.x < kMwWaves) ms.E[threadIdx.x] = ms.O[threadIdx.x] = ~0ull;
  if (threadIdx.x == 0) ms.tmo = 0;
  __syncthreads();
  uint64_t scur = sbeg;
  int sfail = CPK_OK;
  uint32_t tb = 0;  // tag of the next piece's first window
  for (uint32_t seg = p0; seg < p1; ++seg) {
    // (the piece's values are wave-uniform: scalar registers, not VGPRs)
    const uint64_t w0 = rfl64(swo[seg]);
    const int W = __builtin_amdgcn_readfirstlane((int)(swo[seg + 1] - w0));
    const uint64_t a = rfl64(scur);
    if (sfail != CPK_OK || W == 0) {  // (a read() of nothing consumes nothing)
      if (threadIdx.x == 0) {
        status[seg] = sfail;
        in_off[seg] = a;
      }
      continue;
    }
    const uint32_t P = (uint32_t)min(slim - scur, (uint64_t)0xffffffffu);
    if (threadIdx.x == 0) {
      ms.E[tb % kMwWaves] = (uint64_t)tb << 32;  // the piece's first record: position 0
      ms.O[tb % kMwWaves] = (uint64_t)tb << 32;  // no words before it
      ms.rounds = 0;
    }
    __syncthreads();
    // each wave takes its windows until it meets the piece's end; no
    // barrier between the rounds: the chains order every slot's reuse
    uint32_t r = 0;
    for (;; ++r) {
      const uint32_t k = r * kMwWaves + (uint32_t)w;  // the window's index in the piece
      if (mw_window(wl, lut, ms, lane, packed + a, a, P, W, out + w0, (uint64_t)k * kWin, tb + k)) break;
    }
    // (the last wave to stop passed the most rounds: the next piece's tags
    // start past every wave's)
    if (lane == 0) atomicMax(&ms.rounds, r + 1);
    __syncthreads();
    tb += (uint32_t)__builtin_amdgcn_readfirstlane((int)ms.rounds) * kMwWaves;
    const int st = __builtin_amdgcn_readfirstlane(ms.tmo ? CPK_EDEVICE : ms.st);
    if (threadIdx.x == 0) {
      status[seg] = st;
      in_off[seg] = a;
    }
    if (st == CPK_OK) scur = a + (uint32_t)__builtin_amdgcn_readfirstlane((int)ms.fin);
    sfail = st;
    __syncthreads();  // (ms read by all before the next piece seeds it)
  }
  if (threadIdx.x == 0) *send_out = scur;
}

// cpk_read_message in one launch by one kMwWaves-wave workgroup: the packed
// bytes (pinned host memory) copied to the device, the table (rm_table_body),
// the segments by decode_stream_mw, the info row (rm_final_body) and the
// completion flag
__global__ __launch_bounds__(kMwThreads, 1) void rm_mw_kernel(
    const uint8_t *__restrict__ packed, uint64_t avail, uint64_t limit, uint64_t cap_words,
    uint64_t *__restrict__ swo, uint64_t *__restrict__ info, uint64_t *__restrict__ sdesc,
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
  rm_table_body(packed, avail, limit, cap_words, swo, info, sdesc, nullptr, smem,
                *reinterpret_cast<RmScratch *>(smem + kRmTableBytes), out);
  __syncthreads();  // (the layout before the decode)
  decode_stream_mw(smem, packed, sdesc[0], avail, swo, (uint32_t)sdesc[2], (uint32_t)sdesc[3], out, pst, in_off,
                   send_out);
  __syncthreads();  // (the stream's end and statuses before the fold)
  rm_final_body(send_out, pst, sdesc + 3, info, mirror);
  if (mirror) small_done(mirror + kRmInfo, seq);
}

// cpk_decode_stream of a mid-size stream: pieces 0..n-1 from packed[0, avail)
// by one kMwWaves-wave workgroup (in_off[n]: the stream's end)
__global__ __launch_bounds__(kMwThreads, 1) void stream_mw_kernel(const uint8_t *__restrict__ packed, uint64_t avail,
                                                                  const uint64_t *__restrict__ swo, uint32_t n,
                                                                  uint64_t *__restrict__ out,
                                                                  uint64_t *__restrict__ in_off,
                                                                  int32_t *__restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  decode_stream_mw(smem, packed, 0, avail, swo, 0, n, out, status, in_off, in_off + n);
}
