// decode_v2.hip -- the decoder with a record index (the default).  Included
// from packed_codec.hip (namespace cpk): the window load, the speculative
// chunk walks and the pointer-doubling chain resolution are decode_kernel's;
// what follows differs.
//
// decode_kernel maps every 4-word output block to its covering record by
// walking each true record once per expansion round and writing one map entry
// per block it covers (a 256-word zero run: 64 entries by one lane while the
// others wait), then expands block by block with a branch per word kind.
// Here each true record is written once, as one 32-bit index entry (its
// window position and first output word), by the lane that holds it; the
// expansion then takes 64 consecutive output words per wave instruction,
// lane = word:
//   * the record covering word w is the index entry at rank (records started
//     at or before w): a 2048-bit map of record starts per expansion round
//     and a popcount below the lane give it;
//   * every word is one 8-byte read at the record's bytes and one v_perm
//     through LUT[tag]: a tagged word expands (PackedInputStream.java:84-90),
//     LUT[0] is all zero bytes (a zero run, :92-105), LUT[0xff] the identity
//     (the 0xFF word and its literal run, :106-134, read at tag + 2 + 8 ofs).
// No per-word branches, and the cost of a run is its words, not its length
// in loop trips of one lane.
// A window with more than kD2NI true records (at most kD2Win / 2) is cut at
// its kD2NI-th record; the next window starts there.

constexpr int kD2Threads = 256;  // 4 independent waves
// workgroups per CU the register budget is sized for (LDS allows 5)
constexpr int kD2Wpe = 5;
constexpr uint32_t kD2Chunk = 48;
constexpr uint32_t kD2Win = 64 * kD2Chunk;                           // packed bytes per window
constexpr uint32_t kD2WinBuf = (kD2Win + 15 + 32 + 16 + 15) & ~15u;  // + pad, look-ahead, slack
constexpr uint32_t kD2NI = 1024;  // records indexed per window
constexpr uint32_t kD2Round = 2048;  // output words per expansion round
constexpr int kD2Unroll = 4;  // 64-word groups expanded together
typedef std::conditional<(kD2Chunk <= 32), uint32_t, uint64_t>::type D2Vis;
static_assert(kD2Chunk <= 64, "visited mask bits");
constexpr uint32_t kD2Info = kD2NI * 4;
static_assert(kD2Info >= 64 * sizeof(D2Vis) + 8, "visited masks live over the index");
// record starts of a round: a byte per output word (plain byte stores, one
// per record: consecutive records never contend for one LDS address as bits
// OR-ed into a shared word would), or a bit per word with atomics
constexpr uint32_t kD2Bits = 0 ? kD2Round : kD2Round / 8;
constexpr uint32_t kD2WaveLds = kD2WinBuf + kD2Info + kD2Bits;
constexpr uint32_t kD2Lds = 2048 + 4 * kD2WaveLds;
constexpr int kD2LinesPerLane = (int)((kD2Win + 47 + 15) / 16 + 63) / 64;
static_assert(kD2Win <= 4095, "record positions are 12-bit");

template <bool kStream>
__global__ __launch_bounds__(kD2Threads, kD2Wpe) void decode2_kernel(
    const uint8_t *__restrict__ packed, uint64_t *__restrict__ in_off,
    const uint64_t *__restrict__ swo, uint32_t n, uint64_t *__restrict__ out,
    int32_t *__restrict__ status, uint32_t *ticket, uint64_t avail, DecStreams sd) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t *lut = reinterpret_cast<uint64_t *>(smem);
  const int lane = lane_id(), w = wave_id();
  uint8_t *wl = smem + 2048 + w * kD2WaveLds;
  uint8_t *wbuf = wl;                                            // window bytes
  uint32_t *info = reinterpret_cast<uint32_t *>(wl + kD2WinBuf); // [kD2NI] record index
  uint32_t *bits = reinterpret_cast<uint32_t *>(wl + kD2WinBuf + kD2Info);  // record starts of a round
  D2Vis *visa = reinterpret_cast<D2Vis *>(info);  // [64], over the index (phases 1-3)
  if (sd.skip && __builtin_amdgcn_readfirstlane(*sd.skip)) return;
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
      e = (uint32_t)__builtin_amdgcn_readfirstlane((int)e);  // (wave-uniform: SGPRs, scalar branches)
      ow = __builtin_amdgcn_readfirstlane(ow);
      if (e >= P) {
        if (ow < W) st = CPK_ETRUNC;  // ArrayInputStream EOF -> DecodeException
        break;
      }
      if (ow >= W) break;  // (trailing input is flagged by the record check)
      const uint32_t wend = min(e + kD2Win, P);
      WPH(0)
      // ---- window load: LDS byte x <-> packed[(a + e) & ~15 + x] ----------
      const uint32_t padw = (uint32_t)((a + e) & 15);
      const uint32_t ebase = e - padw;  // piece position of wbuf[0]
      const uint32_t need = min(e + kD2Win + 32, P) - ebase;  // <= kD2Win + 47 bytes
      const uint32_t lines = (need + 15) >> 4;
      const uint4 *gsrc = reinterpret_cast<const uint4 *>(gp - padw + e);
      // all of a lane's lines (<= 3) in flight at once, then the LDS writes:
      // one memory latency per window instead of one per line
      {
        uint4 l[kD2LinesPerLane];
#pragma unroll
        for (int j = 0; j < kD2LinesPerLane; ++j) {
          const uint32_t L = lane + 64 * j;
          l[j] = L < lines ? gsrc[L] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < kD2LinesPerLane; ++j) {
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
      const uint32_t cb = e + kD2Chunk * lane;
      const uint32_t ce = min(cb + kD2Chunk, wend);
      D2Vis vis = 0;
      uint32_t X = cb, wt = 0;  // wt: output words of the walk
      if (cb < wend) {
        uint32_t pos = cb;
        while (pos < ce) {
          vis |= (D2Vis)1 << (pos - cb);
          const DecRec r = rec_at<!kStream>(pkw, pos);
          wt += r.nw;
          pos += r.len;
        }
        X = pos;
      }
      visa[lane] = vis;
      wave_lds_order();
      // ---- 2: walk on until landing on a visited position -------------------
      uint32_t S = X, lw = 0, lr = 0;  // lw / lr: output words / records of the landing walk
      if (cb < wend) {
        while (S < wend) {
          const uint32_t r = S - e;
          const uint32_t ow_ = r / kD2Chunk;
          if ((visa[ow_] >> (r - ow_ * kD2Chunk)) & 1) break;
          const DecRec rr = rec_at<!kStream>(pkw, S);
          lw += rr.nw;
          ++lr;
          S += rr.len;
        }
      }
      WPH(2)
      // ---- 3: true chain over lanes -----------------------------------------
      // lane j's successor is the owner of its landing point (always a later
      // lane); the true records are on the lanes reachable from lane 0, found
      // by pointer doubling (6 rounds cover a chain of 64)
      int nx = (cb < wend && S < wend) ? (int)((S - e) / kD2Chunk) : 64;
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
      if (((onmask >> lane) & 1) && S < wend) visa[(S - e) / kD2Chunk] = (D2Vis)S;
      wave_lds_order();
      const uint32_t entry = lane == 0 ? e : (uint32_t)visa[lane];
      const bool on = (onmask >> lane) & 1;
      WPH(3)
      // ---- 4: output words of each lane's true records ----------------------
      // [entry, S) = the walk's records from entry (a position the walk
      // visited) plus the landing walk: the walk's words minus those before
      // entry (usually one or two records of a false start)
      // ... and its true records: the walk's visited positions from entry on
      // plus the landing walk's
      int myw = 0, myr = 0;
      if (on) {
        uint32_t pre = 0;
        for (uint32_t q = cb; q < entry;) {
          const DecRec r = rec_at<!kStream>(pkw, q);
          pre += r.nw;
          q += r.len;
        }
        myw = (int)(wt - pre + lw);
        const uint32_t eb = entry - cb;  // (< kD2Chunk: entry is a visited position)
        myr = __builtin_popcountll((uint64_t)vis) - __builtin_popcountll((uint64_t)vis & ((1ull << eb) - 1)) +
              (int)lr;
      }
      const int inc = wave_incl_add(myw);
      const int T = readlane(inc, 63);
      const int o0 = inc - myw;  // window-relative output of this lane's first record
      const int incr = wave_incl_add(myr);
      const int NR = readlane(incr, 63);  // true records in the window
      const int r0 = incr - myr;          // rank of this lane's first record
      WPH(4)
      // ---- 5: the index: each true record's window position and first word ----
      // (the reference's error checks run in a window that may reach the
      // piece's end: PackedInputStream.java:53-138)
      // (within one window plus the longest record, 2,050 bytes, of the end:
      // the window's records start before e + kD2Win)
      const bool chk = (ow + T >= W) || (P - e < kD2Win + 2064);
      // a window with more true records than the index holds ends at its
      // kD2NI-th record (scr: that record's position and first word)
      const bool cut = NR > (int)kD2NI;
      int err = 0x7fffffff;
      uint32_t fin = 0;  // end of the record that fills the piece (if any)
      uint32_t cutq = 0, cuto = 0;
      if (on) {
        int o = o0, rk = r0;
        for (uint32_t q = entry; q < S;) {
          const uint32_t tag = pkw[q], c1 = pkw[q + 1], c9 = pkw[q + 9];
          const uint32_t ntag = 1 + __builtin_popcount(tag);
          const uint32_t zm = 0u - (uint32_t)(tag == 0), fm = 0u - (uint32_t)(tag == 0xffu);
          const int nw = 1 + (int)((zm & c1) + (fm & c9));
          const uint32_t adv = ntag + (zm & 1u) + (fm & (8u * c9 + 1u));
          if (rk >= (int)kD2NI) {
            if (rk == (int)kD2NI) {
              cutq = q;
              cuto = (uint32_t)o;
            }
            break;
          }
          const int oo = ow + o;
          if (chk && oo < W && err == 0x7fffffff) {
            // truncated tag bytes / count / literal run -> EOF DecodeException;
            // a run past the piece -> DecodeException / BufferOverflowException
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
          info[rk] = (q - e) | ((uint32_t)o << 12);
          ++rk;
          o += nw;
          q += adv;
        }
      }
      err = __builtin_amdgcn_readfirstlane(wave_min(err));
      if (err != 0x7fffffff) {
        st = -(err & 7);
        break;
      }
      fin = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_max_u(fin));
      uint32_t Teff = (uint32_t)T, eff_next = enext;
      int NRe = NR;
      if (cut) {
        Teff = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_max_u(cuto));
        eff_next = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_max_u(cutq));
        NRe = (int)kD2NI;
      }
      wave_lds_order();
      WPH(5)
      // ---- 6: expansion, rounds of kD2Round words, lane = word ----
      const uint32_t Tlim = min(Teff, (uint32_t)(W - ow));
      uint64_t *dst_w = dst + ow;
      uint32_t ia = 0;  // the record covering the round's first word
      // two copies of the expansion: one for windows whose records all lie in
      // the loaded bytes (eff_next + 12 <= lend), with unchecked reads
      auto expand = [&](auto allin) __attribute__((always_inline)) {
      constexpr bool kAllIn = decltype(allin)::value;
      for (uint32_t rb = 0; rb < Tlim; rb += kD2Round) {
        const uint32_t re = min(rb + kD2Round, Tlim);
        // the round's record starts after its first word
        for (uint32_t i = (uint32_t)lane; i < kD2Bits / 16; i += 64)
          reinterpret_cast<uint4 *>(bits)[i] = make_uint4(0u, 0u, 0u, 0u);
        wave_lds_order();
        uint32_t ib = ia + 1;
        for (;;) {
          const uint32_t i = ib + (uint32_t)lane;
          const uint32_t oi = i < (uint32_t)NRe ? (info[i] >> 12) : 0xffffffffu;
          const bool in = oi < rb + kD2Round;
          if (in) atomicOr(&bits[(oi - rb) >> 5], 1u << ((oi - rb) & 31));
          const uint64_t outm = __ballot(!in);
          if (outm) {
            ib += (uint32_t)__builtin_ctzll(outm);
            break;
          }
          ib += 64;
        }
        wave_lds_order();
        // kD2Unroll groups of 64 words at a time: their LDS read chains
        // (start map -> index -> tag -> bytes) are independent and overlap
        uint32_t cum = 0;
        for (uint32_t gb = rb; gb < re; gb += 64 * kD2Unroll) {
          uint64_t bm[kD2Unroll];
#pragma unroll
          for (int u = 0; u < kD2Unroll; ++u) {
            const uint32_t g0 = gb + 64 * u;
            const uint32_t gi = (g0 - rb) >> 5;  // (even; past the round: zero bits)
            bm[u] = g0 < rb + kD2Round ? ((uint64_t)bits[gi] | ((uint64_t)bits[gi + 1] << 32)) : 0ull;
          }
          const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1);
#pragma unroll
          for (int u = 0; u < kD2Unroll; ++u) {
            const uint32_t g0 = gb + 64 * u;
            const uint32_t rec = ia + cum + (uint32_t)__builtin_popcountll(bm[u] & le);
            cum += (uint32_t)__builtin_popcountll(bm[u]);
            const uint32_t wv = g0 + (uint32_t)lane;
            const uint32_t inf = info[min(rec, kD2NI - 1)];
            const uint32_t q = e + (inf & 0xfffu);
            const uint32_t ofs = wv - (inf >> 12);
            const uint32_t tag = pkw[q];
            uint32_t x0 = 0, x1 = 0;
            // 64 words of zero runs (the mostly-zero batches this form takes)
            // have no bytes to read: the group skips the reads and the LUT
            // (round 6: config 4 decode -1.0 %)
            if (__ballot(tag != 0u)) {
              // the word's bytes: after the tag, or the literal run's ofs-th word
              const uint32_t src = q + 1 + ((tag == 0xffu && ofs) ? 1u + 8u * ofs : 0u);
              const uint64_t raw = read8<kAllIn>(pkw, src, lend, gp, glim, ph, e);
              const uint64_t sel = lut[tag];
              const uint32_t rl = (uint32_t)raw, rh = (uint32_t)(raw >> 32);
              x0 = __builtin_amdgcn_perm(rh, rl, (uint32_t)sel);
              x1 = __builtin_amdgcn_perm(rh, rl, (uint32_t)(sel >> 32));
            }
            // (nontemporal: plain stores wrote 5 % fewer bytes and took 1.7 % longer)
            if (wv < re) __builtin_nontemporal_store((uint64_t)x0 | ((uint64_t)x1 << 32), &dst_w[wv]);
          }
        }
        // the record covering the next round's first word
        const uint32_t ob = ib < (uint32_t)NRe ? (info[ib] >> 12) : 0xffffffffu;
        ia = ob == rb + kD2Round ? ib : ib - 1;
        wave_lds_order();  // bits / info reused
      }
      };
      if (eff_next + 12 <= lend) expand(std::true_type{});
      else
        expand(std::false_type{});
      WPH(6)
      if (ow + (int)Teff >= W && fin) {  // the piece is full: next piece starts at fin
        ow = W;
        e = fin;
        break;
      }
      ow += (int)Teff;
      e = eff_next;
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

// ---- decoder choice on the device (cpk_decode_batch, no host sync) --------
// Sparse batches (packed bytes under 15 % of the words' bytes: long zero
// runs) go to the record-index decoder, which measured 2.75 against 3.46 ms
// per 131,072 config-4 pieces; the others to the block-map decoder (4.5
// against 6.2 ms at config 2).  skip[0]: the block-map decoder's flag,
// skip[1]: the record-index decoder's.
// After a few large pieces were decoded as one stream (cpk_decode_batch):
// when every piece ended exactly at its packed range's end and decoded, the
// batch decoders are told to skip (both flags); else they run and give each
// piece its batch-form status.  One block; n <= 32.
__global__ void dec_stream_check_kernel(const uint64_t *__restrict__ found, const uint64_t *__restrict__ in_off,
                                        const int32_t *__restrict__ st, uint32_t n, uint32_t *skip) {
  const uint32_t i = threadIdx.x;
  const bool ok = i > n || (found[i] == in_off[i] - in_off[0] && (i == n || st[i] == CPK_OK));
  if (__syncthreads_and(ok) && i == 0) {
    skip[0] = 1u;
    skip[1] = 1u;
    skip[2] = 1u;
  }
}

__global__ void dec_gate_kernel(const uint64_t *__restrict__ in_off, const uint64_t *__restrict__ swo, uint32_t n,
                                uint32_t *skip) {
  if (threadIdx.x == 0) {
    const uint64_t P = in_off[n] - in_off[0], U = 8 * (swo[n] - swo[0]);
    // skip[0]: the block-map decoder, [1] the record-index one (sparse
    // batches), [2] the block-map decoder's dense form (serial walks of
    // windows of few long records: packed bytes >= 80 % of the words')
    const bool v2 = 100 * P < 15 * U, dense = 100 * P >= 80 * U;
    skip[0] = (v2 || dense) ? 1u : 0u;
    skip[1] = v2 ? 0u : 1u;
    skip[2] = dense ? 0u : 1u;
  }
}
