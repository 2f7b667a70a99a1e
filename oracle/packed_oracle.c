/*
 * packed_oracle.c -- CPU restatement of capnproto-java's packed codec.
 *
 * TEST INFRASTRUCTURE ONLY (see packed_oracle.h).  Each function cites the
 * reference lines it restates; paths are relative to the reference root.
 * Parity pinned by SerializePackedTest.java:20-60 and SerializeTest.java
 * vectors (tests/golden/, tests/test_oracle.py).
 */
#include "packed_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t load64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

size_t cpko_packed_bound(size_t words) { return 8 * words + 2 * ((words + 1) / 2); }

/* PackedOutputStream.write(ByteBuffer), runtime/src/main/java/org/capnproto/
 * PackedOutputStream.java:35-205.  The 20-byte slowBuffer path (:44-59,
 * :197-201) and the direct inner.write of long literal runs (:172-193)
 * only change how bytes reach the sink, never which bytes: the sink here
 * is a buffer with room for the worst case, so the fast path is taken. */
size_t cpko_pack(const uint8_t *in, size_t len, uint8_t *out) {
  size_t inPtr = 0, o = 0;
  const size_t inEnd = len;                      /* :36, :42 */
  while (inPtr < inEnd) {                        /* :43 */
    size_t tagPos = o++;                         /* :61-62 */
    uint8_t tag = 0;
    for (int i = 0; i < 8; ++i) {                /* :66-112, byte by byte */
      uint8_t b = in[inPtr++];
      if (b != 0) {
        out[o++] = b;
        tag |= (uint8_t)(1u << i);
      }
    }
    out[tagPos] = tag;                           /* :114-117 */
    if (tag == 0) {                              /* :119-131 zero run */
      size_t runStart = inPtr, limit = inEnd;
      if (limit - inPtr > 255 * 8) limit = inPtr + 255 * 8;
      while (inPtr < limit && load64(in + inPtr) == 0) inPtr += 8;
      out[o++] = (uint8_t)((inPtr - runStart) / 8);
    } else if (tag == 0xff) {                    /* :133-193 literal run */
      size_t runStart = inPtr, limit = inEnd;
      if (limit - inPtr > 255 * 8) limit = inPtr + 255 * 8;
      while (inPtr < limit) {                    /* :149-161 */
        int c = 0;
        for (int ii = 0; ii < 8; ++ii) c += (in[inPtr++] == 0);
        if (c >= 2) {                            /* :155-159 */
          inPtr -= 8;
          break;
        }
      }
      size_t count = inPtr - runStart;           /* :163-164 */
      out[o++] = (uint8_t)(count / 8);
      memcpy(out + o, in + runStart, count);     /* :166-171 */
      o += count;
    }
  }
  return o;                                      /* :203-204 (returns length) */
}

/* PackedInputStream.read(ByteBuffer) over an ArrayInputStream,
 * runtime/src/main/java/org/capnproto/PackedInputStream.java:35-140 and
 * ArrayInputStream.java:35-59.  The fast (:82-90) and slow (:53-81) tag
 * paths produce the same bytes; the slow path's per-byte refill is where
 * an exhausted ArrayInputStream throws DecodeException (:53-58) -> ETRUNC.
 * Exceptions map to status codes; the one documented divergence: a literal
 * run truncated by end of input is ETRUNC here, while the reference can
 * accept it silently (PackedInputStream.java:116-129 ignores read()'s -1). */
int cpko_unpack(const uint8_t *in, size_t in_len, size_t *consumed,
                uint8_t *out, size_t out_len) {
  size_t ip = 0, op = 0;
  if (consumed) *consumed = 0;
  if (out_len == 0) return CPKO_OK;              /* :37-38 */
  if (out_len % 8 != 0) return CPKO_EINVAL;      /* :40-42 */
  for (;;) {
    if (ip >= in_len) return CPKO_ETRUNC;        /* getReadBuffer() at EOF */
    uint8_t tag = in[ip++];
    for (int i = 0; i < 8; ++i) {                /* :68-77 / :85-89 */
      if (tag & (1u << i)) {
        if (ip >= in_len) return CPKO_ETRUNC;
        out[op++] = in[ip++];
      } else {
        out[op++] = 0;
      }
    }
    if (tag == 0) {                              /* :92-105 */
      if (ip >= in_len) return CPKO_ETRUNC;      /* :79-80 refill, :93-95 */
      size_t run = (size_t)in[ip++] * 8;
      /* :99 compares against the whole request (outPtr is never advanced);
       * :103-105 then overflow the buffer.  Either way: an exception. */
      if (run > out_len - op) return CPKO_EOVERRUN;
      memset(out + op, 0, run);
      op += run;
    } else if (tag == 0xff) {                    /* :106-134 */
      if (ip >= in_len) return CPKO_ETRUNC;
      size_t run = (size_t)in[ip++] * 8;
      if (run > out_len - op) return CPKO_EOVERRUN; /* BufferOverflowException */
      if (in_len - ip < run) return CPKO_ETRUNC;    /* documented divergence */
      memcpy(out + op, in + ip, run);
      ip += run;
      op += run;
    }
    if (op == out_len) {                         /* :136-138 */
      if (consumed) *consumed = ip;
      return CPKO_OK;
    }
  }
}

/* ---- batch helpers (independent pieces; Serialize.java:283-287 issues one
 * write() per segment, so pieces never share run state) ---- */

typedef struct {
  const uint8_t *in;
  const uint64_t *seg_word_off;
  uint8_t *out;
  const uint64_t *off;   /* in: packed offsets (unpack) */
  uint64_t *sizes;       /* out: packed sizes (pack)   */
  int32_t *status;
  uint32_t begin, end;
  uint8_t *scratch;
} cpko_job;

static void *pack_worker(void *arg) {
  cpko_job *j = (cpko_job *)arg;
  for (uint32_t i = j->begin; i < j->end; ++i) {
    uint64_t w0 = j->seg_word_off[i], w1 = j->seg_word_off[i + 1];
    j->sizes[i] = cpko_pack(j->in + 8 * w0, 8 * (w1 - w0), j->scratch);
  }
  return NULL;
}

static void *pack_emit_worker(void *arg) {
  cpko_job *j = (cpko_job *)arg;
  for (uint32_t i = j->begin; i < j->end; ++i) {
    uint64_t w0 = j->seg_word_off[i], w1 = j->seg_word_off[i + 1];
    cpko_pack(j->in + 8 * w0, 8 * (w1 - w0), j->out + j->off[i]);
  }
  return NULL;
}

static void *unpack_worker(void *arg) {
  cpko_job *j = (cpko_job *)arg;
  for (uint32_t i = j->begin; i < j->end; ++i) {
    uint64_t w0 = j->seg_word_off[i], w1 = j->seg_word_off[i + 1];
    size_t used = 0;
    size_t in_len = (size_t)(j->off[i + 1] - j->off[i]);
    int st = cpko_unpack(j->in + j->off[i], in_len, &used, j->out + 8 * w0,
                         8 * (w1 - w0));
    if (st == CPKO_OK && used != in_len) st = CPKO_ETRAILING;
    j->status[i] = st;
  }
  return NULL;
}

static void run_jobs(void *(*fn)(void *), cpko_job *proto, uint32_t n,
                     int threads) {
  if (threads < 1) threads = 1;
  if ((uint32_t)threads > n) threads = n ? (int)n : 1;
  cpko_job *jobs = (cpko_job *)calloc((size_t)threads, sizeof(cpko_job));
  pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t] = *proto;
    jobs[t].begin = (uint32_t)((uint64_t)n * t / threads);
    jobs[t].end = (uint32_t)((uint64_t)n * (t + 1) / threads);
  }
  if (threads == 1) {
    fn(&jobs[0]);
  } else {
    for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  }
  free(jobs);
  free(tid);
}

size_t cpko_pack_batch(const uint8_t *in, const uint64_t *seg_word_off,
                       uint32_t n, uint8_t *out, uint64_t *out_off,
                       int threads) {
  /* Pass 1 sizes (parallel), exclusive scan, pass 2 emit (parallel). */
  uint64_t *sizes = (uint64_t *)calloc((size_t)n + 1, sizeof(uint64_t));
  uint64_t maxw = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t w = seg_word_off[i + 1] - seg_word_off[i];
    if (w > maxw) maxw = w;
  }
  int nt = threads < 1 ? 1 : threads;
  uint8_t **scratch = (uint8_t **)calloc((size_t)nt, sizeof(uint8_t *));
  cpko_job proto;
  memset(&proto, 0, sizeof proto);
  proto.in = in;
  proto.seg_word_off = seg_word_off;
  proto.sizes = sizes;
  if (nt == 1) {
    /* scalar form: emit straight into out, exactly like one sink */
    uint64_t o = 0;
    for (uint32_t i = 0; i < n; ++i) {
      out_off[i] = o;
      uint64_t w0 = seg_word_off[i], w1 = seg_word_off[i + 1];
      o += cpko_pack(in + 8 * w0, 8 * (w1 - w0), out + o);
    }
    out_off[n] = o;
    free(sizes);
    free(scratch);
    return (size_t)o;
  }
  /* threaded: per-thread scratch for the sizing pass */
  {
    if ((uint32_t)nt > n) nt = n ? (int)n : 1;
    cpko_job *jobs = (cpko_job *)calloc((size_t)nt, sizeof(cpko_job));
    pthread_t *tid = (pthread_t *)calloc((size_t)nt, sizeof(pthread_t));
    for (int t = 0; t < nt; ++t) {
      jobs[t] = proto;
      jobs[t].begin = (uint32_t)((uint64_t)n * t / nt);
      jobs[t].end = (uint32_t)((uint64_t)n * (t + 1) / nt);
      scratch[t] = (uint8_t *)malloc(cpko_packed_bound(maxw) + 16);
      jobs[t].scratch = scratch[t];
      pthread_create(&tid[t], NULL, pack_worker, &jobs[t]);
    }
    for (int t = 0; t < nt; ++t) {
      pthread_join(tid[t], NULL);
      free(scratch[t]);
    }
    free(jobs);
    free(tid);
  }
  uint64_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    out_off[i] = o;
    o += sizes[i];
  }
  out_off[n] = o;
  proto.out = out;
  proto.off = out_off;
  run_jobs(pack_emit_worker, &proto, n, nt);
  free(sizes);
  free(scratch);
  return (size_t)o;
}

int cpko_unpack_batch(const uint8_t *packed, const uint64_t *in_off,
                      const uint64_t *seg_word_off, uint32_t n,
                      uint8_t *out, int32_t *status, int threads) {
  cpko_job proto;
  memset(&proto, 0, sizeof proto);
  proto.in = packed;
  proto.off = in_off;
  proto.seg_word_off = seg_word_off;
  proto.out = out;
  proto.status = status;
  run_jobs(unpack_worker, &proto, n, threads);
  int bad = 0;
  for (uint32_t i = 0; i < n; ++i) bad += status[i] != CPKO_OK;
  return bad ? CPKO_ETRUNC : CPKO_OK;
}

/* Serialize.writeSegmentTable + Serialize.write (Serialize.java:256-288)
 * through PackedOutputStream: the table is one write() call, then one per
 * segment. */
size_t cpko_write_message(const uint8_t *const *segs, const uint32_t *seg_words,
                          uint32_t nseg, uint8_t *out) {
  size_t tableWords = ((size_t)nseg + 2) & ~(size_t)1;   /* :258 (in ints) */
  uint8_t *table = (uint8_t *)calloc(tableWords, 4);
  uint32_t v = nseg - 1;
  memcpy(table, &v, 4);                                  /* :263 */
  for (uint32_t i = 0; i < nseg; ++i) memcpy(table + 4 * (i + 1), &seg_words[i], 4);
  size_t o = cpko_pack(table, tableWords * 4, out);
  free(table);
  for (uint32_t i = 0; i < nseg; ++i)                    /* :283-287 */
    o += cpko_pack(segs[i], 8 * (size_t)seg_words[i], out + o);
  return o;
}

/* Serialize.read / doRead over PackedInputStream(ArrayInputStream),
 * Serialize.java:119-178: first word, validation, rest of table, then one
 * fillBuffer per segment.  Each fillBuffer is one PackedInputStream.read. */
int cpko_read_message(const uint8_t *in, size_t in_len, size_t *consumed,
                      uint32_t *nseg, uint32_t *seg_words, uint32_t max_seg,
                      uint8_t *out, size_t out_cap,
                      uint64_t traversal_limit_words) {
  size_t ip = 0, used = 0;
  uint8_t first[8];
  int st = cpko_unpack(in, in_len, &used, first, 8);     /* :120-121 */
  if (st) return st;
  ip += used;
  int32_t raw;
  memcpy(&raw, first, 4);
  if (raw < 0 || raw > 511) return CPKO_EFRAME;          /* :128-131 */
  uint32_t count = (uint32_t)raw + 1;
  int32_t s0;
  memcpy(&s0, first + 4, 4);
  if (s0 < 0) return CPKO_EFRAME;                        /* :135-137 */
  if (count > max_seg) return CPKO_EINVAL;
  seg_words[0] = (uint32_t)s0;
  uint64_t total = (uint64_t)s0;
  if (count > 1) {                                       /* :144-157 */
    size_t rest = 4 * (size_t)(count & ~1u);
    uint8_t *raw_sizes = (uint8_t *)malloc(rest);
    st = cpko_unpack(in + ip, in_len - ip, &used, raw_sizes, rest);
    if (st) {
      free(raw_sizes);
      return st;
    }
    ip += used;
    for (uint32_t i = 0; i + 1 < count; ++i) {
      int32_t s;
      memcpy(&s, raw_sizes + 4 * i, 4);
      if (s < 0) {
        free(raw_sizes);
        return CPKO_EFRAME;
      }
      seg_words[i + 1] = (uint32_t)s;
      total += (uint64_t)s;
    }
    free(raw_sizes);
  }
  if (total > traversal_limit_words) return CPKO_EFRAME; /* :160-162 */
  if (8 * total > out_cap) return CPKO_EINVAL;
  size_t op = 0;
  for (uint32_t i = 0; i < count; ++i) {                 /* :165-175 */
    if (seg_words[i] > 0x0fffffffu) return CPKO_EFRAME;  /* makeByteBufferForWords, :45-53 */
    size_t bytes = 8 * (size_t)seg_words[i];
    st = cpko_unpack(in + ip, in_len - ip, &used, out + op, bytes);
    if (st) return st;
    ip += used;
    op += bytes;
  }
  *nseg = count;
  if (consumed) *consumed = ip;
  return CPKO_OK;
}

/* ---- synthetic generator ---- */

typedef struct {
  int32_t x, y, z, w;
} fastrand;

/* Common.FastRand.nextInt (benchmark/.../Common.java:31-38); the shifts
 * right are Java's arithmetic >> on int. */
static inline uint32_t fr_next(fastrand *r) {
  uint32_t ux = (uint32_t)r->x;
  uint32_t tmp = ux ^ (ux << 11);
  r->x = r->y;
  r->y = r->z;
  r->z = r->w;
  uint32_t w = (uint32_t)r->w;
  w = w ^ (uint32_t)(r->w >> 19) ^ tmp ^ (uint32_t)((int32_t)tmp >> 8);
  r->w = (int32_t)w;
  return w;
}

static inline uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static void seed_segment(fastrand *r, uint32_t cfg, uint64_t seg) {
  uint64_t s = 0x1d2acd47ULL ^ ((uint64_t)cfg << 40) ^ (seg * 0xD1B54A32D192ED03ULL);
  uint64_t a = splitmix64(&s), b = splitmix64(&s);
  r->x = (int32_t)(uint32_t)a;
  r->y = (int32_t)(uint32_t)(a >> 32);
  r->z = (int32_t)(uint32_t)b;
  r->w = (int32_t)(uint32_t)(b >> 32);
  if ((r->x | r->y | r->z | r->w) == 0) r->w = 1;
}

void cpko_generate(const cpko_gen_params *p, const uint64_t *seg_word_off,
                   uint32_t first_seg, uint32_t count, uint8_t *out) {
  uint64_t base = seg_word_off[first_seg];
  for (uint32_t s = first_seg; s < first_seg + count; ++s) {
    fastrand r;
    seed_segment(&r, p->cfg, s);
    uint64_t w0 = seg_word_off[s], w1 = seg_word_off[s + 1];
    uint8_t *dst = out + 8 * (w0 - base);
    int zero = (uint64_t)fr_next(&r) < p->t_zero0;
    for (uint64_t k = 0; k < w1 - w0; ++k) {
      if (k) {
        uint32_t t = fr_next(&r);
        if (zero) zero = !((uint64_t)t < p->t_z2n);
        else zero = (uint64_t)t < p->t_n2z;
      }
      if (zero) {
        memset(dst + 8 * k, 0, 8);
      } else {
        for (int b = 0; b < 8; ++b) {
          uint32_t t = fr_next(&r);
          dst[8 * k + b] = ((uint64_t)t < p->t_qbyte) ? 0 : (uint8_t)(1 + (t >> 8) % 255);
        }
      }
    }
  }
}
