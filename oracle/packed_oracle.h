/*
 * packed_oracle.h -- CPU restatement of capnproto-java's packed codec.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under capnproto-java_amd/ links or
 * calls this file; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, as the checker and as the labelled "port"
 * CPU baseline.
 *
 * Parity is pinned by the reference's own known-answer tests
 * (runtime/src/test/java/org/capnproto/SerializePackedTest.java:20-60,
 * SerializeTest.java:90-140, :173-189), committed as data under
 * tests/golden/ and checked by tests/test_oracle.py.  The reference itself
 * (pure Java) cannot run in this image: there is no JDK.
 */
#ifndef CPK_PACKED_ORACLE_H
#define CPK_PACKED_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: the same values as include/capnp_packed.h. */
#define CPKO_OK 0
#define CPKO_EINVAL (-1)   /* misaligned length (PackedInputStream.java:40-42) */
#define CPKO_ETRUNC (-2)   /* input ended early (ArrayInputStream.java:53-58)  */
#define CPKO_EOVERRUN (-3) /* run past the end of the output (PackedInputStream.java:99-105, :110-114) */
#define CPKO_ETRAILING (-4) /* batch form only: bytes left after the piece filled */
#define CPKO_EFRAME (-7)   /* segment table invalid (Serialize.java:125-163) */

/* One PackedOutputStream.write() call (PackedOutputStream.java:35-205).
 * len must be a multiple of 8.  out must hold cpko_packed_bound(len/8)
 * bytes.  Returns the packed length. */
size_t cpko_pack(const uint8_t *in, size_t len, uint8_t *out);

/* Worst-case packed size of `words` words: 8w + 2*ceil(w/2). */
size_t cpko_packed_bound(size_t words);

/* One PackedInputStream.read() call over an ArrayInputStream holding
 * in[0..in_len) (PackedInputStream.java:35-140).  Fills out[0..out_len)
 * exactly; *consumed = input bytes used.  Returns a status code. */
int cpko_unpack(const uint8_t *in, size_t in_len, size_t *consumed,
                uint8_t *out, size_t out_len);

/* Batch helpers over n independent pieces (one write()/read() each).
 * seg_word_off[n+1]: word offsets of the pieces in `in`.
 * cpko_pack_batch writes out_off[n+1] (byte offsets into out) and returns
 * the total.  cpko_unpack_batch decodes piece i from
 * packed[in_off[i]..in_off[i+1]) into out + 8*seg_word_off[i] and writes
 * status[i] (ETRAILING if the piece filled before its range ended).
 * Both use `threads` POSIX threads (1 = the scalar reference loop). */
size_t cpko_pack_batch(const uint8_t *in, const uint64_t *seg_word_off,
                       uint32_t n, uint8_t *out, uint64_t *out_off,
                       int threads);
int cpko_unpack_batch(const uint8_t *packed, const uint64_t *in_off,
                      const uint64_t *seg_word_off, uint32_t n,
                      uint8_t *out, int32_t *status, int threads);

/* Serialize.write over a PackedOutputStream: pack(table) || pack(seg0) ...
 * (Serialize.java:256-307).  Returns bytes written to out. */
size_t cpko_write_message(const uint8_t *const *segs, const uint32_t *seg_words,
                          uint32_t nseg, uint8_t *out);

/* Serialize.read over a PackedInputStream (Serialize.java:119-178).
 * On success writes *nseg, seg_words[] (capacity max_seg) and the
 * concatenated segment words into out (capacity out_cap bytes) and
 * *consumed.  Returns a status code. */
int cpko_read_message(const uint8_t *in, size_t in_len, size_t *consumed,
                      uint32_t *nseg, uint32_t *seg_words, uint32_t max_seg,
                      uint8_t *out, size_t out_cap,
                      uint64_t traversal_limit_words);

/* Synthetic segment generator shared with the device generator in
 * capnproto-java_amd/csrc (bench + tests; not part of the reference).
 * PRNG core: benchmark/src/main/java/org/capnproto/benchmark/Common.java:25-38
 * (FastRand xorshift128, Java arithmetic >>).  Thresholds are out of 2^31:
 * every draw is non-negative (bit 31 is cleared by the arithmetic shifts). */
typedef struct {
  uint64_t t_zero0;  /* P(first word is in the zero state)   */
  uint64_t t_z2n;    /* P(zero -> nonzero) per word          */
  uint64_t t_n2z;    /* P(nonzero -> zero) per word          */
  uint64_t t_qbyte;  /* P(byte of a nonzero-state word is 0) */
  uint32_t cfg;      /* config id, part of the seed           */
  uint32_t pad;
} cpko_gen_params;

void cpko_generate(const cpko_gen_params *p, const uint64_t *seg_word_off,
                   uint32_t first_seg, uint32_t count, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
