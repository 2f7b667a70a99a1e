/*
 * capnp_packed.h -- C ABI of the MI355X (gfx950) packed-stream codec.
 *
 * Drop-in boundary for capnproto-java's packed encoding
 * (runtime/src/main/java/org/capnproto/PackedOutputStream.java:35-205,
 * PackedInputStream.java:35-140).  Plain pointers and sizes only; the JNI
 * glue in capnproto-java_amd/java/ binds exactly these entry points
 * (INTEGRATION.md).
 *
 * A "piece" is what one PackedOutputStream.write() / PackedInputStream.read()
 * call handles.  Serialize.write issues one write() per segment and one for
 * the segment table (Serialize.java:256-288), and each call starts from fresh
 * run state (PackedOutputStream.java:36-43), so a batch of pieces is encoded
 * and decoded independently, bit-exact with the reference.
 *
 * Threading: reentrant; a context may be used from one host thread at a time,
 * different contexts concurrently.  All *_batch calls are asynchronous on the
 * given stream (hipStream_t passed as void*; NULL = the device's null stream).
 * Calls on one context share its device workspace (counters, piece sizes,
 * step boundaries): issue them on one stream, or order the streams, so that
 * they do not run at the same time.
 */
#ifndef CAPNP_PACKED_H
#define CAPNP_PACKED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPK_ABI_VERSION 1

/* Status codes.  Decode errors are the reference's exceptions:
 *   CPK_EINVAL    piece length not a multiple of 8 -> DecodeException
 *                 ("PackedInputStream reads must be word-aligned",
 *                 PackedInputStream.java:40-42); bad arguments.
 *   CPK_ETRUNC    packed input ended before the piece was filled ->
 *                 DecodeException (ArrayInputStream.java:53-58,
 *                 PackedInputStream.java:93-95).  Also a literal run cut
 *                 short by end of input, which the reference may accept
 *                 silently through ArrayInputStream (documented divergence,
 *                 DESIGN.md).
 *   CPK_EOVERRUN  a 0x00/0xFF run runs past the end of the piece ->
 *                 DecodeException / BufferOverflowException
 *                 (PackedInputStream.java:99-105, :110-114).
 *   CPK_ETRAILING batch form only: the piece was filled before the end of
 *                 its packed byte range (the reference would leave the
 *                 bytes to the next read()).
 *   CPK_EFRAME    segment table invalid: count over 512, a negative size, a
 *                 message over the traversal limit or a segment over 2^28-1
 *                 words -> DecodeException (Serialize.java:45-53, :125-163).
 *   CPK_ENOMEM, CPK_EDEVICE  allocation / HIP runtime failure (-> IOException).
 *   CPK_EUNSUPPORTED  a piece outside what this build handles.
 */
#define CPK_OK 0
#define CPK_EINVAL (-1)
#define CPK_ETRUNC (-2)
#define CPK_EOVERRUN (-3)
#define CPK_ETRAILING (-4)
#define CPK_ENOMEM (-5)
#define CPK_EDEVICE (-6)
#define CPK_EFRAME (-7)
#define CPK_EUNSUPPORTED (-8)

typedef struct cpk_ctx_s *cpk_ctx;

int cpk_abi_version(void);
const char *cpk_status_string(int status);

/* Worst-case packed size of one piece of `words` words: 8w + 2*ceil(w/2).
 * (An isolated all-nonzero word costs 10 bytes) */
uint64_t cpk_packed_bound(uint64_t words);

/* Capacity, in bytes, the caller must allocate for the packed output of a
 * batch whose pieces have the given word counts: sum of the bounds plus 16
 * bytes of read slack (the decoder reads whole 16-byte lines). */
uint64_t cpk_batch_packed_capacity(const uint64_t *h_seg_word_off, uint32_t n);

/* Context bound to one HIP device.  Holds the look-back workspace. */
int cpk_ctx_create(int device, cpk_ctx *out);
void cpk_ctx_destroy(cpk_ctx ctx);
int cpk_ctx_device(cpk_ctx ctx);
/* Times a one-launch host path (small messages) found its kernel's pinned
 * completion flag unset even after the stream synchronisation it falls back
 * to when the flag has not turned within 5 ms (a late launch on a busy GPU
 * only takes that fallback and is not counted).  Zero in normal operation: a
 * count that grows means a lost completion flag (a device-side bug). */
uint64_t cpk_ctx_small_fallbacks(cpk_ctx ctx);
/* Diagnostics of the last batch / message decode on this context (synchronises
 * `stream`): windows the dense block-map form walked with one lane along the
 * true chain, and serial walks it gave back to the parallel walks (too many
 * records); both 0 when another decoder form took the batch.  Counted only by
 * the diagnostics build (libcapnp_packed_hip_diag.so: the counters cost the
 * dense forms ~2 %); the product library returns CPK_EUNSUPPORTED. */
int cpk_ctx_dense_windows(cpk_ctx ctx, void *stream, uint64_t *serial, uint64_t *given_back);

/* Batch encode of n pieces, device-resident (replaces n calls of
 * PackedOutputStream.write, PackedOutputStream.java:35-205).  Pieces of any
 * size.  The encoder is chosen on the device from the piece sizes (no host
 * sync): like-sized pieces of 4 Ki words or more (the largest at most twice
 * the smallest) take the single-pass encoder (read the words once, write the
 * packed bytes once, work ticketed per 8192-word chunk, offsets by a decoupled
 * look-back over the chunks; pieces over one chunk need max_seg_words), in
 * its sparse form (twice the workgroups per CU) when >= 85 % of a sample of
 * the words are zero; other batches the two-pass one (a size pass, a scan of
 * the sizes, an emit pass).
 *   d_in            : 8-byte aligned words; piece i is words
 *                     [d_seg_word_off[i], d_seg_word_off[i+1]).
 *   d_seg_word_off  : uint64[n+1], device.
 *   max_seg_words   : host bound on every piece's size in words, 0 = unknown
 *                     (the call then reads d_seg_word_off[0], [n] back,
 *                     synchronising `stream`).  A piece larger than a nonzero
 *                     bound is reported by cpk_ctx_take_error (output
 *                     undefined for that piece).
 *   d_out           : 16-byte aligned, capacity cpk_batch_packed_capacity().
 *   d_out_off       : uint64[n+1], device, written: piece i's packed bytes
 *                     are d_out[d_out_off[i] .. d_out_off[i+1]), contiguous
 *                     and in order, i.e. exactly the bytes the reference
 *                     writes for pieces 0..n-1 through one sink.
 * Returns CPK_OK or an error; asynchronous on `stream`. */
int cpk_encode_batch(cpk_ctx ctx, const void *d_in, const uint64_t *d_seg_word_off,
                     uint32_t n, uint64_t max_seg_words, void *d_out,
                     uint64_t *d_out_off, void *stream);

/* Batch of messages (Serialize.write through PackedOutputStream for each,
 * SerializePacked.write, Serialize.java:256-288): message m's segments are
 * pieces [d_msg_seg_off[m], d_msg_seg_off[m+1]) of d_in / d_seg_word_off
 * (nseg pieces in message order, d_msg_seg_off[0] = 0, [nm] = nseg); its segment table (count - 1, the sizes in
 * words, zero pad; :256-273) is built and packed on the device, so the
 * output holds, per message, packed(table) || packed(seg 0) || ... -- the
 * bytes SerializePacked.write produces, messages back to back.
 *   max_seg_words   : host bound on every segment's words (required, > 0;
 *                     a segment over it is reported by cpk_ctx_take_error).
 *   d_out           : 16-byte aligned, capacity cpk_batch_packed_capacity()
 *                     of the segments + 10 * ((count + 2) / 2 + 1) bytes per
 *                     message of `count` segments.
 *   d_out_off       : uint64[nm + nseg + 1], written: piece offsets in
 *                     message order (table, segments; next message); message
 *                     m starts at d_out_off[d_msg_seg_off[m] + m] and the
 *                     last entry is the total.
 * Asynchronous on `stream`. */
int cpk_encode_messages(cpk_ctx ctx, const void *d_in, const uint64_t *d_seg_word_off,
                        uint32_t nseg, const uint64_t *d_msg_seg_off, uint32_t nm,
                        uint64_t max_seg_words, void *d_out, uint64_t *d_out_off, void *stream);

/* The same two calls with the byte capacity of d_out (the reference's sink
 * refuses a write that does not fit: ArrayOutputStream.write throws
 * IOException, ArrayOutputStream.java:36-44).  A piece whose packed bytes
 * would pass out_cap is reported -- cpk_ctx_take_error returns CPK_ENOMEM --
 * and no byte at or past d_out + out_cap is ever stored; pieces wholly below
 * it are written as usual (the bytes of the piece that crosses it are
 * undefined).  cpk_encode_batch / cpk_encode_messages are these calls with
 * out_cap = UINT64_MAX: they trust the documented capacity. */
int cpk_encode_batch_cap(cpk_ctx ctx, const void *d_in, const uint64_t *d_seg_word_off,
                         uint32_t n, uint64_t max_seg_words, void *d_out, uint64_t out_cap,
                         uint64_t *d_out_off, void *stream);
int cpk_encode_messages_cap(cpk_ctx ctx, const void *d_in, const uint64_t *d_seg_word_off,
                            uint32_t nseg, const uint64_t *d_msg_seg_off, uint32_t nm,
                            uint64_t max_seg_words, void *d_out, uint64_t out_cap,
                            uint64_t *d_out_off, void *stream);

/* Synchronises `stream` and returns the first problem an encode issued since
 * the last call met (and clears it): CPK_ENOMEM if packed bytes would have
 * passed an out_cap (the *_cap forms), CPK_EINVAL if a piece was larger than
 * its max_seg_words bound, else CPK_OK.  The host forms below check it
 * themselves. */
int cpk_ctx_take_error(cpk_ctx ctx, void *stream);

/* Batch decode of n pieces, device-resident (replaces n calls of
 * PackedInputStream.read, PackedInputStream.java:35-140).
 *   d_packed        : packed bytes, readable up to round_up(d_in_off[n], 16).
 *   d_in_off        : uint64[n+1], device; piece i's packed bytes.
 *   d_seg_word_off  : uint64[n+1], device; piece i's unpacked words.
 *   d_out           : 8-byte aligned; piece i -> words d_seg_word_off[i]...
 *   d_status        : int32[n], device, written per piece (CPK_* codes).
 * Returns CPK_OK if launched; per-piece results are in d_status.  A batch of
 * at most 32 pieces reads its extent back (one sync of `stream`): with
 * >= 8 Mi words per piece on average it is decoded as one stream, 256-byte
 * blocks in parallel, the batch decoders running after it only when some
 * piece did not end exactly at its packed range's end. */
int cpk_decode_batch(cpk_ctx ctx, const void *d_packed, const uint64_t *d_in_off,
                     const uint64_t *d_seg_word_off, uint32_t n, void *d_out,
                     int32_t *d_status, void *stream);

/* Stream decode (Serialize.read over PackedInputStream, Serialize.java:
 * 165-175): pieces 0..n-1 are decoded back to back from one packed stream of
 * `avail` bytes; each piece's read() stops when the piece is full and leaves
 * the rest to the next (PackedInputStream.java:35-140), so no packed offsets
 * are needed.  d_in_off[n+1] is written with the piece boundaries found
 * (d_in_off[n] = bytes consumed).  A failed piece stops the stream: it and
 * every later piece get its status.  Asynchronous on `stream`. */
int cpk_decode_stream(cpk_ctx ctx, const void *d_packed, uint64_t avail,
                      const uint64_t *d_seg_word_off, uint32_t n, void *d_out,
                      uint64_t *d_in_off, int32_t *d_status, void *stream);

/* Batch of packed messages (Serialize.read over PackedInputStream for each,
 * SerializePacked.read, Serialize.java:119-178): message m is the packed
 * bytes [d_msg_off[m], d_msg_off[m+1]) -- its segment table (two read()
 * calls: the first word, then 4 * (count & ~1) bytes), validated, then its
 * segments back to back.  Segments of all messages are written contiguously
 * in message order:
 *   d_msg_seg_off   : uint64[nm+1], written: message m's segments are
 *                     [d_msg_seg_off[m], d_msg_seg_off[m+1]) (none when its
 *                     table failed).
 *   d_seg_word_off  : uint64[segments+1], written: segment words in d_out.
 *   d_seg_in_off    : uint64[segments], written: segment packed starts.
 *   d_seg_status    : int32[segments], written (a failed segment stops its
 *                     message: later segments carry its status).
 *   d_msg_status    : int32[nm], written: CPK_OK, the table's error
 *                     (CPK_EFRAME, CPK_ETRUNC, ...), the first failed
 *                     segment's, or CPK_ETRAILING if the message's bytes
 *                     outlast its segments.
 *   traversal_limit_words: ReaderOptions.traversalLimitInWords (reference
 *                     default 8 Mi words).
 *   h_totals[2]     : host, written: total words, total segments.
 * The call synchronises `stream` once (to read the totals) and returns
 * CPK_ENOMEM, without decoding, if they exceed out_cap_words / seg_cap.
 * d_packed readable up to round_up(d_msg_off[nm], 16). */
int cpk_decode_messages(cpk_ctx ctx, const void *d_packed, const uint64_t *d_msg_off, uint32_t nm,
                        uint64_t traversal_limit_words, void *d_out, uint64_t out_cap_words,
                        uint64_t *d_seg_word_off, uint64_t *d_seg_in_off, int32_t *d_seg_status,
                        uint32_t seg_cap, uint64_t *d_msg_seg_off, int32_t *d_msg_status,
                        uint64_t *h_totals, void *stream);

/* One message from the front of a packed byte stream whose length is not
 * known in advance (SerializePacked.read / readFromUnbuffered: Serialize.read
 * over PackedInputStream, Serialize.java:119-178), in one enqueue with no
 * host sync.  The device reads the segment table as the reference does (the
 * first word, then 4 * (count & ~1) bytes), validates it (count <= 512,
 * sizes >= 0, total <= traversal_limit_words, segments <= 2^28-1 words,
 * Serialize.java:45-53, :125-163) and decodes every segment back to back
 * from where the table ends.  Bytes after the message are left alone.
 *   d_packed : the stream's first `avail` bytes, 16-byte aligned, readable
 *              up to round_up(avail, 16).
 *   d_out    : 8-byte aligned, out_cap_words + CPK_MSG_HEAD_WORDS words: the
 *              table's words land first, segment i is words
 *              [d_info[4 + i], d_info[5 + i]).
 *   d_info   : uint64[CPK_MSG_INFO_WORDS], device, written: [0] status (as
 *              int64), [1] bytes consumed, [2] segment count, [3] total
 *              segment words, [4 .. 4 + count] segment word offsets.
 * Status: CPK_OK; CPK_ETRUNC when the bytes end inside the message (a
 * channel reader takes more and calls again); CPK_EFRAME / CPK_EOVERRUN as
 * Serialize.read would throw; CPK_ENOMEM when the segments exceed
 * out_cap_words (nothing decoded; [2] and [3] say how many).  Only
 * min(avail, 10 * (out_cap_words + CPK_MSG_HEAD_WORDS) + 16) bytes are read. */
#define CPK_MSG_HEAD_WORDS 257
#define CPK_MSG_INFO_WORDS 517
int cpk_read_message(cpk_ctx ctx, const void *d_packed, uint64_t avail, uint64_t traversal_limit_words,
                     void *d_out, uint64_t out_cap_words, uint64_t *d_info, void *stream);

/* Host-memory convenience forms (the socket/file ByteBuffer path,
 * SerializePacked.java:75-96, :119-134).  Synchronous.  encode_host and
 * decode_host pipeline the batch in chunks of whole pieces through pinned
 * staging kept in the context (CPK_HOST_CHUNK_MB, default 256;
 * CPK_HOST_THREADS copy threads, default 8); decode_stream_host and
 * read_message_host stage only the bytes the pieces can reach (10 per word
 * at most), the rest of `avail` may be later messages.
 *   cpk_read_message_host: cpk_read_message over host memory; h_out gets the
 *                    segments only, back to back (out_cap_words words), and
 *                    h_info[4 + i] their word offsets from 0.  Two syncs (the
 *                    info row, then the words).
 *   cpk_encode_host: h_out capacity >= cpk_batch_packed_capacity();
 *                    h_out_off[n+1] written.
 *   cpk_decode_host: h_status[n] written; returns CPK_OK iff all pieces OK. */
int cpk_encode_host(cpk_ctx ctx, const void *h_in, const uint64_t *h_seg_word_off,
                    uint32_t n, void *h_out, uint64_t h_out_cap, uint64_t *h_out_off);
/* Gather form of cpk_encode_host (builder segments in
 * their own direct ByteBuffers, DefaultAllocator.java:56-62, packed without a
 * host-side concatenation): piece i is the h_swo[i+1] - h_swo[i] words at
 * h_pieces[i] (any host pointer, no alignment needed; NULL only for an empty
 * piece); h_swo is read only for the sizes.  Output as cpk_encode_host. */
int cpk_encode_host_gather(cpk_ctx ctx, const void *const *h_pieces, const uint64_t *h_swo,
                           uint32_t n, void *h_out, uint64_t h_out_cap, uint64_t *h_out_off);
int cpk_decode_host(cpk_ctx ctx, const void *h_packed, const uint64_t *h_in_off,
                    const uint64_t *h_seg_word_off, uint32_t n, void *h_out,
                    int32_t *h_status);
int cpk_decode_stream_host(cpk_ctx ctx, const void *h_packed, uint64_t avail,
                           const uint64_t *h_seg_word_off, uint32_t n, void *h_out,
                           uint64_t *h_in_off, int32_t *h_status);
int cpk_read_message_host(cpk_ctx ctx, const void *h_packed, uint64_t avail, uint64_t traversal_limit_words,
                          void *h_out, uint64_t out_cap_words, uint64_t *h_info);

/* Host-memory forms of the message batches (staged whole through device
 * memory; synchronous).
 *   cpk_encode_messages_host: h_msg_seg_off[0] = 0, [nm] = nseg; h_out
 *     capacity as cpk_encode_messages; h_out_off[nm + nseg + 1] written.
 *   cpk_decode_messages_host: h_msg_seg_off[nm+1], h_msg_status[nm],
 *     h_seg_word_off[segments+1] (segment words in h_out) and h_totals[2]
 *     written; CPK_ENOMEM (with the totals) if out_cap_words / seg_cap are
 *     too small -- call with 0 / NULL first to size them; otherwise returns
 *     the first failed message's status or CPK_OK. */
int cpk_encode_messages_host(cpk_ctx ctx, const void *h_in, const uint64_t *h_seg_word_off,
                             uint32_t nseg, const uint64_t *h_msg_seg_off, uint32_t nm,
                             void *h_out, uint64_t h_out_cap, uint64_t *h_out_off);
/* Gather form of cpk_encode_messages_host: segment i is the
 * h_swo[i+1] - h_swo[i] words at h_segs[i] (any host pointer; NULL only for
 * an empty segment), e.g. each MessageBuilder's own segment buffers
 * (BuilderArena.getSegmentsForOutput, BuilderArena.java:143-154).  Output as
 * cpk_encode_messages_host. */
int cpk_encode_messages_host_gather(cpk_ctx ctx, const void *const *h_segs, const uint64_t *h_swo,
                                    uint32_t nseg, const uint64_t *h_msg_seg_off, uint32_t nm,
                                    void *h_out, uint64_t h_out_cap, uint64_t *h_out_off);
int cpk_decode_messages_host(cpk_ctx ctx, const void *h_packed, const uint64_t *h_msg_off,
                             uint32_t nm, uint64_t traversal_limit_words, void *h_out,
                             uint64_t out_cap_words, uint64_t *h_seg_word_off, uint32_t seg_cap,
                             uint64_t *h_msg_seg_off, int32_t *h_msg_status, uint64_t *h_totals);

/* ---- benchmark support (synthetic device-resident workloads) ---- */

/* Device generator of the synthetic segments described in SURVEY.md 8d:
 * a 2-state Markov chain over words (thresholds out of 2^31: FastRand draws
 * are never negative), seeded per
 * segment from (cfg, segment index).  Identical stream to the host copy in
 * oracle/packed_oracle.c:cpko_generate. */
typedef struct {
  uint64_t t_zero0, t_z2n, t_n2z, t_qbyte;
  uint32_t cfg, pad;
} cpk_gen_params;

int cpk_generate(cpk_ctx ctx, const cpk_gen_params *params, const uint64_t *d_seg_word_off,
                 uint32_t n, void *d_out, void *stream);

/* Counts 8-byte words that differ between two device buffers into
 * *d_mismatch (uint64, device, accumulated; zero it first). */
int cpk_count_mismatch(cpk_ctx ctx, const void *d_a, const void *d_b, uint64_t words,
                       uint64_t *d_mismatch, void *stream);

#ifdef __cplusplus
}
#endif
#endif
