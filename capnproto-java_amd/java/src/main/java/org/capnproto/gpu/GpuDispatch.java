// The hook every public SerializePacked method takes when the MI355X codec is
// enabled (integration/capnproto-java.patch adds one dispatch line to each of
// runtime/src/main/java/org/capnproto/SerializePacked.java:35-134).
//
// Enabled by -Dorg.capnproto.gpu=true or CAPNP_GPU=1 (device: CAPNP_GPU_DEVICE,
// default 0).  Output bytes and exceptions are the reference's: a write packs
// the segment table and segments on the device (Serialize.java:256-288); a
// read runs Serialize.read's sequence (Serialize.java:119-178) on the device
// in one library call (cpk_read_message_host).
//
// Size thresholds: a message of fewer than MIN_WRITE_BYTES (written) or
// MIN_READ_BYTES (read) unpacked bytes (table + segments) stays on the
// reference's own PackedOutputStream / PackedInputStream -- a GPU call costs
// ~20-50 microseconds of launch and PCIe latency, which only pays above the
// crossovers measured in INTEGRATION.md.  -Dorg.capnproto.gpu.minWriteBytes
// / minReadBytes (CAPNP_GPU_MIN_WRITE_BYTES / CAPNP_GPU_MIN_READ_BYTES) move
// one, -Dorg.capnproto.gpu.minBytes (CAPNP_GPU_MIN_BYTES) both; 0 sends every
// message to the GPU.  For a read the size comes from the message's segment
// table, peeked (not consumed) from the bytes the stream has buffered.
//
// Streams: a GPU read consumes exactly the bytes the reference's
// PackedInputStream would -- up to the end of the record that completes the
// message's last word (PackedInputStream.java:47-59, :84-88).  The message's
// packed extent is found on the host by walking record headers only
// (tag, count, literal-run skip; no bytes are expanded), buffer by buffer:
// every upstream read buffer the message fills completely is taken, the last
// one is advanced only by the bytes the message used, so the stream can go
// on being read by anything (Serialize.read, a direct read, the GPU).
// Channels (readFromUnbuffered) get one persistent Source each, so, unlike
// the reference's per-call 8 KiB wrapper (SerializePacked.java:92-96), no
// bytes past a message are dropped.  No lock is held across a blocking read:
// the only shared state is the weak map of channel Sources, locked for
// lookups.
package org.capnproto.gpu;

import java.io.IOException;
import java.lang.ref.WeakReference;
import java.nio.ByteBuffer;
import java.nio.channels.ReadableByteChannel;
import java.nio.channels.WritableByteChannel;
import java.util.Collections;
import java.util.Map;
import java.util.Optional;
import java.util.WeakHashMap;

public final class GpuDispatch {
    private GpuDispatch() {}

    private static final boolean ENABLED =
        Boolean.getBoolean("org.capnproto.gpu") || "1".equals(System.getenv("CAPNP_GPU"));

    /** Messages below these many unpacked bytes take the reference's CPU
     *  codec (defaults: the write and read crossovers of the multi-segment
     *  passByBytes replay, INTEGRATION.md, tests/cpp/pass_by_bytes.cpp). */
    public static final long DEFAULT_MIN_WRITE_BYTES = 1L << 20;
    public static final long DEFAULT_MIN_READ_BYTES = 2L << 20;
    public static final long MIN_WRITE_BYTES =
        threshold("minWriteBytes", "CAPNP_GPU_MIN_WRITE_BYTES", DEFAULT_MIN_WRITE_BYTES);
    public static final long MIN_READ_BYTES =
        threshold("minReadBytes", "CAPNP_GPU_MIN_READ_BYTES", DEFAULT_MIN_READ_BYTES);

    private static long threshold(String prop, String env, long dflt) {
        String v = System.getProperty("org.capnproto.gpu." + prop);
        if (v == null) v = System.getenv(env);
        if (v == null) v = System.getProperty("org.capnproto.gpu.minBytes");  // (both at once)
        if (v == null) v = System.getenv("CAPNP_GPU_MIN_BYTES");
        return v == null ? dflt : Long.parseLong(v.trim());
    }

    /** One context per process, created on first use (the library loads then). */
    private static final class Holder {
        static final PackedGpu GPU =
            new PackedGpu(Integer.parseInt(System.getenv().getOrDefault("CAPNP_GPU_DEVICE", "0")));
    }

    public static boolean enabled() { return ENABLED; }

    public static PackedGpu gpu() { return Holder.GPU; }

    /** Unpacked bytes of a message: its segment table (Serialize.java:258)
     *  plus its segments. */
    static long messageBytes(ByteBuffer[] segments) {
        long b = 4L * ((segments.length + 2) & ~1);
        for (ByteBuffer s : segments) b += s.remaining();
        return b;
    }

    // ------------------------------------------------------------------ write

    /** SerializePacked.write(output, message) for a message of `segments`
     *  (MessageBuilder.getSegmentsForOutput, BuilderArena.java:143-154, or a
     *  MessageReader's segments, Serialize.java:293-299).  Returns false,
     *  having written nothing, for a message below MIN_WRITE_BYTES: the caller then
     *  runs the reference's PackedOutputStream. */
    public static boolean write(org.capnproto.BufferedOutputStream output, ByteBuffer[] segments)
            throws IOException {
        if (messageBytes(segments) < MIN_WRITE_BYTES) return false;
        ByteBuffer bytes = packed(segments);
        while (bytes.hasRemaining()) output.write(bytes);
        return true;
    }

    /** SerializePacked.writeToUnbuffered(channel, message): the packed bytes
     *  straight to the channel -- the bytes the reference's 8 KiB
     *  BufferedOutputStreamWrapper + flush put there (SerializePacked.java:
     *  119-134).  False, nothing written, below MIN_WRITE_BYTES. */
    public static boolean writeToUnbuffered(WritableByteChannel output, ByteBuffer[] segments)
            throws IOException {
        if (messageBytes(segments) < MIN_WRITE_BYTES) return false;
        ByteBuffer bytes = packed(segments);
        while (bytes.hasRemaining()) output.write(bytes);
        return true;
    }

    private static ByteBuffer packed(ByteBuffer[] segments) throws IOException {
        PackedGpu.Packed p = gpu().encodeMessages(new ByteBuffer[][] {segments});
        ByteBuffer bytes = p.bytes.duplicate();
        bytes.position(0);
        return bytes;
    }

    // ------------------------------------------------------------------- read

    private static final Map<Object, Source> SOURCES = Collections.synchronizedMap(new WeakHashMap<>());

    /** The persistent buffered stream of a channel (readFromUnbuffered /
     *  tryReadFromUnbuffered read through it, GPU or reference path). */
    public static org.capnproto.BufferedInputStream stream(ReadableByteChannel channel) {
        synchronized (SOURCES) {
            Source s = SOURCES.get(channel);
            if (s == null) SOURCES.put(channel, s = new Source(channel));
            return s;
        }
    }

    /** SerializePacked.read(input, options): the message, read on the GPU;
     *  null when it is below MIN_READ_BYTES (or its table is not yet buffered) --
     *  nothing consumed, the caller runs the reference path over input. */
    public static org.capnproto.MessageReader read(org.capnproto.BufferedInputStream input,
                                                   org.capnproto.ReaderOptions options) throws IOException {
        // (getReadBuffer: DecodeException at the end of the stream, as the
        //  reference's first read throws)
        ByteBuffer head = input.getReadBuffer();
        if (!head.hasRemaining()) throw new org.capnproto.DecodeException("premature EOF");
        long bytes = peekMessageBytes(head);
        if (bytes < 0 || bytes < MIN_READ_BYTES) return null;
        long words = bytes / 8;
        if (input instanceof org.capnproto.ArrayInputStream) {
            // the whole array is the read buffer (ArrayInputStream.java:53-58)
            ByteBuffer[] segs = gpu().readMessage(head, options.traversalLimitInWords, words);
            if (segs == null) throw new org.capnproto.DecodeException("Premature EOF");
            return new org.capnproto.MessageReader(segs, options);
        }
        if (input instanceof Source) return readFrom((Source) input, options, words);
        return readFromStream(input, options, words);
    }

    /** SerializePacked.tryRead(input, options): Optional.empty() when the
     *  stream ends before a message starts (the documented contract,
     *  SerializePacked.java:31-46); null when the message is below MIN_READ_BYTES
     *  (the caller then runs the reference path over input). */
    public static Optional<org.capnproto.MessageReader> tryRead(org.capnproto.BufferedInputStream input,
                                                                org.capnproto.ReaderOptions options)
            throws IOException {
        ByteBuffer head;
        try {
            head = input.getReadBuffer();
        } catch (org.capnproto.DecodeException eof) {
            return Optional.empty();
        }
        if (!head.hasRemaining()) return Optional.empty();
        org.capnproto.MessageReader m = read(input, options);
        return m == null ? null : Optional.of(m);
    }

    /** GPU read of one message from a BufferedInputStream, consuming exactly
     *  its packed bytes: each read buffer is copied (not consumed) behind the
     *  message's earlier bytes and walked for the message's end (Extent);
     *  a buffer the message runs past is then taken whole and the next one
     *  fetched (getReadBuffer refills -- DecodeException at the end of the
     *  stream, as the reference's read()), the one it ends in is advanced by
     *  the bytes it used.  One library call per message.  A malformed
     *  message (a run past its words) goes to the device as far as it was
     *  walked, which throws the reference's DecodeException. */
    private static org.capnproto.MessageReader readFromStream(org.capnproto.BufferedInputStream input,
                                                              org.capnproto.ReaderOptions options,
                                                              long words) throws IOException {
        Extent ext = new Extent(words);
        ByteBuffer carry = PackedGpu.directBuffer(1 << 16);
        carry.limit(0);
        for (;;) {
            ByteBuffer cur = input.getReadBuffer();
            if (!cur.hasRemaining()) throw new org.capnproto.DecodeException("premature EOF");
            int base = carry.limit();
            carry = append(carry, cur);
            long end = ext.walk(carry);
            if (end == Extent.MORE) {
                cur.position(cur.limit());   // (all of it is the message's)
                continue;
            }
            int take = end >= 0 ? (int) end : carry.limit();
            ByteBuffer msg = carry.duplicate();
            msg.position(0).limit(take);
            ByteBuffer[] segs = gpu().readMessage(msg, options.traversalLimitInWords, words);
            if (segs == null) throw new org.capnproto.DecodeException("premature EOF");
            cur.position(cur.position() + (msg.position() - base));
            return new org.capnproto.MessageReader(segs, options);
        }
    }

    /** carry + src's remaining bytes (src not consumed), growing by doubling. */
    private static ByteBuffer append(ByteBuffer carry, ByteBuffer src) {
        int need = carry.limit() + src.remaining();
        if (need > carry.capacity()) {
            int cap = carry.capacity();
            while (cap < need) cap = Math.multiplyExact(cap, 2);
            ByteBuffer grown = PackedGpu.directBuffer(cap);
            ByteBuffer old = carry.duplicate();
            old.position(0);
            grown.put(old);
            carry = grown;
        }
        ByteBuffer w = carry.duplicate();
        w.limit(need).position(carry.limit());
        w.put(src.duplicate());
        carry.limit(need).position(0);
        return carry;
    }

    /** The packed extent of a message of `words` words, walked record by
     *  record over bytes that arrive in pieces (PackedInputStream.java:
     *  92-134's records: a tag, its nonzero bytes, then for 0x00 a zero-run
     *  count, for 0xFF a count and that many verbatim words).  walk() resumes
     *  at the first record it could not finish. */
    static final class Extent {
        static final long MORE = -1, MALFORMED = -2;
        private long wordsLeft;
        private int at;   // the next record's first byte

        Extent(long words) { this.wordsLeft = words; }

        /** The byte just past the message in b (absolute index), MORE when
         *  b ends first, MALFORMED when a run passes the message's words. */
        long walk(ByteBuffer b) {
            final int end = b.limit();
            while (wordsLeft > 0) {
                int p = at;
                if (p >= end) return MORE;
                int tag = b.get(p) & 0xff;
                p += 1 + Integer.bitCount(tag);
                long w = 1;
                if (tag == 0 || tag == 0xff) {
                    if (p >= end) return MORE;
                    int run = b.get(p) & 0xff;
                    p += 1 + (tag == 0xff ? 8 * run : 0);
                    w += run;
                }
                if (p > end) return MORE;
                if (w > wordsLeft) return MALFORMED;
                wordsLeft -= w;
                at = p;
            }
            return at;
        }
    }

    /** GPU read of one message from a channel's Source: a try on the bytes
     *  buffered so far; while they end inside the message, more are taken --
     *  until twice as many as at the last try are buffered, the upstream
     *  pauses (a short read: waiting longer could wait on a peer that waits
     *  on us), or the table's bound on the message's packed bytes is
     *  reached.  A message of M bytes costs O(log M) tries plus one per
     *  pause, and the buffer grows geometrically; bytes past the message
     *  stay in the Source for the channel's next read. */
    private static org.capnproto.MessageReader readFrom(Source s, org.capnproto.ReaderOptions options,
                                                        long words) throws IOException {
        final long bound = 10 * (words + 1) + 16;   // packed bytes of the message, at most
        long tried = 0;
        for (;;) {
            if (s.buf.remaining() > tried) {
                ByteBuffer[] segs = gpu().readMessage(s.buf, options.traversalLimitInWords, words);
                if (segs != null) return new org.capnproto.MessageReader(segs, options);
                tried = s.buf.remaining();
            }
            long target = Math.min(Math.max(2 * tried, tried + 1), bound);
            // (a parse takes at most 10 bytes per word: with `bound` bytes
            //  buffered the message cannot be cut short)
            if (target <= s.buf.remaining()) throw new org.capnproto.DecodeException("premature EOF");
            while (s.buf.remaining() < target) {
                if (!s.fill()) break;   // (a short read: the upstream paused)
            }
        }
    }

    // ------------------------------------------------------------------ peek

    /** Unpacked bytes (table + segments) of the message whose packed bytes
     *  start at b.position(), from its segment table alone (Serialize.java:
     *  119-163: the first word, then 4 * (count & ~1) bytes); -1 when b does
     *  not hold the whole table or the table is invalid (the reference path
     *  then reads more, or throws the reference's exception).  Reads with
     *  absolute gets: b is not consumed. */
    static long peekMessageBytes(ByteBuffer b) {
        long[] first = new long[1];
        int p = unpackWords(b, b.position(), b.limit(), first, 1);
        if (p < 0) return -1;
        int raw = (int) first[0];
        int s0 = (int) (first[0] >>> 32);
        if (raw < 0 || raw > 511 || s0 < 0) return -1;
        int count = raw + 1;
        long total = s0;
        int more = (count & ~1) / 2;
        if (more > 0) {
            long[] sizes = new long[more];
            if (unpackWords(b, p, b.limit(), sizes, more) < 0) return -1;
            for (int i = 0; i < count - 1; ++i) {
                int sz = (int) (sizes[i / 2] >>> (32 * (i & 1)));
                if (sz < 0) return -1;
                total += sz;
            }
        }
        return 8L * (1 + more) + 8L * total;
    }

    /** `n` words unpacked from b[p, end) into out (PackedInputStream.java:
     *  49-134's record rules); the position after them, or -1 if the bytes
     *  end first or a run passes the n words. */
    private static int unpackWords(ByteBuffer b, int p, int end, long[] out, int n) {
        int wi = 0;
        while (wi < n) {
            if (p >= end) return -1;
            int tag = b.get(p++) & 0xff;
            long w = 0;
            for (int i = 0; i < 8; ++i) {
                if ((tag >>> i & 1) != 0) {
                    if (p >= end) return -1;
                    w |= (long) (b.get(p++) & 0xff) << (8 * i);
                }
            }
            out[wi++] = w;
            if (tag == 0 || tag == 0xff) {
                if (p >= end) return -1;
                int run = b.get(p++) & 0xff;
                if (run > n - wi) return -1;
                for (int k = 0; k < run; ++k) {
                    long v = 0;
                    if (tag == 0xff) {
                        if (end - p < 8) return -1;
                        for (int i = 0; i < 8; ++i) v |= (long) (b.get(p++) & 0xff) << (8 * i);
                    }
                    out[wi++] = v;
                }
            }
        }
        return p;
    }

    // ---------------------------------------------------------------- Source

    /** A channel's persistent BufferedInputStream (BufferedInputStream.java:
     *  27-38): a carry buffer the channel refills, what the GPU path and the
     *  reference path (readFromUnbuffered) both read.  Direct memory (passed
     *  to JNI zero-copy), grown by doubling. */
    static final class Source implements org.capnproto.BufferedInputStream {
        // (weak: the map's value must not keep its key alive -- the entry
        // goes when the caller drops the channel)
        private final WeakReference<ReadableByteChannel> channelRef;
        ByteBuffer buf;   // [position, limit): bytes not yet consumed

        Source(ReadableByteChannel channel) {
            this.channelRef = new WeakReference<>(channel);
            this.buf = PackedGpu.directBuffer(1 << 16);
            this.buf.limit(0);
        }

        private ReadableByteChannel channel() throws IOException {
            ReadableByteChannel c = channelRef.get();
            if (c == null) throw new IOException("channel closed");
            return c;
        }

        /** Room for `more` bytes after the limit: compact, or grow by doubling. */
        private void reserve(int more) {
            if (buf.capacity() - buf.limit() >= more) return;
            int have = buf.remaining();
            if (buf.capacity() - have >= more && buf.position() >= buf.capacity() / 2) {
                ByteBuffer rest = buf.slice();
                buf.clear();
                buf.put(rest);   // (no overlap: at most cap/2 bytes from past cap/2)
                buf.flip();
                return;
            }
            int cap = buf.capacity();
            while (cap - have < more) cap = Math.multiplyExact(cap, 2);
            ByteBuffer grown = PackedGpu.directBuffer(cap);
            grown.put(buf);
            grown.flip();
            buf = grown;
        }

        /** One read from the channel appended to the buffer (blocking for >= 1
         *  byte).  DecodeException("premature EOF") at the end of the stream
         *  (BufferedInputStreamWrapper.java:98-108).  True if the read filled
         *  all the room it was offered (more may be ready). */
        boolean fill() throws IOException {
            ReadableByteChannel channel = channel();
            reserve(8192);
            int lim = buf.limit();
            ByteBuffer w = buf.duplicate();
            w.position(lim).limit(buf.capacity());
            int offered = w.remaining();
            int n = 0;
            while (n == 0) {
                n = channel.read(w);
                if (n < 0) throw new org.capnproto.DecodeException("premature EOF");
            }
            buf.limit(lim + n);
            return n == offered;
        }

        @Override
        public ByteBuffer getReadBuffer() throws IOException {
            if (!buf.hasRemaining()) {
                buf.clear();
                buf.limit(0);
                fill();
            }
            return buf;
        }

        @Override
        public int read(ByteBuffer dst) throws IOException {
            int want = dst.remaining();
            while (buf.remaining() < want) fill();   // (premature EOF thrown at the end)
            ByteBuffer from = buf.duplicate();
            from.limit(from.position() + want);
            dst.put(from);
            buf.position(buf.position() + want);
            return want;
        }

        @Override
        public boolean isOpen() {
            ReadableByteChannel c = channelRef.get();
            return c != null && c.isOpen();
        }

        @Override
        public void close() throws IOException {
            channel().close();
        }
    }
}
