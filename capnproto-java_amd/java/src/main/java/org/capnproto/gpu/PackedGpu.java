// Java facade over the MI355X packed codec (include/capnp_packed.h via JNI).
//
// Additive batch API next to the reference's stream classes
// (runtime/src/main/java/org/capnproto/PackedOutputStream.java,
//  PackedInputStream.java, SerializePacked.java): one call encodes / decodes
// every piece of a batch -- the segment table and each segment of a message
// are pieces, exactly the write() calls Serialize.write issues
// (Serialize.java:256-288).  Output bytes are identical to the reference's.
package org.capnproto.gpu;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;

public final class PackedGpu implements AutoCloseable {
    static {
        System.loadLibrary("capnp_packed_jni");   // + libcapnp_packed_hip.so beside it
    }

    private static native long nativeCreate(int device);
    private static native void nativeDestroy(long handle);
    private static native long nativeCapacity(long[] segWordOff);
    private static native void nativeEncode(long handle, ByteBuffer in, long[] segWordOff,
                                            ByteBuffer out, long[] outOff);
    private static native void nativeDecode(long handle, ByteBuffer packed, long[] inOff,
                                            long[] segWordOff, ByteBuffer out);

    private static native void nativeEncodeMessages(long handle, ByteBuffer in, long[] segWordOff,
                                                    long[] msgSegOff, ByteBuffer out, long[] outOff);
    private static native void nativeDecodeMessages(long handle, ByteBuffer packed, long[] msgOff,
                                                    long traversalLimit, ByteBuffer out,
                                                    long[] segWordOff, long[] msgSegOff,
                                                    long[] totals);
    private static native void nativeEncodeGather(long handle, ByteBuffer[] pieces, int[] positions,
                                                  long[] segWordOff, ByteBuffer out, long[] outOff);
    private static native void nativeEncodeMessagesGather(long handle, ByteBuffer[] segs, int[] positions,
                                                          long[] segWordOff, long[] msgSegOff,
                                                          ByteBuffer out, long[] outOff);
    private static native long nativeDecodeStream(long handle, ByteBuffer packed, int position,
                                                  int limit, long[] segWordOff, ByteBuffer out);
    private static native int nativeReadMessage(long handle, ByteBuffer packed, int position, int limit,
                                                long traversalLimit, ByteBuffer out, long[] info);

    /** Status codes nativeReadMessage returns instead of throwing
     *  (include/capnp_packed.h). */
    static final int CPK_OK = 0, CPK_ETRUNC = -2, CPK_ENOMEM = -5;
    /** CPK_MSG_INFO_WORDS: status, consumed, count, words, offsets. */
    static final int MSG_INFO_WORDS = 517;

    private long handle;

    /** The message of the DecodeException thrown when the packed bytes end
     *  inside what a read must fill (CPK_ETRUNC, cpk_status_string; the
     *  reference's "Premature EOF", ArrayInputStream.java:53-58).
     *  DecodeException is final, so GpuDispatch tells truncation apart by it
     *  and takes more bytes from a channel. */
    public static final String TRUNCATED = "premature end of packed input";

    public static boolean isTruncation(org.capnproto.DecodeException e) {
        return TRUNCATED.equals(e.getMessage());
    }

    /** A direct buffer of `bytes` bytes: ByteBuffer capacities are ints, so a
     *  batch whose packed or unpacked size passes 2 GiB - 1 must be split by
     *  the caller (an IOException here rather than a wrapped (int) cast). */
    private static ByteBuffer direct(long bytes) throws IOException {
        if (bytes < 0 || bytes > Integer.MAX_VALUE)
            throw new IOException("batch of " + bytes + " bytes exceeds one ByteBuffer (2 GiB - 1): split it");
        return ByteBuffer.allocateDirect((int) bytes).order(ByteOrder.LITTLE_ENDIAN);
    }

    /** A little-endian direct buffer of `bytes` bytes (GpuDispatch's stream
     *  buffers). */
    static ByteBuffer directBuffer(int bytes) {
        return ByteBuffer.allocateDirect(bytes).order(ByteOrder.LITTLE_ENDIAN);
    }

    /** `b`'s remaining bytes in a direct buffer (itself when already direct). */
    private static ByteBuffer asDirect(ByteBuffer b) throws IOException {
        return asDirect(b, Long.MAX_VALUE);
    }

    /** At most `max` of `b`'s remaining bytes in a direct buffer (b itself
     *  when already direct): a heap buffer is copied only as far as a read
     *  can reach. */
    private static ByteBuffer asDirect(ByteBuffer b, long max) throws IOException {
        if (b.isDirect()) return b;
        ByteBuffer src = b.duplicate();
        if (src.remaining() > max) src.limit(src.position() + (int) max);
        ByteBuffer d = direct(src.remaining());
        d.put(src).flip();
        return d;
    }

    public PackedGpu(int device) {
        this.handle = nativeCreate(device);
    }

    @Override
    public void close() {
        if (handle != 0) {
            nativeDestroy(handle);
            handle = 0;
        }
    }

    /** Result of encodeBatch: the packed stream and each piece's byte range. */
    public static final class Packed {
        public final ByteBuffer bytes;   // direct, limit = total packed length
        public final long[] offsets;     // n + 1 entries
        Packed(ByteBuffer b, long[] o) { bytes = b; offsets = o; }
    }

    /** Packs each buffer as one PackedOutputStream.write() piece; the
     *  buffers' [position, limit) must be word-aligned (as the reference
     *  assumes, PackedOutputStream.java:66-112). */
    public Packed encodeBatch(ByteBuffer[] pieces) throws IOException {
        int n = pieces.length;
        long[] swo = new long[n + 1];
        long words = 0;
        for (int i = 0; i < n; ++i) {
            int len = pieces[i].remaining();
            if (len % 8 != 0) throw new IllegalArgumentException("piece not word-aligned");
            swo[i] = words;
            words += len / 8;
        }
        swo[n] = words;
        ByteBuffer out = direct(nativeCapacity(swo));
        long[] off = new long[n + 1];
        boolean direct = true;
        for (ByteBuffer p : pieces) direct &= p.isDirect();
        if (direct) {  // builder segments allocated DIRECT: packed where they lie
            int[] pos = new int[n];
            for (int i = 0; i < n; ++i) pos[i] = pieces[i].position();
            nativeEncodeGather(handle, pieces, pos, swo, out, off);
        } else {
            ByteBuffer in = direct(words * 8);
            for (ByteBuffer p : pieces) in.put(p.duplicate());
            nativeEncode(handle, in, swo, out, off);
        }
        for (ByteBuffer p : pieces) p.position(p.limit());   // as write() leaves inBuf (:203)
        out.limit((int) off[n]);
        return new Packed(out, off);
    }

    /** SerializePacked.write for each message (its segments, as
     *  MessageBuilder.getSegmentsForOutput returns them,
     *  BuilderArena.java:143-154): the segment tables are built and packed on
     *  the device; the bytes equal one SerializePacked.write per message,
     *  back to back.  offsets: nm + nseg + 1 piece offsets, message order. */
    public Packed encodeMessages(ByteBuffer[][] messages) throws IOException {
        int nm = messages.length, nseg = 0;
        for (ByteBuffer[] m : messages) nseg += m.length;
        long[] swo = new long[nseg + 1];
        long[] mso = new long[nm + 1];
        long words = 0, tableCap = 0;
        int s = 0;
        for (int i = 0; i < nm; ++i) {
            mso[i] = s;
            tableCap += 10L * ((messages[i].length + 2) / 2 + 1);
            for (ByteBuffer b : messages[i]) {
                if (b.remaining() % 8 != 0) throw new IllegalArgumentException("segment not word-aligned");
                swo[s++] = words;
                words += b.remaining() / 8;
            }
        }
        mso[nm] = s;
        swo[nseg] = words;
        ByteBuffer out = direct(nativeCapacity(swo) + tableCap);
        long[] off = new long[nm + nseg + 1];
        ByteBuffer[] flat = new ByteBuffer[nseg];
        boolean direct = true;
        s = 0;
        for (ByteBuffer[] m : messages)
            for (ByteBuffer b : m) { flat[s++] = b; direct &= b.isDirect(); }
        if (direct) {  // DIRECT builder segments: packed where they lie
            int[] pos = new int[nseg];
            for (int i = 0; i < nseg; ++i) pos[i] = flat[i].position();
            nativeEncodeMessagesGather(handle, flat, pos, swo, mso, out, off);
        } else {
            ByteBuffer in = direct(words * 8 + 8);
            for (ByteBuffer b : flat) in.put(b.duplicate());
            nativeEncodeMessages(handle, in, swo, mso, out, off);
        }
        out.limit((int) off[nm + nseg]);
        return new Packed(out, off);
    }

    /** SerializePacked.read for each message: message m is packed bytes
     *  [msgOff[m], msgOff[m+1]) (direct buffer).  Returns each message's
     *  segments (ByteBuffer[] per message, little-endian, as Serialize.read
     *  hands them to MessageReader, Serialize.java:165-177).
     *  @throws org.capnproto.DecodeException for the first bad message */
    public ByteBuffer[][] decodeMessages(ByteBuffer packed, long[] msgOff, long traversalLimitInWords)
            throws IOException {
        int nm = msgOff.length - 1;
        long[] mso = new long[nm + 1];
        long[] tot = new long[2];
        nativeDecodeMessages(handle, packed, msgOff, traversalLimitInWords, null, null, mso, tot);
        ByteBuffer out = direct(tot[0] * 8 + 8);
        long[] swo = new long[(int) tot[1] + 1];
        nativeDecodeMessages(handle, packed, msgOff, traversalLimitInWords, out, swo, mso, tot);
        ByteBuffer[][] res = new ByteBuffer[nm][];
        for (int m = 0; m < nm; ++m) {
            int a = (int) mso[m], b = (int) mso[m + 1];
            res[m] = new ByteBuffer[b - a];
            for (int j = a; j < b; ++j) {
                ByteBuffer seg = out.duplicate();
                seg.position((int) (swo[j] * 8)).limit((int) (swo[j + 1] * 8));
                res[m][j - a] = seg.slice().order(ByteOrder.LITTLE_ENDIAN);
            }
        }
        return res;
    }

    /** Unpacks piece i into outs[i] (filled to its limit, like
     *  PackedInputStream.read, PackedInputStream.java:35-140).
     *  @throws org.capnproto.DecodeException on malformed input */
    public void decodeBatch(ByteBuffer packed, long[] inOff, ByteBuffer[] outs) throws IOException {
        int n = outs.length;
        long[] swo = new long[n + 1];
        long words = 0;
        for (int i = 0; i < n; ++i) {
            int len = outs[i].remaining();
            if (len % 8 != 0)
                throw new org.capnproto.DecodeException("PackedInputStream reads must be word-aligned");
            swo[i] = words;
            words += len / 8;
        }
        swo[n] = words;
        ByteBuffer pk = asDirect(packed);
        ByteBuffer out = direct(words * 8);
        nativeDecode(handle, pk, inOff, swo, out);
        for (int i = 0; i < n; ++i) {
            ByteBuffer slice = out.duplicate();
            slice.position((int) (swo[i] * 8)).limit((int) (swo[i + 1] * 8));
            outs[i].put(slice);
        }
    }
    /** read() calls back to back on one packed stream, as fillBuffer issues
     *  them (Serialize.java:74-83 over PackedInputStream.read,
     *  PackedInputStream.java:35-140): outs[i] is filled to its limit from
     *  packed[position, limit), each read consuming only the bytes it needs.
     *  packed.position advances by the bytes consumed (as the reference's
     *  BufferedInputStream does).
     *  @throws org.capnproto.DecodeException on malformed input */
    public void decodeStream(ByteBuffer packed, ByteBuffer[] outs) throws IOException {
        ByteBuffer pk = asDirect(packed);
        long used = decodeStreamDirect(pk, pk.position(), outs);
        packed.position(packed.position() + (int) used);
    }

    /** decodeStream on a direct buffer from byte `at`; returns the bytes
     *  consumed (the buffer's position is left alone). */
    private long decodeStreamDirect(ByteBuffer pk, int at, ByteBuffer[] outs) throws IOException {
        int n = outs.length;
        long[] swo = new long[n + 1];
        long words = 0;
        for (int i = 0; i < n; ++i) {
            int len = outs[i].remaining();
            if (len % 8 != 0)
                throw new org.capnproto.DecodeException("PackedInputStream reads must be word-aligned");
            swo[i] = words;
            words += len / 8;
        }
        swo[n] = words;
        ByteBuffer out = direct(words * 8 + 8);
        long used = nativeDecodeStream(handle, pk, at, pk.limit(), swo, out);
        for (int i = 0; i < n; ++i) {
            ByteBuffer slice = out.duplicate();
            slice.position((int) (swo[i] * 8)).limit((int) (swo[i + 1] * 8));
            outs[i].put(slice);
        }
        return used;
    }

    /** SerializePacked.read of one message from the front of `packed`
     *  (Serialize.java:119-178 over PackedInputStream) in ONE library call
     *  (cpk_read_message_host): the device reads the first word and the rest
     *  of the table, runs doRead's checks (count, sizes, traversal limit,
     *  makeByteBufferForWords's bound) and decodes every segment.  The
     *  segments come back as slices of one direct buffer (zero-copy for JNI,
     *  SURVEY.md §8f row 4), little-endian; packed.position advances past the
     *  message.  Returns null, consuming nothing, when the bytes end inside
     *  the message (a channel reader takes more and calls again).
     *  @param wordsHint expected unpacked words (e.g. from the table), 0 if
     *         unknown: the output is sized by a first call then
     *  @throws org.capnproto.DecodeException for a malformed message */
    public ByteBuffer[] readMessage(ByteBuffer packed, long traversalLimitInWords, long wordsHint)
            throws IOException {
        long cap = Math.max(wordsHint, 0);
        // a heap buffer is copied to direct memory once, only as far as a
        // message of `cap` words can reach (10 bytes per word at most)
        ByteBuffer pk = asDirect(packed, cap > 0 ? 10 * (cap + 257) + 16 : Long.MAX_VALUE);
        long[] info = new long[MSG_INFO_WORDS];
        for (;;) {
            ByteBuffer out = direct(8 * cap + 8);
            int st = nativeReadMessage(handle, pk, pk.position(), pk.limit(), traversalLimitInWords, out, info);
            if (st == CPK_ENOMEM && info[3] > cap) {   // (the table says how many words)
                cap = info[3];
                // a heap buffer's copy reaches only as far as the old hint's
                // words can: copy it again for the table's count
                if (pk != packed) pk = asDirect(packed, 10 * (cap + 257) + 16);
                continue;
            }
            if (st == CPK_ETRUNC) return null;
            if (st != CPK_OK) throw new IOException("cpk_read_message_host: status " + st);
            packed.position(packed.position() + (int) info[1]);
            int count = (int) info[2];
            ByteBuffer[] segs = new ByteBuffer[count];
            for (int i = 0; i < count; ++i) {
                ByteBuffer seg = out.duplicate();
                seg.position((int) (info[4 + i] * 8)).limit((int) (info[5 + i] * 8));
                segs[i] = seg.slice().order(ByteOrder.LITTLE_ENDIAN);
            }
            return segs;
        }
    }

    /** readMessage with the output sized by the call itself; a message cut
     *  short is the reference's premature EOF (ArrayInputStream.java:53-58). */
    public ByteBuffer[] readMessage(ByteBuffer packed, long traversalLimitInWords) throws IOException {
        ByteBuffer[] segs = readMessage(packed, traversalLimitInWords, 0);
        if (segs == null) throw new org.capnproto.DecodeException(TRUNCATED);
        return segs;
    }

    /** Serialize.java:45 (largest segment makeByteBufferForWords accepts). */
    public static final int MAX_SEGMENT_WORDS = (1 << 28) - 1;
}
