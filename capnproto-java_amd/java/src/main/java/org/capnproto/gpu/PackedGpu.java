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

    private long handle;

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
        ByteBuffer in = ByteBuffer.allocateDirect((int) (words * 8)).order(ByteOrder.LITTLE_ENDIAN);
        for (ByteBuffer p : pieces) in.put(p.duplicate());
        ByteBuffer out = ByteBuffer.allocateDirect((int) nativeCapacity(swo));
        long[] off = new long[n + 1];
        nativeEncode(handle, in, swo, out, off);
        for (ByteBuffer p : pieces) p.position(p.limit());   // as write() leaves inBuf (:203)
        out.limit((int) off[n]);
        return new Packed(out, off);
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
        ByteBuffer pk = packed.isDirect() ? packed
                : (ByteBuffer) ByteBuffer.allocateDirect(packed.remaining()).put(packed.duplicate()).flip();
        ByteBuffer out = ByteBuffer.allocateDirect((int) (words * 8));
        nativeDecode(handle, pk, inOff, swo, out);
        for (int i = 0; i < n; ++i) {
            ByteBuffer slice = out.duplicate();
            slice.position((int) (swo[i] * 8)).limit((int) (swo[i + 1] * 8));
            outs[i].put(slice);
        }
    }
}
