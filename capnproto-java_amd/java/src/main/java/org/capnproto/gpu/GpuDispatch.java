// The hook SerializePacked.write / read take when the MI355X codec is enabled
// (integration/capnproto-java.patch adds the two dispatch lines to
// runtime/src/main/java/org/capnproto/SerializePacked.java:58-61, :101-114).
//
// Enabled by -Dorg.capnproto.gpu=true or CAPNP_GPU=1 (device: CAPNP_GPU_DEVICE,
// default 0).  Output bytes and exceptions are the reference's: write packs the
// segment table and segments on the device (Serialize.java:256-288); read runs
// Serialize.read's sequence (Serialize.java:119-178) on the device over the
// bytes the stream has buffered.
package org.capnproto.gpu;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.util.Map;
import java.util.WeakHashMap;

public final class GpuDispatch {
    private GpuDispatch() {}

    private static final boolean ENABLED =
        Boolean.getBoolean("org.capnproto.gpu") || "1".equals(System.getenv("CAPNP_GPU"));

    /** One context per process, created on first use (the library loads then). */
    private static final class Holder {
        static final PackedGpu GPU =
            new PackedGpu(Integer.parseInt(System.getenv().getOrDefault("CAPNP_GPU_DEVICE", "0")));
    }

    public static boolean enabled() { return ENABLED; }

    public static PackedGpu gpu() { return Holder.GPU; }

    /** SerializePacked.write(output, message): the packed bytes of
     *  table + segments, written to `output` (flushed, as writeToUnbuffered
     *  does, SerializePacked.java:119-124). */
    public static void write(org.capnproto.BufferedOutputStream output,
                             org.capnproto.MessageBuilder message) throws IOException {
        PackedGpu.Packed p = gpu().encodeMessages(new ByteBuffer[][] {message.getSegmentsForOutput()});
        ByteBuffer bytes = p.bytes.duplicate();
        bytes.position(0);
        while (bytes.hasRemaining()) output.write(bytes);
        output.flush();
    }

    // Bytes taken from a channel-backed stream (BufferedInputStreamWrapper,
    // 8 KiB at a time, BufferedInputStreamWrapper.java:28-108) but not yet
    // used by a message: a message's packed length is known only once it is
    // decoded, so the reader may take bytes past it.  Kept per stream.
    private static final Map<org.capnproto.BufferedInputStream, ByteBuffer> CARRY = new WeakHashMap<>();

    /** SerializePacked.read(input, options). */
    public static synchronized org.capnproto.MessageReader read(org.capnproto.BufferedInputStream input,
                                                                org.capnproto.ReaderOptions options)
            throws IOException {
        if (input instanceof org.capnproto.ArrayInputStream) {
            // the whole array is the read buffer (ArrayInputStream.java:53-58)
            ByteBuffer buf = input.getReadBuffer();
            ByteBuffer[] segs = gpu().readMessage(buf, options.traversalLimitInWords);
            return new org.capnproto.MessageReader(segs, options);
        }
        ByteBuffer acc = CARRY.get(input);
        for (;;) {
            if (acc != null && acc.hasRemaining()) {
                try {
                    ByteBuffer[] segs = gpu().readMessage(acc, options.traversalLimitInWords);
                    CARRY.put(input, acc);   // (position now past the message)
                    return new org.capnproto.MessageReader(segs, options);
                } catch (org.capnproto.DecodeException e) {
                    if (!PackedGpu.isTruncation(e)) throw e;
                    // the bytes so far end inside the message: take more
                }
            }
            ByteBuffer src = input.getReadBuffer();   // blocks for >= 1 byte; DecodeException at EOF
            int have = acc == null ? 0 : acc.remaining();
            ByteBuffer grown = ByteBuffer.allocateDirect(have + src.remaining());
            if (acc != null) grown.put(acc);
            grown.put(src);   // (src.position reaches its limit: the bytes are taken)
            grown.flip();
            acc = grown;
        }
    }
}
