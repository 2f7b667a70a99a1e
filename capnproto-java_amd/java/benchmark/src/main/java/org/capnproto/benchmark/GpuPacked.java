// Compression.GPU_PACKED for the reference's benchmark harness (SURVEY.md
// §8f row 3): the same bytes as Packed (benchmark/.../Packed.java, i.e.
// SerializePacked.write / read) with the packed codec on the MI355X through
// org.capnproto.gpu.PackedGpu.  INTEGRATION.md shows the two-line additions
// to Compression.java:33-34 and TestCase.java:188-195 that select it with the
// argument "gpu-packed", and the do_benchmarks.bash lines that run it.
package org.capnproto.benchmark;

import java.io.IOException;
import java.nio.ByteBuffer;

import org.capnproto.gpu.PackedGpu;

public final class GpuPacked implements Compression {
    // One device context per process (cpk_ctx_create on device 0, or
    // CAPNP_GPU_DEVICE); the harness is single-threaded (TestCase.java).
    private static final PackedGpu GPU =
        new PackedGpu(Integer.parseInt(System.getenv().getOrDefault("CAPNP_GPU_DEVICE", "0")));

    public void writeBuffered(org.capnproto.BufferedOutputStream writer,
                              org.capnproto.MessageBuilder message) throws IOException {
        // Segment table + segments packed on the device in one call
        // (cpk_encode_messages_host): SerializePacked.write's bytes.
        PackedGpu.Packed p = GPU.encodeMessages(new ByteBuffer[][] {message.getSegmentsForOutput()});
        ByteBuffer bytes = p.bytes.duplicate();
        bytes.position(0);
        while (bytes.hasRemaining()) {
            writer.write(bytes);
        }
        writer.flush();
    }

    public org.capnproto.MessageReader newBufferedReader(
        org.capnproto.BufferedInputStream inputStream) throws IOException {
        // The packed format carries no length, so the message is read from
        // the source's buffered bytes (getReadBuffer: the whole array for
        // the "bytes" mode's ArrayInputStream, ArrayInputStream.java:53-58)
        // with the reference's read() sequence; the buffer's position
        // advances past exactly the bytes the message used.
        ByteBuffer buf = inputStream.getReadBuffer();
        ByteBuffer[] segments = GPU.readMessage(
            buf, org.capnproto.ReaderOptions.DEFAULT_READER_OPTIONS.traversalLimitInWords);
        return new org.capnproto.MessageReader(segments, org.capnproto.ReaderOptions.DEFAULT_READER_OPTIONS);
    }
}
