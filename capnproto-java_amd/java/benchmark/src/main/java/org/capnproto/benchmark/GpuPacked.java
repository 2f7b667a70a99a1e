// Compression.GPU_PACKED for the reference's benchmark harness (SURVEY.md
// §8f row 3): the same bytes as Packed (benchmark/.../Packed.java, i.e.
// SerializePacked.write / read) with the packed codec on the MI355X through
// org.capnproto.gpu.GpuDispatch.  integration/capnproto-java.patch adds it to
// Compression.java:33-34, the "gpu-packed" argument to TestCase.java:188-195
// and its runs to do_benchmarks.bash.
package org.capnproto.benchmark;

import java.io.IOException;

import org.capnproto.gpu.GpuDispatch;

public final class GpuPacked implements Compression {
    // (the device context and the native library are created on first use,
    // GpuDispatch.Holder: naming GPU_PACKED costs nothing on a host without
    // a GPU)

    public void writeBuffered(org.capnproto.BufferedOutputStream writer,
                              org.capnproto.MessageBuilder message) throws IOException {
        // segment table + segments packed on the device in one call
        // (cpk_encode_messages_host): SerializePacked.write's bytes
        GpuDispatch.write(writer, message);
    }

    public org.capnproto.MessageReader newBufferedReader(
        org.capnproto.BufferedInputStream inputStream) throws IOException {
        // "bytes" mode: the whole ArrayInputStream is the read buffer; client /
        // server modes: BufferedInputStreamWrapper's 8 KiB windows are taken
        // until the message decodes (GpuDispatch.read)
        return GpuDispatch.read(inputStream, org.capnproto.ReaderOptions.DEFAULT_READER_OPTIONS);
    }
}
