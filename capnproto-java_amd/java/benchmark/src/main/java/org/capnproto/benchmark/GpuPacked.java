// Compression.GPU_PACKED for the reference's benchmark harness (SURVEY.md
// §8f row 3): the bytes of Packed (benchmark/.../Packed.java, i.e.
// SerializePacked.write / read) with the codec on the MI355X through
// org.capnproto.gpu.GpuDispatch, whatever -Dorg.capnproto.gpu says.
// integration/capnproto-java.patch adds it to Compression.java:33-34, the
// "gpu-packed" argument to TestCase.java:188-195 and its runs to
// do_benchmarks.bash.  Messages below GpuDispatch.MIN_WRITE_BYTES /
// MIN_READ_BYTES take the reference's codec, as every dispatched
// SerializePacked call does: with the default thresholds none of the
// harness's carsales / catrank / eval messages (a few KiB, under the 1 MiB
// scratch of TestCase.java:46) reaches the GPU; the do_benchmarks.bash lines
// the patch adds pass -Dorg.capnproto.gpu.minBytes=0, every message on the
// GPU, to time the device path itself.
package org.capnproto.benchmark;

import java.io.IOException;

import org.capnproto.ReaderOptions;
import org.capnproto.SerializePacked;
import org.capnproto.gpu.GpuDispatch;

public final class GpuPacked implements Compression {
    // (the device context and the native library are created on first use,
    // GpuDispatch.Holder: naming GPU_PACKED costs nothing on a host without
    // a GPU)

    public void writeBuffered(org.capnproto.BufferedOutputStream writer,
                              org.capnproto.MessageBuilder message) throws IOException {
        // table + segments packed on the device in one call
        // (cpk_encode_messages_host), or the reference's PackedOutputStream
        // for a small message
        if (!GpuDispatch.write(writer, message.getSegmentsForOutput())) {
            SerializePacked.write(writer, message);
        }
        writer.flush();
    }

    public org.capnproto.MessageReader newBufferedReader(
        org.capnproto.BufferedInputStream inputStream) throws IOException {
        // one cpk_read_message_host call ("bytes" mode: the whole
        // ArrayInputStream; client / server: the wrapper's windows until the
        // message decodes), or the reference's PackedInputStream
        org.capnproto.MessageReader m = GpuDispatch.read(inputStream, ReaderOptions.DEFAULT_READER_OPTIONS);
        return m != null ? m : SerializePacked.read(inputStream);
    }
}
