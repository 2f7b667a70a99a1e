"""Regenerates integration/capnproto-java.patch: the reference-side changes a
capnproto-java maintainer applies (patch -p1 at the repository root) to
select the MI355X codec.

  runtime/.../SerializePacked.java  every public method dispatches to GpuDispatch
                                    when enabled (SerializePacked.java:35-134)
  benchmark/.../Compression.java    Compression.GPU_PACKED (Compression.java:33-34)
  benchmark/.../TestCase.java       the "gpu-packed" argument (TestCase.java:188-195)
  do_benchmarks.bash                gpu-packed runs beside each packed run
  + the new files: runtime/.../gpu/{PackedGpu,GpuDispatch}.java and
    benchmark/.../GpuPacked.java, copied from capnproto-java_amd/java/.

Run in the build container (reads the reference checkout):
  python integration/make_patch.py [/root/reference]
"""
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
JAVA = REPO / "capnproto-java_amd" / "java"
EDITED = ["runtime/src/main/java/org/capnproto/SerializePacked.java",
          "benchmark/src/main/java/org/capnproto/benchmark/Compression.java",
          "benchmark/src/main/java/org/capnproto/benchmark/TestCase.java",
          "do_benchmarks.bash"]
NEW = {"runtime/src/main/java/org/capnproto/gpu/PackedGpu.java":
       JAVA / "src/main/java/org/capnproto/gpu/PackedGpu.java",
       "runtime/src/main/java/org/capnproto/gpu/GpuDispatch.java":
       JAVA / "src/main/java/org/capnproto/gpu/GpuDispatch.java",
       "benchmark/src/main/java/org/capnproto/benchmark/GpuPacked.java":
       JAVA / "benchmark/src/main/java/org/capnproto/benchmark/GpuPacked.java"}


def edit(path: Path, old: str, new: str):
    s = path.read_text()
    assert old in s, (path, old)
    path.write_text(s.replace(old, new, 1))


def main():
    ref = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
    with tempfile.TemporaryDirectory(dir=REPO / "build") as td:
        a, b = Path(td) / "a", Path(td) / "b"
        for f in EDITED:
            for d in (a, b):
                (d / f).parent.mkdir(parents=True, exist_ok=True)
                shutil.copy(ref / f, d / f)
        sp = b / EDITED[0]
        G = "org.capnproto.gpu.GpuDispatch"
        # every public method dispatches (SerializePacked.java:35-134); the
        # one-argument overloads delegate to the two-argument ones
        for sig, kind in ((" tryRead(BufferedInputStream input, ReaderOptions options) throws java.io.IOException {\n",
                           "tryRead"),
                          (" read(BufferedInputStream input, ReaderOptions options) throws java.io.IOException {\n",
                           "read")):
            ret = "Optional<MessageReader>" if kind == "tryRead" else "MessageReader"
            edit(sp, sig, sig +
                 f"        if ({G}.enabled()) {{\n"
                 f"            {ret} m = {G}.{kind}(input, options);\n"
                 f"            if (m != null) return m;  // (null: below {G}.MIN_READ_BYTES, the codec below)\n"
                 f"        }}\n")
        for tail, kind in (("        return Serialize.tryRead(packedInput, options);\n", "tryRead"),
                           ("        return Serialize.read(packedInput, options);\n", "read")):
            body = ("        PackedInputStream packedInput = new PackedInputStream(new BufferedInputStreamWrapper(input));\n"
                    + tail)
            edit(sp, "ReaderOptions options) throws java.io.IOException {\n" + body,
                 "ReaderOptions options) throws java.io.IOException {\n"
                 f"        if ({G}.enabled()) {{  // (one persistent buffered stream per channel)\n"
                 f"            return {kind}({G}.stream(input), options);\n"
                 "        }\n" + body)
        for msg, segs in (("MessageBuilder", "message.getSegmentsForOutput()"), ("MessageReader", "segmentsOf(message)")):
            edit(sp, f"{msg} message) throws java.io.IOException {{\n        PackedOutputStream packedOutputStream",
                 f"{msg} message) throws java.io.IOException {{\n"
                 f"        if ({G}.enabled() && {G}.write(output, {segs})) {{\n"
                 "            return;  // (false: below MIN_WRITE_BYTES, the codec below)\n"
                 "        }\n"
                 "        PackedOutputStream packedOutputStream")
            edit(sp, f"{msg} message) throws java.io.IOException {{\n        BufferedOutputStreamWrapper buffered",
                 f"{msg} message) throws java.io.IOException {{\n"
                 f"        if ({G}.enabled() && {G}.writeToUnbuffered(output, {segs})) {{\n"
                 "            return;  // (the packed bytes straight to the channel)\n"
                 "        }\n"
                 "        BufferedOutputStreamWrapper buffered")
        t = sp.read_text()
        k = t.rstrip().rindex("}")
        sp.write_text(t[:k] + "    // a MessageReader's segments, as Serialize.write(channel, MessageReader) takes them\n"
                      "    private static java.nio.ByteBuffer[] segmentsOf(MessageReader message) {\n"
                      "        java.nio.ByteBuffer[] s = new java.nio.ByteBuffer[message.arena.segments.size()];\n"
                      "        for (int i = 0; i < s.length; ++i) {\n"
                      "            s[i] = message.arena.segments.get(i).buffer.duplicate();\n"
                      "        }\n"
                      "        return s;\n"
                      "    }\n" + t[k:])
        edit(b / EDITED[1], "    public final Compression UNCOMPRESSED = new Uncompressed();",
             "    public final Compression UNCOMPRESSED = new Uncompressed();\n"
             "    public final Compression GPU_PACKED = new GpuPacked();")
        edit(b / EDITED[2], '        } else if (args[2].equals("none")) {\n'
                            '            compression = Compression.UNCOMPRESSED;\n',
             '        } else if (args[2].equals("none")) {\n'
             '            compression = Compression.UNCOMPRESSED;\n'
             '        } else if (args[2].equals("gpu-packed")) {\n'
             '            compression = Compression.GPU_PACKED;\n')
        db = b / EDITED[3]
        edit(db, 'alias run_java="java -cp runtime/target/classes:benchmark/target/classes"',
             'alias run_java="java -cp runtime/target/classes:benchmark/target/classes"\n'
             '# gpu-packed: the MI355X codec (libcapnp_packed_jni.so + libcapnp_packed_hip.so '
             'on java.library.path), every message on the device (minBytes=0: the harness\'s '
             'messages are all under the default size thresholds)\n'
             'alias run_java_gpu="java -Djava.library.path=${CAPNP_GPU_LIB:-lib} '
             '-Dorg.capnproto.gpu.minBytes=0 -cp runtime/target/classes:benchmark/target/classes"')
        for t in ("CarSales", "CatRank", "Eval"):
            line = f"time run_java org.capnproto.benchmark.{t} bytes no-reuse packed $ITERS\n"
            edit(db, line, line + f"time run_java_gpu org.capnproto.benchmark.{t} bytes no-reuse gpu-packed $ITERS\n")
            line = (f"time run_java org.capnproto.benchmark.{t} client no-reuse packed $ITERS < fifo | "
                    f"run_java org.capnproto.benchmark.{t} server no-reuse packed $ITERS > fifo\n")
            edit(db, line, line + f"time run_java_gpu org.capnproto.benchmark.{t} client no-reuse gpu-packed "
                                  f"$ITERS < fifo | run_java_gpu org.capnproto.benchmark.{t} server no-reuse "
                                  f"gpu-packed $ITERS > fifo\n")
        for f, src in NEW.items():
            (b / f).parent.mkdir(parents=True, exist_ok=True)
            shutil.copy(src, b / f)
        r = subprocess.run(["diff", "-ruN", "a", "b"], cwd=td, capture_output=True, text=True)
        assert r.returncode in (0, 1), r.stderr
        # (no timestamps: the patch is stable under regeneration)
        lines = [ln.split("\t")[0] if ln.startswith(("--- ", "+++ ")) else ln
                 for ln in r.stdout.splitlines()]
        (REPO / "integration" / "capnproto-java.patch").write_text("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
