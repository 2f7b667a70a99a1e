"""integration/capnproto-java.patch: the reference-side hook (SerializePacked
dispatch, Compression.GPU_PACKED, TestCase "gpu-packed", do_benchmarks.bash
runs) is present, and the Java files it adds are the repository's current
ones (regenerate with integration/make_patch.py after editing them)."""
import re
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PATCH = REPO / "integration" / "capnproto-java.patch"
JAVA = REPO / "capnproto-java_amd" / "java"


def _files(text):
    """{path: (removed lines, added lines)} per file of a unified diff."""
    out, cur = {}, None
    for ln in text.splitlines():
        m = re.match(r"^\+\+\+ b/(\S+)", ln)
        if m:
            cur = out.setdefault(m.group(1), ([], []))
            continue
        if cur is None or ln.startswith(("--- ", "diff ", "@@")):
            continue
        if ln.startswith("+"):
            cur[1].append(ln[1:])
        elif ln.startswith("-"):
            cur[0].append(ln[1:])
    return out


def test_patch_hooks():
    f = _files(PATCH.read_text())
    sp = f["runtime/src/main/java/org/capnproto/SerializePacked.java"]
    assert not sp[0], "the dispatch only adds lines"
    assert any("GpuDispatch.read(input, options)" in ln for ln in sp[1])
    assert any("GpuDispatch.write(output, message)" in ln for ln in sp[1])
    assert any("GPU_PACKED = new GpuPacked()" in ln
               for ln in f["benchmark/src/main/java/org/capnproto/benchmark/Compression.java"][1])
    assert any('"gpu-packed"' in ln for ln in f["benchmark/src/main/java/org/capnproto/benchmark/TestCase.java"][1])
    runs = [ln for ln in f["do_benchmarks.bash"][1] if ln.startswith("time ") and "gpu-packed" in ln]
    assert len(runs) == 6  # bytes and client/server for CarSales, CatRank, Eval


def test_patch_new_files_are_current():
    f = _files(PATCH.read_text())
    for rel, src in {"runtime/src/main/java/org/capnproto/gpu/PackedGpu.java":
                     JAVA / "src/main/java/org/capnproto/gpu/PackedGpu.java",
                     "runtime/src/main/java/org/capnproto/gpu/GpuDispatch.java":
                     JAVA / "src/main/java/org/capnproto/gpu/GpuDispatch.java",
                     "benchmark/src/main/java/org/capnproto/benchmark/GpuPacked.java":
                     JAVA / "benchmark/src/main/java/org/capnproto/benchmark/GpuPacked.java"}.items():
        removed, added = f[rel]
        assert not removed
        assert added == src.read_text().splitlines(), f"{rel} is stale: run integration/make_patch.py"
