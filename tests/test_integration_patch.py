"""integration/capnproto-java.patch: the reference-side hook (SerializePacked
dispatch, Compression.GPU_PACKED, TestCase "gpu-packed", do_benchmarks.bash
runs) is present, and the Java files it adds are the repository's current
ones (regenerate with integration/make_patch.py after editing them)."""
import re
from pathlib import Path

import pytest

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
    for call in ("GpuDispatch.read(input, options)", "GpuDispatch.tryRead(input, options)",
                 "GpuDispatch.stream(input)", "GpuDispatch.write(output, message.getSegmentsForOutput())",
                 "GpuDispatch.write(output, segmentsOf(message))",
                 "GpuDispatch.writeToUnbuffered(output, message.getSegmentsForOutput())",
                 "GpuDispatch.writeToUnbuffered(output, segmentsOf(message))"):
        assert any(call in ln for ln in sp[1]), call
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


REF = Path("/root/reference")


def _methods(java: str):
    """{signature: body} of every public static method (brace matched)."""
    out = {}
    for m in re.finditer(r"public static [^;{]*?\b(\w+)\(([^)]*)\)[^{;]*\{", java):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(java[i], 0)
            i += 1
        params = re.sub(r"\s+", " ", m.group(2)).strip()
        out[f"{m.group(1)}({params})"] = java[m.end(): i - 1]
    return out


def test_every_public_serialize_packed_method_dispatches(tmp_path):
    """The patched SerializePacked.java (SerializePacked.java:35-134): each of
    its 12 public methods either hands the call to GpuDispatch or is a
    one-line overload (default ReaderOptions) of one that does -- no packed
    read or write can reach the CPU codec without passing the dispatch."""
    import shutil
    import subprocess
    if not REF.exists():
        pytest.skip("needs the reference checkout (build container)")
    rel = "runtime/src/main/java/org/capnproto/SerializePacked.java"
    (tmp_path / rel).parent.mkdir(parents=True)
    shutil.copy(REF / rel, tmp_path / rel)
    sp_patch = PATCH.read_text().split("diff -ruN ")
    hunk = "diff -ruN " + next(h for h in sp_patch if h.startswith(f"a/{rel} "))
    r = subprocess.run(["patch", "-p1"], input=hunk, cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    ms = _methods((tmp_path / rel).read_text())
    assert len(ms) == 12, sorted(ms)
    direct = {k for k, body in ms.items() if "GpuDispatch" in body}
    for k, body in ms.items():
        if k in direct:
            continue
        m = re.fullmatch(r"\s*return (\w+)\(input, ReaderOptions\.DEFAULT_READER_OPTIONS\);\s*", body)
        assert m, f"{k} neither dispatches nor delegates: {body!r}"
        target = [d for d in direct if d.startswith(m.group(1) + "(") and "ReaderOptions" in d
                  and d.split(",")[0] == k.rstrip(")")]
        assert target, f"{k} delegates to an undispatched overload"
    assert len(direct) == 8
