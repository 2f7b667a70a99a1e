"""The host forms' per-message latency against the CPU codec
(tests/cpp/threshold_probe.cpp): one SerializePacked.write
(cpk_encode_messages_host) and one SerializePacked.read
(cpk_read_message_host) per size, each checked byte for byte against the
oracle first.  The table goes to gpurun_out/threshold_probe.txt; it sets
GpuDispatch.DEFAULT_MIN_BYTES."""
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
def test_threshold_probe(tmp_path):
    exe = tmp_path / "probe"
    lib = REPO / "capnproto-java_amd" / "lib"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", f"-I{REPO / 'include'}",
                    str(REPO / "tests" / "cpp" / "threshold_probe.cpp"), str(REPO / "oracle" / "packed_oracle.c"),
                    f"-L{lib}", "-lcapnp_packed_hip", f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "1024"], capture_output=True, text=True, timeout=100)
    out = REPO / "gpurun_out"
    out.mkdir(exist_ok=True)
    (out / "threshold_probe.txt").write_text(r.stdout)
    print(r.stdout)
    assert r.returncode == 0 and "MISMATCH" not in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_pass_by_bytes_replay(tmp_path):
    """TestCase.passByBytes (TestCase.java:80-123) replayed in C++ over the
    facade's mirror (tests/cpp/pass_by_bytes.cpp): what the gpu-packed lines
    of do_benchmarks.bash cost per iteration against the packed codec, for
    messages of 1 KiB - 4 MiB; every size is checked against the oracle first.
    The table goes to gpurun_out/pass_by_bytes.txt."""
    exe = tmp_path / "pbb"
    lib = REPO / "capnproto-java_amd" / "lib"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", f"-I{REPO / 'include'}",
                    str(REPO / "tests" / "cpp" / "pass_by_bytes.cpp"), str(REPO / "oracle" / "packed_oracle.c"),
                    f"-L{lib}", "-lcapnp_packed_hip", f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "4096", "50"], capture_output=True, text=True, timeout=100)
    out = REPO / "gpurun_out"
    out.mkdir(exist_ok=True)
    (out / "pass_by_bytes.txt").write_text(r.stdout)
    print(r.stdout)
    assert r.returncode == 0 and "MISMATCH" not in r.stdout, r.stdout + r.stderr
