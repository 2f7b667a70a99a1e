"""GpuDispatch.Extent (capnproto-java_amd/java/.../GpuDispatch.java): the host
walk that finds a message's packed extent so a GPU read consumes exactly the
bytes the reference's PackedInputStream does (PackedInputStream.java:47-59,
:84-88).  No JDK here: the walk is restated line for line below and checked
against the oracle's Serialize.read (bytes consumed) over streams of several
messages cut into read buffers at every size; a textual check keeps the
restatement tied to the Java source."""
import re
from pathlib import Path

import numpy as np

JAVA = (Path(__file__).resolve().parents[1] / "capnproto-java_amd" / "java" / "src" / "main" / "java"
        / "org" / "capnproto" / "gpu" / "GpuDispatch.java")
MORE, MALFORMED = -1, -2


class Extent:
    """GpuDispatch.Extent, restated."""

    def __init__(self, words):
        self.words_left = words
        self.at = 0

    def walk(self, b: bytes):
        end = len(b)
        while self.words_left > 0:
            p = self.at
            if p >= end:
                return MORE
            tag = b[p]
            p += 1 + bin(tag).count("1")
            w = 1
            if tag in (0, 0xFF):
                if p >= end:
                    return MORE
                run = b[p]
                p += 1 + (8 * run if tag == 0xFF else 0)
                w += run
            if p > end:
                return MORE
            if w > self.words_left:
                return MALFORMED
            self.words_left -= w
            self.at = p
        return self.at


def test_restatement_tracks_java_source():
    src = JAVA.read_text()
    body = src[src.index("static final class Extent"):src.index("GPU read of one message from a channel")]
    for line in ("p += 1 + Integer.bitCount(tag);", "if (tag == 0 || tag == 0xff) {",
                 "p += 1 + (tag == 0xff ? 8 * run : 0);", "if (p > end) return MORE;",
                 "if (w > wordsLeft) return MALFORMED;", "at = p;"):
        assert line in body, line
    assert re.search(r"cur\.position\(cur\.position\(\) \+ \(msg\.position\(\) - base\)\)", src)


def _stream(oracle, rng, nmsg):
    msgs, words = [], []
    for _ in range(nmsg):
        nseg = int(rng.integers(1, 5))
        segs = []
        for _ in range(nseg):
            n = int(rng.integers(0, 400))
            cfg = int(rng.choice([2, 3, 4]))
            swo = np.array([0, n], np.uint64)
            p = oracle.preset(cfg)
            p.cfg = int(rng.integers(0, 1 << 20))
            segs.append(oracle.generate(p, swo).tobytes())
        msgs.append(oracle.write_message(segs))
        words.append((nseg + 2) // 2 + sum(len(s) // 8 for s in segs))
    return msgs, words


def test_extent_equals_reference_consumption(oracle):
    """Each message's walked extent = the bytes Serialize.read consumes, with
    the stream delivered in read buffers of 1 .. 9000 bytes (the walk resumes
    across buffers; a buffer the message ends in is used only in part)."""
    rng = np.random.default_rng(17)
    msgs, words = _stream(oracle, rng, 40)
    stream = b"".join(msgs)
    for chunk in (1, 7, 64, 1000, 8192, 9000):
        pos = 0
        for m, w in zip(msgs, words):
            st, _, used = oracle.read_message(stream[pos:])
            assert st == oracle.OK and used == len(m)
            ext, carry, q = Extent(w), b"", pos
            while True:
                nxt = stream[q: q + chunk]
                assert nxt, "ran out of bytes"
                base = len(carry)
                carry += nxt
                e = ext.walk(carry)
                if e == MORE:
                    q += len(nxt)
                    continue
                assert e >= 0 and base <= e <= len(carry)
                q += e - base
                break
            assert q - pos == used
            pos = q


def test_extent_flags_runs_past_the_message():
    # one word, then a zero run of 3 more: a 2-word message cannot hold it
    assert Extent(2).walk(bytes([0, 3])) == MALFORMED
    assert Extent(4).walk(bytes([0, 3])) == 2
    assert Extent(5).walk(bytes([0xFF]) + bytes(range(1, 9)) + bytes([1])) == MORE
