"""ctypes wrapper over oracle/packed_oracle.c -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of capnproto-java's packed codec
(runtime/src/main/java/org/capnproto/PackedOutputStream.java:35-205,
PackedInputStream.java:35-140, Serialize.java:119-178 / :256-307).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the checker; the product (capnproto-java_amd/) never does.
Parity pinned by the reference's KATs in tests/golden/ (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "_build" / "libcpk_oracle.so"

OK, EINVAL, ETRUNC, EOVERRUN, ETRAILING, EFRAME = 0, -1, -2, -3, -4, -7

# Synthetic workload presets: (zero-word fraction z,
# mean zero-run length Lz, zero-byte probability q in nonzero words).
CONFIGS = {
    2: dict(z=0.5, lz=4.0, q=0.25),      # 1 M x 64 KiB, ~50 % zero words
    3: dict(z=0.05, lz=1.5, q=1 / 256),  # dense, 0xFF literal-run heavy
    4: dict(z=0.9, lz=64.0, q=0.25),     # sparse, 0x00 RLE heavy
}


def build() -> Path:
    """Compile the oracle with the committed Makefile (gcc)."""
    src = [_HERE / "packed_oracle.c", _HERE / "packed_oracle.h"]
    if not _LIB_PATH.exists() or any(
        s.stat().st_mtime > _LIB_PATH.stat().st_mtime for s in src
    ):
        subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


class GenParams(ctypes.Structure):
    _fields_ = [
        ("t_zero0", ctypes.c_uint64),
        ("t_z2n", ctypes.c_uint64),
        ("t_n2z", ctypes.c_uint64),
        ("t_qbyte", ctypes.c_uint64),
        ("cfg", ctypes.c_uint32),
        ("pad", ctypes.c_uint32),
    ]


def _thr(p: float) -> int:
    # FastRand.nextInt() is never negative: with Java's arithmetic `>>`
    # (Common.java:36) bit 31 of `w ^ (w >> 19)` and of `tmp ^ (tmp >> 8)` is
    # always clear, so every draw lies in [0, 2^31) and a probability p is the
    # threshold p * 2^31 (round 3 used 2^32: every probability doubled).
    return int(min(max(p, 0.0), 1.0) * (1 << 31))


def gen_params(cfg: int, z: float, lz: float, q: float) -> GenParams:
    """Integer thresholds (out of 2^31: draws are non-negative) of the 2-state Markov generator.
    Stationary zero fraction z: P(z->n) = 1/Lz, P(n->z) = (1/Lz) z/(1-z)."""
    a = 1.0 / lz
    b = 1.0 if z >= 1.0 else a * z / (1.0 - z)
    return GenParams(_thr(z), _thr(a), _thr(b), _thr(q), cfg, 0)


def preset(cfg: int) -> GenParams:
    c = CONFIGS[cfg]
    return gen_params(cfg, c["z"], c["lz"], c["q"])


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = ctypes.CDLL(str(build()))
        u8p = ctypes.c_void_p
        L.cpko_pack.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.cpko_pack.restype = ctypes.c_size_t
        L.cpko_packed_bound.argtypes = [ctypes.c_size_t]
        L.cpko_packed_bound.restype = ctypes.c_size_t
        L.cpko_unpack.argtypes = [u8p, ctypes.c_size_t,
                                  ctypes.POINTER(ctypes.c_size_t), u8p, ctypes.c_size_t]
        L.cpko_unpack.restype = ctypes.c_int
        L.cpko_pack_batch.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, u8p, ctypes.c_int]
        L.cpko_pack_batch.restype = ctypes.c_size_t
        L.cpko_unpack_batch.argtypes = [u8p, u8p, u8p, ctypes.c_uint32, u8p, u8p, ctypes.c_int]
        L.cpko_unpack_batch.restype = ctypes.c_int
        L.cpko_write_message.argtypes = [ctypes.POINTER(ctypes.c_void_p), u8p,
                                         ctypes.c_uint32, u8p]
        L.cpko_write_message.restype = ctypes.c_size_t
        L.cpko_read_message.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                        ctypes.POINTER(ctypes.c_uint32), u8p, ctypes.c_uint32,
                                        u8p, ctypes.c_size_t, ctypes.c_uint64]
        L.cpko_read_message.restype = ctypes.c_int
        L.cpko_generate.argtypes = [ctypes.POINTER(GenParams), u8p, ctypes.c_uint32,
                                    ctypes.c_uint32, u8p]
        L.cpko_generate.restype = None
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def packed_bound(words: int) -> int:
    return 8 * words + 2 * ((words + 1) // 2)


def pack(data: bytes | np.ndarray) -> bytes:
    """One PackedOutputStream.write() of `data` (len % 8 == 0)."""
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    assert a.size % 8 == 0, "PackedOutputStream input must be word-aligned"
    out = np.zeros(packed_bound(a.size // 8) + 16, dtype=np.uint8)
    n = lib().cpko_pack(_ptr(a) if a.size else None, a.size, _ptr(out))
    return out[:n].tobytes()


def unpack(packed: bytes, out_len: int) -> tuple[int, bytes, int]:
    """One PackedInputStream.read() of out_len bytes. -> (status, bytes, consumed)."""
    a = np.frombuffer(bytes(packed) + b"\0" * 16, dtype=np.uint8)
    out = np.zeros(max(out_len, 1), dtype=np.uint8)
    used = ctypes.c_size_t(0)
    st = lib().cpko_unpack(_ptr(a), len(packed), ctypes.byref(used), _ptr(out), out_len)
    return st, out[:out_len].tobytes(), used.value


def pack_batch(data: np.ndarray, seg_word_off: np.ndarray, threads: int = 1):
    """Pack each segment as its own piece. -> (packed uint8 array, out_off uint64[n+1])."""
    n = len(seg_word_off) - 1
    words = np.diff(seg_word_off)
    cap = int(sum(packed_bound(int(w)) for w in words)) if n < 4096 else \
        int(8 * words.sum() + 2 * ((words + 1) // 2).sum())
    out = np.zeros(cap + 16, dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.uint64)
    swo = np.ascontiguousarray(seg_word_off, dtype=np.uint64)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    total = lib().cpko_pack_batch(_ptr(data), _ptr(swo), n, _ptr(out), _ptr(off), threads)
    return out[:total], off


def unpack_batch(packed: np.ndarray, in_off: np.ndarray, seg_word_off: np.ndarray,
                 threads: int = 1):
    """-> (decoded uint8 array, status int32[n])."""
    n = len(seg_word_off) - 1
    swo = np.ascontiguousarray(seg_word_off, dtype=np.uint64)
    io = np.ascontiguousarray(in_off, dtype=np.uint64)
    pk = np.concatenate([np.ascontiguousarray(packed, dtype=np.uint8), np.zeros(16, np.uint8)])
    out = np.zeros(int(8 * swo[-1]) + 8, dtype=np.uint8)
    st = np.zeros(n, dtype=np.int32)
    lib().cpko_unpack_batch(_ptr(pk), _ptr(io), _ptr(swo), n, _ptr(out), _ptr(st), threads)
    return out[: int(8 * swo[-1])], st


def write_message(segments: list[bytes]) -> bytes:
    """Serialize.write through PackedOutputStream (SerializePacked.write)."""
    n = len(segments)
    bufs = [np.frombuffer(s + b"\0" * 8, dtype=np.uint8) for s in segments]
    ptrs = (ctypes.c_void_p * n)(*[_ptr(b) for b in bufs])
    words = np.array([len(s) // 8 for s in segments], dtype=np.uint32)
    cap = packed_bound(n + 2) + sum(packed_bound(len(s) // 8) for s in segments) + 16
    out = np.zeros(cap, dtype=np.uint8)
    m = lib().cpko_write_message(ptrs, _ptr(words), n, _ptr(out))
    return out[:m].tobytes()


def read_message(data: bytes, traversal_limit_words: int = 8 * 1024 * 1024,
                 max_seg: int = 512, out_cap: int | None = None):
    """Serialize.read through PackedInputStream. -> (status, [segments], consumed)."""
    a = np.frombuffer(bytes(data) + b"\0" * 16, dtype=np.uint8)
    cap = out_cap if out_cap is not None else 64 * len(data) * 32 + 4096
    out = np.zeros(cap, dtype=np.uint8)
    words = np.zeros(max_seg, dtype=np.uint32)
    nseg = ctypes.c_uint32(0)
    used = ctypes.c_size_t(0)
    st = lib().cpko_read_message(_ptr(a), len(data), ctypes.byref(used), ctypes.byref(nseg),
                                 _ptr(words), max_seg, _ptr(out), cap, traversal_limit_words)
    if st != OK:
        return st, [], used.value
    segs, o = [], 0
    for i in range(nseg.value):
        b = 8 * int(words[i])
        segs.append(out[o:o + b].tobytes())
        o += b
    return st, segs, used.value


def generate(params: GenParams, seg_word_off: np.ndarray, first: int = 0,
             count: int | None = None) -> np.ndarray:
    """Host copy of the synthetic generator (same stream as the device one)."""
    swo = np.ascontiguousarray(seg_word_off, dtype=np.uint64)
    n = len(swo) - 1
    if count is None:
        count = n - first
    words = int(swo[first + count] - swo[first])
    out = np.zeros(8 * words + 8, dtype=np.uint8)
    lib().cpko_generate(ctypes.byref(params), _ptr(swo), first, count, _ptr(out))
    return out[: 8 * words]


if __name__ == "__main__":  # pragma: no cover
    print(build(), os.path.getsize(build()))
