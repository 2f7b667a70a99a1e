"""Host-side binding of the MI355X packed codec (C ABI: include/capnp_packed.h).

Mirrors capnproto-java's packed API for the hot path:
  * encode_batch / decode_batch -- n independent pieces, device-resident
    (each piece = one PackedOutputStream.write / PackedInputStream.read,
    runtime/src/main/java/org/capnproto/PackedOutputStream.java:35-205,
    PackedInputStream.java:35-140).
  * encode_messages / decode_messages -- SerializePacked.write / read per
    message (Serialize.java:256-288, :119-178), segment tables on the device.
  * host-memory forms (encode_host, decode_host, *_gather, decode_stream_host)
    for ByteBuffers that start and end in host memory.
The reference's stream classes themselves are mirrored in C++
(csrc/host/packed_stream.hpp) and Java (java/).

torch is used only for device memory and streams.  There is no CPU fallback:
if the HIP library cannot be loaded every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parents[1]
LIB_PATH = _PKG / "lib" / "libcapnp_packed_hip.so"

OK, EINVAL, ETRUNC, EOVERRUN, ETRAILING, ENOMEM, EDEVICE, EUNSUPPORTED = 0, -1, -2, -3, -4, -5, -6, -8
EFRAME = -7  # segment table invalid (Serialize.java:45-53, :125-163)

EXPORTS = [
    "cpk_abi_version", "cpk_status_string", "cpk_packed_bound", "cpk_batch_packed_capacity",
    "cpk_ctx_create", "cpk_ctx_destroy", "cpk_ctx_device", "cpk_encode_batch",
    "cpk_decode_batch", "cpk_decode_stream", "cpk_encode_host", "cpk_decode_host",
    "cpk_decode_stream_host", "cpk_generate", "cpk_count_mismatch", "cpk_ctx_take_error",
    "cpk_decode_messages", "cpk_encode_messages", "cpk_encode_messages_host",
    "cpk_decode_messages_host", "cpk_encode_host_gather", "cpk_encode_messages_host_gather",
    "cpk_read_message", "cpk_read_message_host", "cpk_ctx_small_fallbacks",
    "cpk_encode_batch_cap", "cpk_encode_messages_cap", "cpk_ctx_dense_windows",
]
MSG_HEAD_WORDS, MSG_INFO_WORDS = 257, 517  # CPK_MSG_HEAD_WORDS, CPK_MSG_INFO_WORDS


class CodecError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {status_string(status)} ({status})" if what else status_string(status))


class DecodeException(CodecError):
    """org.capnproto.DecodeException (runtime/.../DecodeException.java:24-27)."""


class GenParams(ctypes.Structure):
    _fields_ = [("t_zero0", ctypes.c_uint64), ("t_z2n", ctypes.c_uint64),
                ("t_n2z", ctypes.c_uint64), ("t_qbyte", ctypes.c_uint64),
                ("cfg", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


_lib = None


def load(path: Path | None = None, strict: bool = True) -> ctypes.CDLL:
    """Load the HIP codec library; raises if it is missing (no fallback).
    strict=False tolerates an older build without some entry points (A/B
    timing tools only)."""
    global _lib
    if _lib is not None:
        return _lib
    # (CPK_LIB: a variant build for A/B timing and profiling tools, so that no
    # probe ever overwrites the tree's library)
    p = Path(path or os.environ.get("CPK_LIB") or LIB_PATH)
    if os.environ.get("CPK_LIB") and not path:
        strict = False  # (a variant may predate some entry points)
    if not p.exists():
        raise ImportError(f"capnp_packed: HIP library {p} not built "
                          "(run python capnproto-java_amd/build_native.py)")
    L = ctypes.CDLL(str(p))
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    sig = {
        "cpk_abi_version": ([], i32),
        "cpk_status_string": ([i32], ctypes.c_char_p),
        "cpk_packed_bound": ([u64], u64),
        "cpk_batch_packed_capacity": ([vp, u32], u64),
        "cpk_ctx_create": ([i32, ctypes.POINTER(vp)], i32),
        "cpk_ctx_destroy": ([vp], None),
        "cpk_ctx_device": ([vp], i32),
        "cpk_encode_batch": ([vp, vp, vp, u32, u64, vp, vp, vp], i32),
        "cpk_encode_batch_cap": ([vp, vp, vp, u32, u64, vp, u64, vp, vp], i32),
        "cpk_encode_messages_cap": ([vp, vp, vp, u32, vp, u32, u64, vp, u64, vp, vp], i32),
        "cpk_decode_batch": ([vp, vp, vp, vp, u32, vp, vp, vp], i32),
        "cpk_encode_host": ([vp, vp, vp, u32, vp, u64, vp], i32),
        "cpk_encode_host_gather": ([vp, vp, vp, u32, vp, u64, vp], i32),
        "cpk_decode_host": ([vp, vp, vp, vp, u32, vp, vp], i32),
        "cpk_decode_stream": ([vp, vp, u64, vp, u32, vp, vp, vp, vp], i32),
        "cpk_decode_stream_host": ([vp, vp, u64, vp, u32, vp, vp, vp], i32),
        "cpk_generate": ([vp, ctypes.POINTER(GenParams), vp, u32, vp, vp], i32),
        "cpk_count_mismatch": ([vp, vp, vp, u64, vp, vp], i32),
        "cpk_ctx_take_error": ([vp, vp], i32),
        "cpk_ctx_small_fallbacks": ([vp], u64),
        "cpk_ctx_dense_windows": ([vp, vp, ctypes.POINTER(u64), ctypes.POINTER(u64)], i32),
        "cpk_decode_messages": ([vp, vp, vp, u32, u64, vp, u64, vp, vp, vp, u32, vp, vp, vp, vp], i32),
        "cpk_encode_messages": ([vp, vp, vp, u32, vp, u32, u64, vp, vp, vp], i32),
        "cpk_encode_messages_host": ([vp, vp, vp, u32, vp, u32, vp, u64, vp], i32),
        "cpk_encode_messages_host_gather": ([vp, vp, vp, u32, vp, u32, vp, u64, vp], i32),
        "cpk_decode_messages_host": ([vp, vp, vp, u32, u64, vp, u64, vp, u32, vp, vp, vp], i32),
        "cpk_read_message": ([vp, vp, u64, u64, vp, u64, vp, vp], i32),
        "cpk_read_message_host": ([vp, vp, u64, u64, vp, u64, vp], i32),
    }
    for name, (args, res) in sig.items():
        if not strict and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def status_string(s: int) -> str:
    try:
        return load().cpk_status_string(int(s)).decode()
    except ImportError:
        return f"status {s}"


def packed_bound(words: int) -> int:
    return 8 * words + 2 * ((words + 1) // 2)


def batch_capacity(seg_word_off: np.ndarray) -> int:
    w = np.diff(np.asarray(seg_word_off, dtype=np.int64))
    return int(8 * w.sum() + 2 * ((w + 1) // 2).sum() + 16)


def _check(rc: int, what: str):
    if rc != OK:
        raise CodecError(rc, what)


class Context:
    """One HIP device + its look-back workspace (cpk_ctx_create)."""

    def __init__(self, device: int = 0):
        self._lib = load()
        h = ctypes.c_void_p()
        _check(self._lib.cpk_ctx_create(device, ctypes.byref(h)), "cpk_ctx_create")
        self.handle = h
        self.device = device
        # (the decoder choice the library read at creation: CPK_DECODER 1 / 2
        # force one decoder, anything else lets the device pick by density)
        self.decoder_forced = os.environ.get("CPK_DECODER", "") in ("1", "2")

    def close(self):
        if getattr(self, "handle", None):
            self._lib.cpk_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ---- device-resident batch API (torch tensors) -----------------------
    @staticmethod
    def _stream(stream):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        return ctypes.c_void_p(s.cuda_stream)

    def encode_batch(self, d_in, d_seg_word_off, max_seg_words: int, d_out, d_out_off,
                     stream=None):
        n = d_seg_word_off.numel() - 1
        rc = self._lib.cpk_encode_batch(self.handle, d_in.data_ptr(), d_seg_word_off.data_ptr(), n,
                                        int(max_seg_words), d_out.data_ptr(), d_out_off.data_ptr(),
                                        self._stream(stream))
        _check(rc, "cpk_encode_batch")

    def encode_batch_cap(self, d_in, d_seg_word_off, max_seg_words: int, d_out, out_cap: int,
                         d_out_off, stream=None):
        """cpk_encode_batch_cap: as encode_batch, with d_out's byte capacity;
        packed bytes past it are never stored and take_error() then returns
        CPK_ENOMEM (ArrayOutputStream.java:40-42)."""
        n = d_seg_word_off.numel() - 1
        rc = self._lib.cpk_encode_batch_cap(self.handle, d_in.data_ptr(), d_seg_word_off.data_ptr(), n,
                                            int(max_seg_words), d_out.data_ptr(), int(out_cap),
                                            d_out_off.data_ptr(), self._stream(stream))
        _check(rc, "cpk_encode_batch_cap")

    def encode_messages_cap(self, d_in, d_seg_word_off, d_msg_seg_off, max_seg_words: int, d_out,
                            out_cap: int, d_out_off, stream=None):
        """cpk_encode_messages_cap: encode_messages with d_out's byte capacity."""
        nseg = d_seg_word_off.numel() - 1
        nm = d_msg_seg_off.numel() - 1
        rc = self._lib.cpk_encode_messages_cap(self.handle, d_in.data_ptr(), d_seg_word_off.data_ptr(),
                                               nseg, d_msg_seg_off.data_ptr(), nm, int(max_seg_words),
                                               d_out.data_ptr(), int(out_cap), d_out_off.data_ptr(),
                                               self._stream(stream))
        _check(rc, "cpk_encode_messages_cap")

    def take_error(self, stream=None) -> int:
        """Synchronises `stream`; CPK_ENOMEM if an encode since the last call
        would have stored packed bytes past its out_cap (the *_cap forms),
        CPK_EINVAL if it met a piece larger than its max_seg_words hint
        (output undefined)."""
        return self._lib.cpk_ctx_take_error(self.handle, self._stream(stream))

    def dense_windows(self, stream=None) -> tuple[int, int]:
        """(windows walked serially, serial walks given back) by the block
        map's dense form in the last decode (cpk_ctx_dense_windows)."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._lib.cpk_ctx_dense_windows(self.handle, self._stream(stream), ctypes.byref(a),
                                               ctypes.byref(b)), "cpk_ctx_dense_windows")
        return int(a.value), int(b.value)

    def small_fallbacks(self) -> int:
        """One-launch host calls whose completion flag was still unset after
        the stream sync that stands in past 5 ms (a lost flag); 0 in normal
        operation, late launches on a busy GPU included."""
        return int(self._lib.cpk_ctx_small_fallbacks(self.handle))

    def decode_batch(self, d_packed, d_in_off, d_seg_word_off, d_out, d_status, stream=None):
        n = d_seg_word_off.numel() - 1
        rc = self._lib.cpk_decode_batch(self.handle, d_packed.data_ptr(), d_in_off.data_ptr(),
                                        d_seg_word_off.data_ptr(), n, d_out.data_ptr(),
                                        d_status.data_ptr(), self._stream(stream))
        _check(rc, "cpk_decode_batch")

    def decode_stream(self, d_packed, avail: int, d_seg_word_off, d_out, d_in_off, d_status,
                      stream=None):
        """Serialize.read-style decode of pieces back to back from one packed
        stream of `avail` bytes (cpk_decode_stream); d_in_off[n+1] gets the
        piece boundaries found.  Synchronises `stream` once for streams of
        256 KiB and more (they are cut into blocks and decoded in parallel)."""
        n = d_seg_word_off.numel() - 1
        rc = self._lib.cpk_decode_stream(self.handle, d_packed.data_ptr(), int(avail),
                                         d_seg_word_off.data_ptr(), n, d_out.data_ptr(),
                                         d_in_off.data_ptr(), d_status.data_ptr(), self._stream(stream))
        _check(rc, "cpk_decode_stream")

    def encode_messages(self, d_in, d_seg_word_off, d_msg_seg_off, max_seg_words: int, d_out,
                        d_out_off, stream=None):
        """SerializePacked.write per message (cpk_encode_messages): the
        segment tables are built and packed on the device.  d_out_off gets
        nm + nseg + 1 piece offsets in message order."""
        nseg = d_seg_word_off.numel() - 1
        nm = d_msg_seg_off.numel() - 1
        rc = self._lib.cpk_encode_messages(self.handle, d_in.data_ptr(), d_seg_word_off.data_ptr(),
                                           nseg, d_msg_seg_off.data_ptr(), nm, int(max_seg_words),
                                           d_out.data_ptr(), d_out_off.data_ptr(),
                                           self._stream(stream))
        _check(rc, "cpk_encode_messages")

    def decode_messages(self, d_packed, d_msg_off, d_out, d_seg_word_off, d_seg_in_off,
                        d_seg_status, d_msg_seg_off, d_msg_status,
                        traversal_limit_words: int = 8 * 1024 * 1024, stream=None):
        """Serialize.read per message over a batch of packed messages with
        known byte ranges (cpk_decode_messages).  Capacities come from the
        tensors' sizes.  -> (status, total words, total segments); status
        CPK_ENOMEM (nothing decoded) if the capacities are too small."""
        nm = d_msg_off.numel() - 1
        tot = (ctypes.c_uint64 * 2)()
        seg_cap = min(d_seg_status.numel() if d_seg_status is not None else 0,
                      d_seg_word_off.numel() - 1 if d_seg_word_off is not None else 0)

        def ptr(t):
            return t.data_ptr() if t is not None else None
        rc = self._lib.cpk_decode_messages(
            self.handle, d_packed.data_ptr(), d_msg_off.data_ptr(), nm, int(traversal_limit_words),
            ptr(d_out), d_out.numel() * d_out.element_size() // 8 if d_out is not None else 0,
            ptr(d_seg_word_off), ptr(d_seg_in_off), ptr(d_seg_status), seg_cap,
            d_msg_seg_off.data_ptr(), d_msg_status.data_ptr(), tot, self._stream(stream))
        if rc not in (OK, ENOMEM):
            _check(rc, "cpk_decode_messages")
        return rc, int(tot[0]), int(tot[1])

    def generate(self, params: GenParams, d_seg_word_off, d_out, stream=None):
        n = d_seg_word_off.numel() - 1
        _check(self._lib.cpk_generate(self.handle, ctypes.byref(params), d_seg_word_off.data_ptr(),
                                      n, d_out.data_ptr(), self._stream(stream)), "cpk_generate")

    def count_mismatch(self, d_a, d_b, words: int, d_cnt, stream=None):
        _check(self._lib.cpk_count_mismatch(self.handle, d_a.data_ptr(), d_b.data_ptr(), int(words),
                                            d_cnt.data_ptr(), self._stream(stream)),
               "cpk_count_mismatch")

    # ---- host-memory forms (numpy) -----------------------------------------
    def encode_host(self, data: np.ndarray, seg_word_off: np.ndarray, out: np.ndarray = None):
        """-> (packed bytes as uint8 array, out_off uint64[n+1]).  `out`: a
        reusable uint8 buffer of at least batch_capacity() bytes."""
        swo = np.ascontiguousarray(seg_word_off, dtype=np.uint64)
        n = len(swo) - 1
        data = np.ascontiguousarray(data, dtype=np.uint8)
        cap = batch_capacity(swo)
        if out is None:
            out = np.zeros(cap, dtype=np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < cap:
            raise ValueError("out: contiguous uint8, at least batch_capacity() bytes")
        off = np.zeros(n + 1, dtype=np.uint64)
        rc = self._lib.cpk_encode_host(self.handle, data.ctypes.data if data.size else None,
                                       swo.ctypes.data, n, out.ctypes.data, cap, off.ctypes.data)
        _check(rc, "cpk_encode_host")
        return out[: int(off[-1])], off

    def encode_host_gather(self, pieces, out: np.ndarray = None):
        """Gather form: `pieces` = list of uint64 word arrays, one per piece,
        each left where it lies (no concatenation).  -> (packed uint8, out_off)."""
        pieces = [np.ascontiguousarray(x, dtype=np.uint64) for x in pieces]
        n = len(pieces)
        swo = np.zeros(n + 1, dtype=np.uint64)
        swo[1:] = np.cumsum([x.size for x in pieces])
        ptrs = (ctypes.c_void_p * max(n, 1))(*[x.ctypes.data if x.size else None for x in pieces])
        cap = batch_capacity(swo)
        if out is None:
            out = np.zeros(cap, dtype=np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < cap:
            raise ValueError("out: contiguous uint8, at least batch_capacity() bytes")
        off = np.zeros(n + 1, dtype=np.uint64)
        rc = self._lib.cpk_encode_host_gather(self.handle, ptrs, swo.ctypes.data, n,
                                              out.ctypes.data, cap, off.ctypes.data)
        _check(rc, "cpk_encode_host_gather")
        return out[: int(off[-1])], off

    def decode_host(self, packed: np.ndarray, in_off: np.ndarray, seg_word_off: np.ndarray,
                    out: np.ndarray = None):
        """-> (decoded uint8 array, status int32[n]).  Never raises on bad data.
        `out`: a reusable uint8 buffer of at least 8 * seg_word_off[-1] bytes."""
        swo = np.ascontiguousarray(seg_word_off, dtype=np.uint64)
        io = np.ascontiguousarray(in_off, dtype=np.uint64)
        n = len(swo) - 1
        pk = np.ascontiguousarray(packed, dtype=np.uint8)
        if out is None:
            out = np.zeros(int(8 * swo[-1]) + 8, dtype=np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < int(8 * swo[-1]):
            raise ValueError("out: contiguous uint8, at least 8 * seg_word_off[-1] bytes")
        st = np.zeros(max(n, 1), dtype=np.int32)
        rc = self._lib.cpk_decode_host(self.handle, pk.ctypes.data if pk.size else None,
                                       io.ctypes.data, swo.ctypes.data, n, out.ctypes.data,
                                       st.ctypes.data)
        if rc not in (OK, ETRUNC, EOVERRUN, ETRAILING, EUNSUPPORTED, EINVAL):
            _check(rc, "cpk_decode_host")
        return out[: int(8 * swo[-1])], st[:n]


def _encode_messages_host(self, messages):
    """SerializePacked.write for each message (a list of segments, bytes of
    whole words) -> the packed bytes of all messages, back to back."""
    segs = [bytes(s) for m in messages for s in m]
    swo = np.concatenate([[0], np.cumsum([len(s) // 8 for s in segs], dtype=np.uint64)]).astype(np.uint64)
    mso = np.concatenate([[0], np.cumsum([len(m) for m in messages], dtype=np.uint64)]).astype(np.uint64)
    data = np.frombuffer(b"".join(segs) + b"\0" * 8, np.uint8)
    cap = batch_capacity(swo) + sum(10 * ((len(m) + 2) // 2 + 1) for m in messages)
    out = np.zeros(cap, np.uint8)
    off = np.zeros(len(messages) + len(segs) + 1, np.uint64)
    _check(self._lib.cpk_encode_messages_host(self.handle, data.ctypes.data, swo.ctypes.data,
                                              len(segs), mso.ctypes.data, len(messages),
                                              out.ctypes.data, cap, off.ctypes.data),
           "cpk_encode_messages_host")
    return out[: int(off[-1])].tobytes(), off


def _encode_messages_host_gather(self, messages):
    """As _encode_messages_host, each segment passed where it lies
    (cpk_encode_messages_host_gather)."""
    segs = [np.frombuffer(bytes(s), np.uint8) for m in messages for s in m]
    swo = np.concatenate([[0], np.cumsum([s.size // 8 for s in segs], dtype=np.uint64)]).astype(np.uint64)
    mso = np.concatenate([[0], np.cumsum([len(m) for m in messages], dtype=np.uint64)]).astype(np.uint64)
    ptrs = (ctypes.c_void_p * max(len(segs), 1))(*[s.ctypes.data if s.size else None for s in segs])
    cap = batch_capacity(swo) + sum(10 * ((len(m) + 2) // 2 + 1) for m in messages)
    out = np.zeros(cap, np.uint8)
    off = np.zeros(len(messages) + len(segs) + 1, np.uint64)
    _check(self._lib.cpk_encode_messages_host_gather(self.handle, ptrs, swo.ctypes.data,
                                                     len(segs), mso.ctypes.data, len(messages),
                                                     out.ctypes.data, cap, off.ctypes.data),
           "cpk_encode_messages_host_gather")
    return out[: int(off[-1])].tobytes(), off


def _decode_messages_host(self, packed, msg_off, traversal_limit_words: int = 8 * 1024 * 1024):
    """Serialize.read per message -> (message statuses, [[segment bytes]])."""
    pk = np.frombuffer(bytes(packed), np.uint8)
    mo = np.ascontiguousarray(msg_off, dtype=np.uint64)
    nm = len(mo) - 1
    mso = np.zeros(nm + 1, np.uint64)
    mst = np.zeros(max(nm, 1), np.int32)
    tot = np.zeros(2, np.uint64)
    pkp = pk.ctypes.data if pk.size else None
    rc = self._lib.cpk_decode_messages_host(self.handle, pkp, mo.ctypes.data, nm,
                                            traversal_limit_words, None, 0, None, 0,
                                            mso.ctypes.data, mst.ctypes.data, tot.ctypes.data)
    if rc == ENOMEM:
        out = np.zeros(int(tot[0]) * 8 + 8, np.uint8)
        sw = np.zeros(int(tot[1]) + 1, np.uint64)
        rc = self._lib.cpk_decode_messages_host(self.handle, pkp, mo.ctypes.data, nm,
                                                traversal_limit_words, out.ctypes.data, int(tot[0]),
                                                sw.ctypes.data, int(tot[1]), mso.ctypes.data,
                                                mst.ctypes.data, tot.ctypes.data)
    else:
        out, sw = np.zeros(8, np.uint8), np.zeros(1, np.uint64)
    if rc in (ENOMEM, EDEVICE):
        _check(rc, "cpk_decode_messages_host")
    msgs = [[out[8 * int(sw[j]): 8 * int(sw[j + 1])].tobytes() for j in range(int(mso[m]), int(mso[m + 1]))]
            for m in range(nm)]
    return mst[:nm], msgs


Context.encode_messages_host = _encode_messages_host
Context.encode_messages_host_gather = _encode_messages_host_gather
Context.decode_messages_host = _decode_messages_host


def _decode_stream_host(self, packed: np.ndarray, seg_word_off: np.ndarray, out: np.ndarray = None):
    """PackedInputStream.read per piece, back to back over one stream.
    -> (decoded uint8 array, piece boundaries uint64[n+1], status int32[n]).
    `out`: a reusable uint8 buffer of at least 8 * seg_word_off[-1] bytes."""
    swo = np.ascontiguousarray(seg_word_off, dtype=np.uint64)
    n = len(swo) - 1
    pk = np.ascontiguousarray(packed, dtype=np.uint8)
    if out is None:
        out = np.zeros(int(8 * swo[-1]) + 8, dtype=np.uint8)
    elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < int(8 * swo[-1]):
        raise ValueError("out: contiguous uint8, at least 8 * seg_word_off[-1] bytes")
    io = np.zeros(n + 1, dtype=np.uint64)
    st = np.zeros(max(n, 1), dtype=np.int32)
    rc = self._lib.cpk_decode_stream_host(self.handle, pk.ctypes.data if pk.size else None,
                                          pk.size, swo.ctypes.data, n, out.ctypes.data,
                                          io.ctypes.data, st.ctypes.data)
    if rc not in (OK, ETRUNC, EOVERRUN, ETRAILING, EUNSUPPORTED, EINVAL):
        _check(rc, "cpk_decode_stream_host")
    return out[: int(8 * swo[-1])], io, st[:n]


Context.decode_stream_host = _decode_stream_host


def _read_message(self, d_packed, avail: int, d_out, d_info, traversal_limit_words: int = 8 * 1024 * 1024,
                  stream=None):
    """cpk_read_message: one message from the front of a device-resident
    packed stream (Serialize.read, Serialize.java:119-178), no host sync.
    d_out: int64 tensor of out_cap_words + MSG_HEAD_WORDS words; d_info:
    int64[MSG_INFO_WORDS], written on the device."""
    cap = d_out.numel() * d_out.element_size() // 8 - MSG_HEAD_WORDS
    if cap < 0 or d_info.numel() * d_info.element_size() < 8 * MSG_INFO_WORDS:
        raise ValueError("d_out / d_info too small")
    _check(self._lib.cpk_read_message(self.handle, d_packed.data_ptr(), int(avail), int(traversal_limit_words),
                                      d_out.data_ptr(), cap, d_info.data_ptr(), self._stream(stream)),
           "cpk_read_message")


def _read_message_host(self, packed, out_cap_words: int | None = None,
                       traversal_limit_words: int = 8 * 1024 * 1024):
    """cpk_read_message_host -> (status, [segment bytes], bytes consumed,
    info row).  out_cap_words None: sized by a first call (CPK_ENOMEM gives
    the words needed)."""
    pk = np.ascontiguousarray(np.frombuffer(bytes(packed), np.uint8) if not isinstance(packed, np.ndarray)
                              else packed, dtype=np.uint8)
    info = np.zeros(MSG_INFO_WORDS, np.uint64)
    cap = 0 if out_cap_words is None else int(out_cap_words)
    for _ in range(2):
        out = np.zeros(max(cap, 1), np.uint64)
        rc = self._lib.cpk_read_message_host(self.handle, pk.ctypes.data if pk.size else None, pk.size,
                                             int(traversal_limit_words), out.ctypes.data, cap,
                                             info.ctypes.data)
        if rc == ENOMEM and out_cap_words is None and int(info[3]) > cap:
            cap = int(info[3])
            continue
        break
    if rc in (EDEVICE, EINVAL) or (rc == ENOMEM and int(info.view(np.int64)[0]) != ENOMEM):
        _check(rc, "cpk_read_message_host")
    if rc != OK:
        return rc, [], 0, info
    n = int(info[2])
    b = out.view(np.uint8)
    segs = [b[8 * int(info[4 + i]): 8 * int(info[5 + i])].tobytes() for i in range(n)]
    return rc, segs, int(info[1]), info


Context.read_message = _read_message
Context.read_message_host = _read_message_host


def gen_params(cfg: int, z: float, lz: float, q: float) -> GenParams:
    """Thresholds of the synthetic 2-state Markov generator, out of 2^31:
    `FastRand.nextInt()` never returns a negative value (Common.java:31-38,
    arithmetic `>>` clears bit 31), so a draw lies in [0, 2^31)."""
    def thr(p):
        return int(min(max(p, 0.0), 1.0) * (1 << 31))
    a = 1.0 / lz
    b = 1.0 if z >= 1.0 else a * z / (1.0 - z)
    return GenParams(thr(z), thr(a), thr(b), thr(q), cfg, 0)


CONFIGS = {
    2: dict(z=0.5, lz=4.0, q=0.25),
    3: dict(z=0.05, lz=1.5, q=1 / 256),
    4: dict(z=0.9, lz=64.0, q=0.25),
}


def preset(cfg: int) -> GenParams:
    c = CONFIGS[cfg]
    return gen_params(cfg, c["z"], c["lz"], c["q"])
