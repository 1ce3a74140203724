"""ctypes binding of oracle/icrc_oracle.c -- TEST INFRASTRUCTURE ONLY.

Used by tests/ (checker), __graft_entry__.smoke() (checker) and bench.py's
cpu_baseline leg (the timed CPU port).  See icrc_oracle.c for the spec
citations.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p, u32p, u64p = (ctypes.c_void_p,) * 3
        for name in ("oracle_icrc_bitwise_ex", "oracle_icrc_bytewise_ex", "oracle_icrc_fast_ex"):
            f = getattr(L, name)
            f.argtypes = [u8p, ctypes.c_uint32, ctypes.c_int]
            f.restype = ctypes.c_uint32
        L.oracle_icrc_batch_ex.argtypes = [u8p, u64p, u32p, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_uint32, u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_icrc_batch_ex.restype = ctypes.c_int
        L.oracle_synth_batch.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint32, ctypes.c_uint32, u8p]
        L.oracle_synth_batch.restype = None
        L.oracle_synth_ragged.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, u32p, u8p]
        L.oracle_synth_ragged.restype = None
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


FAMILY = {"v4": 0, "v6": 1, "auto": 2}


def icrc_one(pkt: bytes, kind: str = "fast", family: str = "v4") -> int:
    buf = np.frombuffer(bytes(pkt), dtype=np.uint8)
    fn = {"bitwise": lib().oracle_icrc_bitwise_ex, "bytewise": lib().oracle_icrc_bytewise_ex,
          "fast": lib().oracle_icrc_fast_ex}[kind]
    return int(fn(buf.ctypes.data, len(pkt), FAMILY[family]))


def icrc_batch(buf: np.ndarray, offsets=None, lengths=None, stride: int = 0, count=None,
               l3_offset: int = 0, threads: int = 1, kind: str = "fast", family: str = "v4") -> np.ndarray:
    buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    if lengths is not None:
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    if count is None:
        count = len(offsets) if offsets is not None else buf.size // stride
    out = np.empty(count, dtype=np.uint32)
    k = {"bitwise": 0, "bytewise": 1, "fast": 2}[kind]
    lib().oracle_icrc_batch_ex(buf.ctypes.data, _ptr(offsets), _ptr(lengths), stride, count,
                               l3_offset, out.ctypes.data, threads, k, FAMILY[family])
    return out


def synth_batch(seed: int, first: int, count: int, n: int, stride: int | None = None) -> np.ndarray:
    """Host restatement of the device synthetic generator: (count, stride) uint8."""
    stride = stride or n
    buf = np.empty((count, stride), dtype=np.uint8)
    lib().oracle_synth_batch(seed, first, count, n, stride, buf.ctypes.data)
    return buf


def synth_ragged(seed: int, first: int, lengths, offsets=None, size: int | None = None) -> tuple:
    """Host restatement of ricrc_synth_ragged_device: packet k = global packet
    first + k with lengths[k] bytes, at offsets[k] (default: packed back to
    back).  Returns (buf, offsets)."""
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    if offsets is None:
        offsets = np.zeros(len(lengths), np.uint64)
        if len(lengths) > 1:
            offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    if size is None:
        size = int(offsets[-1]) + int(lengths[-1]) if len(lengths) else 0
    buf = np.zeros(size, np.uint8)
    lib().oracle_synth_ragged(seed, first, len(lengths), offsets.ctypes.data, lengths.ctypes.data, buf.ctypes.data)
    return buf, offsets
