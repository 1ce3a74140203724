"""roce_icrc -- Python mirror of libroceicrc, the MI355X RoCEv2 ICRC engine.

This is the host-side interface a caller such as the reference's
``python/simulator.py`` binds through ctypes (the reference has no FFI of its
own for this path; see include/roce_icrc.h and INTEGRATION.md):

* :func:`icrc` / :func:`verify` / :func:`stamp` -- one packet at a time
  (the simulator's wire crossings, simulator.py:49-55 and 59-82); CPU,
  re-entrant, no GPU launch per 60-byte packet.
* :class:`Context` -- batches on the GPUs: host buffers in/out
  (``batch_host``), device-resident buffers (``batch_device`` /
  ``verify_device``, torch tensors or raw pointers, async on a stream) and the
  synthetic batch generator used by bench.py and the tests.

Every batch call runs the gfx950 kernels; there is no CPU fallback.  If the
shared library is missing, importing this package raises.
"""
from __future__ import annotations

import ctypes
import errno
import os

import numpy as np

from . import wire  # noqa: F401  (Packet <-> bytes adapter)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libroceicrc.so")

MIN_LEN = 44
MAX_LEN = 65535

EXPORTED = (
    "ricrc_one", "ricrc_verify_one", "ricrc_stamp_one", "ricrc_is_rocev2", "ricrc_shift",
    "ricrc_one_ex", "ricrc_verify_one_ex", "ricrc_stamp_one_ex", "ricrc_classify", "ricrc_repair_one",
    "ricrc_combine", "ricrc_create", "ricrc_create_devices", "ricrc_destroy", "ricrc_device_count", "ricrc_batch_host",
    "ricrc_batch_device", "ricrc_verify_device", "ricrc_repair_device", "ricrc_batch_host_ex",
    "ricrc_batch_device_ex", "ricrc_verify_device_ex", "ricrc_host_alloc", "ricrc_host_free",
    "ricrc_host_register", "ricrc_host_unregister", "ricrc_synth_device", "ricrc_stream", "ricrc_strerror",
)


class ICRCError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        super().__init__(f"{what}: {rc} ({_strerror(rc)})")


def _load():
    # libroceicrc and PyTorch-ROCm each need a libamdhip64.so.7 (ROCm 7.2 from
    # /opt/rocm, resp. torch's bundled copy) under the same SONAME: whichever
    # is loaded first serves the whole process.  Load torch's first when it is
    # installed so that torch tensors/streams and our kernels share one HIP
    # runtime (the other order leaves torch with "No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libroceicrc.so not found at {LIB_PATH}; build it with "
            "`make -C roce-test_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, u8p = ctypes.c_void_p, ctypes.c_void_p
    u32, u64, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sig = {
        "ricrc_one": ([u8p, u32], u32),
        "ricrc_verify_one": ([u8p, u32], i32),
        "ricrc_stamp_one": ([u8p, u32], i32),
        "ricrc_is_rocev2": ([u8p, u32], i32),
        "ricrc_one_ex": ([u8p, u32, u32], u32),
        "ricrc_verify_one_ex": ([u8p, u32, u32], i32),
        "ricrc_stamp_one_ex": ([u8p, u32, u32], i32),
        "ricrc_classify": ([u8p, u32], i32),
        "ricrc_repair_one": ([u8p, u32, u32, u8p, u32, u32, u32, ctypes.POINTER(u32)], i32),
        "ricrc_shift": ([u32, u64], u32),
        "ricrc_combine": ([u32, u32, u64], u32),
        "ricrc_create": ([ctypes.POINTER(vp), i32], i32),
        "ricrc_create_devices": ([ctypes.POINTER(vp), ctypes.POINTER(i32), i32], i32),
        "ricrc_destroy": ([vp], None),
        "ricrc_device_count": ([vp], i32),
        "ricrc_batch_host": ([vp, u8p, vp, vp, u32, u64, u32, vp], i32),
        "ricrc_batch_device": ([vp, i32, vp, vp, vp, u32, u64, u32, vp, vp], i32),
        "ricrc_verify_device": ([vp, i32, vp, vp, vp, u32, u64, u32, vp, vp], i32),
        "ricrc_batch_host_ex": ([vp, u8p, vp, vp, u32, u64, u32, vp, u32], i32),
        "ricrc_batch_device_ex": ([vp, i32, vp, vp, vp, u32, u64, u32, vp, vp, u32], i32),
        "ricrc_verify_device_ex": ([vp, i32, vp, vp, vp, u32, u64, u32, vp, vp, u32], i32),
        "ricrc_repair_device": ([vp, i32, vp, vp, vp, u32, u64, u32, u32, u32, vp, u32, u32, u32, vp, vp], i32),
        "ricrc_host_alloc": ([vp, u64], vp),
        "ricrc_host_free": ([vp, vp], None),
        "ricrc_host_register": ([vp, vp, u64], i32),
        "ricrc_host_unregister": ([vp, vp], i32),
        "ricrc_synth_device": ([vp, i32, u64, u64, u64, u32, u32, vp, vp], i32),
        "ricrc_stream": ([vp, i32], vp),
        "ricrc_strerror": ([i32], ctypes.c_char_p),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


lib = _load()


def _strerror(rc: int) -> str:
    return lib.ricrc_strerror(rc).decode()


def _buf(pkt):
    """(pointer, length, keepalive) for bytes-like input without copying when possible."""
    if isinstance(pkt, bytes):
        return ctypes.cast(ctypes.c_char_p(pkt), ctypes.c_void_p).value, len(pkt), pkt
    mv = memoryview(pkt).cast("B")
    if mv.readonly:
        b = bytes(mv)
        return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value, len(b), b
    arr = (ctypes.c_uint8 * len(mv)).from_buffer(mv)
    return ctypes.addressof(arr), len(mv), arr


# ------------------------------------------------------------------ per packet
# Address families of the *_ex entry points (include/roce_icrc.h): the
# reference is IPv4-only, and "v4" (the default) is exactly its masks.
FAMILIES = {"v4": 0, "v6": 1, "auto": 2}


def _fam(family: str) -> int:
    try:
        return FAMILIES[family]
    except KeyError:
        raise ValueError(f"family must be one of {sorted(FAMILIES)}, not {family!r}") from None


def icrc(pkt, family: str = "v4") -> int:
    """ICRC of one L3 RoCEv2 packet (bytes / bytearray / memoryview / uint8 array).

    Wire trailer = little-endian bytes of the result (shuffle_egress.p4:493).
    ``family``: "v4" (the reference's IPv4 masks), "v6" (RoCEv2 over IPv6) or
    "auto" (per packet from the IP version nibble)."""
    p, n, _keep = _buf(pkt)
    if n < 4:
        raise ValueError("packet shorter than the 4-byte ICRC trailer")
    return int(lib.ricrc_one_ex(p, n, _fam(family)))


def verify(pkt, family: str = "v4") -> bool:
    """True iff the packet's trailer carries its ICRC (what a NIC checks)."""
    p, n, _keep = _buf(pkt)
    rc = lib.ricrc_verify_one_ex(p, n, _fam(family))
    if rc < 0:
        raise ICRCError(rc, "ricrc_verify_one_ex")
    return rc == 1


def stamp(pkt: bytearray, family: str = "v4") -> bytearray:
    """Write the ICRC into the trailer of a mutable packet, in place; returns it."""
    if not isinstance(pkt, (bytearray, memoryview, np.ndarray)):
        raise TypeError("stamp() needs a mutable buffer (bytearray / memoryview / uint8 array)")
    p, n, _keep = _buf(pkt)
    rc = lib.ricrc_stamp_one_ex(p, n, _fam(family))
    if rc < 0:
        raise ICRCError(rc, "ricrc_stamp_one_ex")
    return pkt


def classify(pkt) -> int:
    """4 (RoCEv2 over IPv4), 6 (RoCEv2 over IPv6) or 0."""
    p, n, _keep = _buf(pkt)
    return int(lib.ricrc_classify(p, n))


def repair(pkt, off: int, old_bytes, old_icrc: int, family: str = "v4") -> int:
    """ICRC of ``pkt`` (already rewritten) from its pre-rewrite ICRC, given the
    old contents of the rewritten range [off, off + len(old_bytes)): O(len)."""
    p, n, _keep = _buf(pkt)
    q, m, _keep2 = _buf(bytes(old_bytes))
    out = ctypes.c_uint32()
    rc = lib.ricrc_repair_one(p, n, off, q, m, old_icrc & 0xFFFFFFFF, _fam(family), ctypes.byref(out))
    if rc < 0:
        raise ICRCError(rc, "ricrc_repair_one")
    return int(out.value)


def is_rocev2(pkt) -> bool:
    p, n, _keep = _buf(pkt)
    return lib.ricrc_is_rocev2(p, n) == 1


def shift(reg: int, nbytes: int) -> int:
    """CRC register advanced over ``nbytes`` zero bytes (GF(2) x^(8n))."""
    return int(lib.ricrc_shift(reg & 0xFFFFFFFF, nbytes))


def combine(crc1: int, crc2: int, len2: int) -> int:
    """crc32(A || B) from crc32(A), crc32(B), len(B)."""
    return int(lib.ricrc_combine(crc1 & 0xFFFFFFFF, crc2 & 0xFFFFFFFF, len2))


# ------------------------------------------------------------------- batches
def _ptr(x):
    """Raw pointer of a torch tensor, numpy array, int or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(f"cannot take a pointer of {type(x)!r}")


def _stream_ptr(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


class Context:
    """GPU context: ``Context(n_gpus=-1)`` uses every visible device,
    ``Context(devices=[local_rank])`` one explicit device (one process per GPU).

    Raises :class:`ICRCError` (-ENODEV) when no GPU is available -- batches are
    never computed on the CPU."""

    def __init__(self, n_gpus: int = -1, devices=None):
        h = ctypes.c_void_p()
        if devices is not None:
            ids = (ctypes.c_int * len(devices))(*devices)
            rc = lib.ricrc_create_devices(ctypes.byref(h), ids, len(devices))
        else:
            rc = lib.ricrc_create(ctypes.byref(h), n_gpus)
        if rc:
            raise ICRCError(rc, "ricrc_create")
        self._h = h

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            lib.ricrc_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def device_count(self) -> int:
        return lib.ricrc_device_count(self._h)

    def stream(self, dev: int = 0) -> int:
        return lib.ricrc_stream(self._h, dev)

    # -- host in, host out ------------------------------------------------
    def batch_host(self, buf, offsets=None, lengths=None, stride: int = 0, l3_offset: int = 0,
                   count: int | None = None, family: str = "v4") -> np.ndarray:
        buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
        off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
        if count is None:
            count = len(off) if off is not None else (len(ln) if ln is not None else buf.size // stride)
        out = np.empty(count, dtype=np.uint32)
        rc = lib.ricrc_batch_host_ex(self._h, buf.ctypes.data, _ptr(off), _ptr(ln), stride, count,
                                     l3_offset, out.ctypes.data, _fam(family))
        if rc:
            raise ICRCError(rc, "ricrc_batch_host")
        return out

    # -- device resident --------------------------------------------------
    def batch_device(self, base, count: int, out, stride: int = 0, offsets=None, lengths=None,
                     l3_offset: int = 0, dev: int = 0, stream=None, verify: bool = False,
                     family: str = "v4") -> None:
        fn = lib.ricrc_verify_device_ex if verify else lib.ricrc_batch_device_ex
        rc = fn(self._h, dev, _ptr(base), _ptr(offsets), _ptr(lengths), stride, count, l3_offset,
                _ptr(out), _stream_ptr(stream), _fam(family))
        if rc:
            raise ICRCError(rc, "ricrc_verify_device" if verify else "ricrc_batch_device")

    def repair_device(self, base, count: int, off: int, old_bytes, out=None, stride: int = 0,
                      offsets=None, lengths=None, l3_offset: int = 0, old_stride: int | None = None,
                      family: str = "v4", stamp: bool = True, dev: int = 0, stream=None) -> None:
        """Incremental ICRC repair after a header rewrite (``ricrc_repair_device``):
        bytes ``[off, off + L)`` of packet i held ``old_bytes[i]`` (a ``count x L``
        uint8 device tensor) when its trailer was stamped.  ``out[i]`` = the new
        ICRC; with ``stamp`` the trailer is rewritten too."""
        ln = int(old_bytes.shape[-1]) if getattr(old_bytes, "ndim", 1) > 1 else int(old_bytes.numel() // max(count, 1))
        if old_stride is None:
            old_stride = ln
        rc = lib.ricrc_repair_device(self._h, dev, _ptr(base), _ptr(offsets), _ptr(lengths), stride, count,
                                     l3_offset, off, ln, _ptr(old_bytes), old_stride, _fam(family),
                                     1 if stamp else 0, _ptr(out), _stream_ptr(stream))
        if rc:
            raise ICRCError(rc, "ricrc_repair_device")

    def synth_device(self, buf, seed: int, first: int, count: int, n: int, stride: int | None = None,
                     dev: int = 0, stream=None) -> None:
        rc = lib.ricrc_synth_device(self._h, dev, seed, first, count, n, stride or n, _ptr(buf),
                                    _stream_ptr(stream))
        if rc:
            raise ICRCError(rc, "ricrc_synth_device")

    def host_alloc(self, nbytes: int) -> np.ndarray:
        """Pinned host buffer (uint8 array); freed with :meth:`host_free`."""
        p = lib.ricrc_host_alloc(self._h, nbytes)
        if not p:
            raise ICRCError(-errno.ENOMEM, "ricrc_host_alloc")
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
        return arr

    def host_free(self, arr: np.ndarray) -> None:
        lib.ricrc_host_free(self._h, arr.ctypes.data)

    def host_register(self, arr: np.ndarray) -> None:
        """Pin an existing contiguous host array (a NIC ring) so host batches
        read it by DMA; undo with :meth:`host_unregister`."""
        if not arr.flags["C_CONTIGUOUS"]:
            raise ValueError("host_register needs a contiguous array")
        rc = lib.ricrc_host_register(self._h, arr.ctypes.data, arr.nbytes)
        if rc:
            raise ICRCError(rc, "ricrc_host_register")

    def host_unregister(self, arr: np.ndarray) -> None:
        rc = lib.ricrc_host_unregister(self._h, arr.ctypes.data)
        if rc:
            raise ICRCError(rc, "ricrc_host_unregister")


def icrc_batch(buf, offsets=None, lengths=None, stride: int = 0, l3_offset: int = 0,
               ctx: Context | None = None) -> np.ndarray:
    """Convenience: host batch through a (temporary) all-GPU context."""
    own = ctx is None
    ctx = ctx or Context()
    try:
        return ctx.batch_host(buf, offsets, lengths, stride, l3_offset)
    finally:
        if own:
            ctx.close()
