"""roce_icrc -- Python mirror of libroceicrc, the MI355X RoCEv2 ICRC engine.

This is the host-side interface a caller such as the reference's
``python/simulator.py`` binds through ctypes (the reference has no FFI of its
own for this path; see include/roce_icrc.h and INTEGRATION.md):

* :func:`icrc` / :func:`verify` / :func:`stamp` -- one packet at a time
  (the simulator's wire crossings, simulator.py:49-55 and 59-82); CPU,
  re-entrant, no GPU launch per 60-byte packet.  These bind
  ``libroceicrc_cpu.so``, the HIP-free build of the per-packet entry points:
  importing this package needs neither ROCm nor torch.
* :class:`Context` -- batches on the GPUs through ``libroceicrc.so`` (gfx950
  kernels + RCCL): host buffers in/out (``batch_host``), device-resident
  buffers (``batch_device`` / ``verify_device``, torch tensors or raw
  pointers, async on a stream), single-process multi-GPU sharding with an
  RCCL all-gather (``batch_device_all``) and the synthetic batch generators
  used by bench.py and the tests.

Every batch call runs the gfx950 kernels; there is no CPU fallback: if the
HIP library is missing, creating a :class:`Context` (or touching
``roce_icrc.lib``) raises.
"""
from __future__ import annotations

import ctypes
import errno
import os

import numpy as np

from . import wire  # noqa: F401  (Packet <-> bytes adapter)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libroceicrc.so")
CPU_LIB_PATH = os.path.join(_HERE, "libroceicrc_cpu.so")

MIN_LEN = 44
MAX_LEN = 65535

# Per-packet CPU section of include/roce_icrc.h: in both libraries.
CPU_EXPORTED = (
    "ricrc_one", "ricrc_verify_one", "ricrc_stamp_one", "ricrc_is_rocev2", "ricrc_shift",
    "ricrc_one_ex", "ricrc_verify_one_ex", "ricrc_stamp_one_ex", "ricrc_classify", "ricrc_repair_one",
    "ricrc_combine", "ricrc_icrc", "ricrc_strerror", "ricrc_batch_cpu", "ricrc_allgather_plan",
)
EXPORTED = CPU_EXPORTED + (
    "ricrc_create", "ricrc_create_devices", "ricrc_destroy", "ricrc_device_count", "ricrc_batch_host",
    "ricrc_batch_device", "ricrc_verify_device", "ricrc_repair_device", "ricrc_batch_host_ex",
    "ricrc_batch_device_ex", "ricrc_verify_device_ex", "ricrc_host_alloc", "ricrc_host_free",
    "ricrc_host_register", "ricrc_host_unregister", "ricrc_synth_device", "ricrc_synth_ragged_device",
    "ricrc_prime", "ricrc_stream", "ricrc_comm_init", "ricrc_batch_device_all", "ricrc_allgather", "ricrc_sync",
    "ricrc_batch_device_st", "ricrc_batch_host_st", "ricrc_classify_device", "ricrc_kernel_path",
    "ricrc_pass_times", "ricrc_launch_info", "ricrc_batch_device_bounded", "ricrc_batch_host_bounded",
)

# Per-packet status of the *_st batch calls (include/roce_icrc.h).
ST_OK, ST_BADLEN, ST_NOTROCE = 0, 1, 2
F_STRICT, F_VERIFY, F_FRAMELEN = 0x100, 0x200, 0x400

_vp = ctypes.c_void_p
_u32, _u64, _i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
_PP = ctypes.POINTER(ctypes.c_void_p)
_SIG = {
    "ricrc_one": ([_vp, _u32], _u32),
    "ricrc_verify_one": ([_vp, _u32], _i32),
    "ricrc_stamp_one": ([_vp, _u32], _i32),
    "ricrc_is_rocev2": ([_vp, _u32], _i32),
    "ricrc_one_ex": ([_vp, _u32, _u32], _u32),
    "ricrc_verify_one_ex": ([_vp, _u32, _u32], _i32),
    "ricrc_stamp_one_ex": ([_vp, _u32, _u32], _i32),
    "ricrc_classify": ([_vp, _u32], _i32),
    "ricrc_repair_one": ([_vp, _u32, _u32, _vp, _u32, _u32, _u32, ctypes.POINTER(_u32)], _i32),
    "ricrc_icrc": ([_vp, _u32, _u32, ctypes.POINTER(_u32)], _i32),
    "ricrc_shift": ([_u32, _u64], _u32),
    "ricrc_combine": ([_u32, _u32, _u64], _u32),
    "ricrc_strerror": ([_i32], ctypes.c_char_p),
    "ricrc_batch_cpu": ([_vp, _vp, _vp, _u32, _u64, _u32, _vp, _u32, _i32], _i32),
    "ricrc_allgather_plan": ([_i32, _vp, _vp, _i32], _i32),
    "ricrc_create": ([ctypes.POINTER(_vp), _i32], _i32),
    "ricrc_create_devices": ([ctypes.POINTER(_vp), ctypes.POINTER(_i32), _i32], _i32),
    "ricrc_destroy": ([_vp], None),
    "ricrc_device_count": ([_vp], _i32),
    "ricrc_batch_host": ([_vp, _vp, _vp, _vp, _u32, _u64, _u32, _vp], _i32),
    "ricrc_batch_device": ([_vp, _i32, _vp, _vp, _vp, _u32, _u64, _u32, _vp, _vp], _i32),
    "ricrc_verify_device": ([_vp, _i32, _vp, _vp, _vp, _u32, _u64, _u32, _vp, _vp], _i32),
    "ricrc_batch_host_ex": ([_vp, _vp, _vp, _vp, _u32, _u64, _u32, _vp, _u32], _i32),
    "ricrc_batch_device_ex": ([_vp, _i32, _vp, _vp, _vp, _u32, _u64, _u32, _vp, _vp, _u32], _i32),
    "ricrc_verify_device_ex": ([_vp, _i32, _vp, _vp, _vp, _u32, _u64, _u32, _vp, _vp, _u32], _i32),
    "ricrc_repair_device": ([_vp, _i32, _vp, _vp, _vp, _u32, _u64, _u32, _u32, _u32, _vp, _u32, _u32, _u32, _vp, _vp],
                            _i32),
    "ricrc_host_alloc": ([_vp, _u64], _vp),
    "ricrc_host_free": ([_vp, _vp], None),
    "ricrc_host_register": ([_vp, _vp, _u64], _i32),
    "ricrc_host_unregister": ([_vp, _vp], _i32),
    "ricrc_synth_device": ([_vp, _i32, _u64, _u64, _u64, _u32, _u32, _vp, _vp], _i32),
    "ricrc_synth_ragged_device": ([_vp, _i32, _u64, _u64, _u64, _vp, _vp, _vp, _vp], _i32),
    "ricrc_prime": ([_vp, _i32, _u32], _i32),
    "ricrc_stream": ([_vp, _i32], _vp),
    "ricrc_comm_init": ([_vp], _i32),
    "ricrc_batch_device_all": ([_vp, _PP, _PP, _PP, _u32, ctypes.POINTER(_u64), _u32, _PP, _u32], _i32),
    "ricrc_allgather": ([_vp, ctypes.POINTER(_u64), _PP], _i32),
    "ricrc_sync": ([_vp], _i32),
    "ricrc_batch_device_st": ([_vp, _i32, _vp, _vp, _vp, _u32, _u64, _u32, _vp, _vp, _vp, _u32], _i32),
    "ricrc_batch_host_st": ([_vp, _vp, _vp, _vp, _u32, _u64, _u32, _vp, _vp, _u32], _i32),
    "ricrc_classify_device": ([_vp, _i32, _vp, _vp, _vp, _u32, _u64, _u32, _vp, _vp], _i32),
    "ricrc_kernel_path": ([_vp, _vp, _vp, _vp, _u32, _u64, _u32, _u32], ctypes.c_char_p),
    "ricrc_pass_times": ([_vp, _i32, ctypes.POINTER(ctypes.c_float), _i32], _i32),
    "ricrc_launch_info": ([_vp, _i32, _vp, _vp, _vp, _u32, _u64, _u32, _vp], _i32),
    "ricrc_batch_device_bounded": ([_vp, _i32, _vp, _u64, _vp, _vp, _u32, _u64, _u32, _vp, _vp, _vp, _u32], _i32),
    "ricrc_batch_host_bounded": ([_vp, _vp, _u64, _vp, _vp, _u32, _u64, _u32, _vp, _vp, _u32], _i32),
}


class LaunchInfo(ctypes.Structure):
    """``ricrc_launch_info_t`` (include/roce_icrc.h)."""
    _fields_ = [("grid", _u32), ("xcd_weights", _u32 * 8), ("start_xcd", _u32), ("pass_grid", _u32),
                ("pass_unroll", _u32), ("one_line", _u32), ("gather_grid", _u32), ("lanes_per_packet", _u32)]


class ICRCError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        super().__init__(f"{what}: {rc} ({_strerror(rc)})")


def _bind(L, names):
    for name in names:
        args, res = _SIG[name]
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


def _load_cpu():
    if not os.path.exists(CPU_LIB_PATH):
        raise ImportError(
            f"libroceicrc_cpu.so not found at {CPU_LIB_PATH}; build it with "
            "`make -C roce-test_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
    return _bind(ctypes.CDLL(CPU_LIB_PATH), CPU_EXPORTED)


def _load_hip():
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
    return _bind(ctypes.CDLL(LIB_PATH), EXPORTED)


cpu = _load_cpu()
_hip = None


def hip_lib():
    """libroceicrc.so (gfx950 kernels + runtime), loaded on first use."""
    global _hip
    if _hip is None:
        _hip = _load_hip()
    return _hip


def __getattr__(name):  # roce_icrc.lib: the full HIP library, loaded lazily
    if name == "lib":
        return hip_lib()
    raise AttributeError(name)


def _strerror(rc: int) -> str:
    return cpu.ricrc_strerror(rc).decode()


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
    return int(cpu.ricrc_one_ex(p, n, _fam(family)))


def verify(pkt, family: str = "v4") -> bool:
    """True iff the packet's trailer carries its ICRC (what a NIC checks)."""
    p, n, _keep = _buf(pkt)
    rc = cpu.ricrc_verify_one_ex(p, n, _fam(family))
    if rc < 0:
        raise ICRCError(rc, "ricrc_verify_one_ex")
    return rc == 1


def stamp(pkt: bytearray, family: str = "v4") -> bytearray:
    """Write the ICRC into the trailer of a mutable packet, in place; returns it."""
    if not isinstance(pkt, (bytearray, memoryview, np.ndarray)):
        raise TypeError("stamp() needs a mutable buffer (bytearray / memoryview / uint8 array)")
    p, n, _keep = _buf(pkt)
    rc = cpu.ricrc_stamp_one_ex(p, n, _fam(family))
    if rc < 0:
        raise ICRCError(rc, "ricrc_stamp_one_ex")
    return pkt


def classify(pkt) -> int:
    """4 (RoCEv2 over IPv4), 6 (RoCEv2 over IPv6) or 0."""
    p, n, _keep = _buf(pkt)
    return int(cpu.ricrc_classify(p, n))


def repair(pkt, off: int, old_bytes, old_icrc: int, family: str = "v4") -> int:
    """ICRC of ``pkt`` (already rewritten) from its pre-rewrite ICRC, given the
    old contents of the rewritten range [off, off + len(old_bytes)): O(len)."""
    p, n, _keep = _buf(pkt)
    q, m, _keep2 = _buf(bytes(old_bytes))
    out = ctypes.c_uint32()
    rc = cpu.ricrc_repair_one(p, n, off, q, m, old_icrc & 0xFFFFFFFF, _fam(family), ctypes.byref(out))
    if rc < 0:
        raise ICRCError(rc, "ricrc_repair_one")
    return int(out.value)


def icrc_checked(pkt, family: str = "v4", strict: bool = False, framelen: bool = False) -> int:
    """``ricrc_icrc``: like :func:`icrc` but with the length contract
    (MIN_LEN..MAX_LEN, else ValueError) and, with ``strict``, the RoCEv2
    classifier (not RoCEv2 of that family -> ValueError).  ``framelen``
    (RICRC_F_FRAMELEN): ``pkt`` runs from the L3 header to the end of its
    Ethernet frame (padding, FCS) and the packet's length is its IP header's."""
    p, n, _keep = _buf(pkt)
    out = ctypes.c_uint32()
    flags = _fam(family) | (F_STRICT if strict else 0) | (F_FRAMELEN if framelen else 0)
    rc = cpu.ricrc_icrc(p, n, flags, ctypes.byref(out))
    if rc < 0:
        raise ValueError(f"ricrc_icrc: {rc} ({_strerror(rc)})")
    return int(out.value)


def is_rocev2(pkt) -> bool:
    p, n, _keep = _buf(pkt)
    return cpu.ricrc_is_rocev2(p, n) == 1


def shift(reg: int, nbytes: int) -> int:
    """CRC register advanced over ``nbytes`` zero bytes (GF(2) x^(8n))."""
    return int(cpu.ricrc_shift(reg & 0xFFFFFFFF, nbytes))


def combine(crc1: int, crc2: int, len2: int) -> int:
    """crc32(A || B) from crc32(A), crc32(B), len(B)."""
    return int(cpu.ricrc_combine(crc1 & 0xFFFFFFFF, crc2 & 0xFFFFFFFF, len2))


def icrc_batch_cpu(buf, offsets=None, lengths=None, stride: int = 0, l3_offset: int = 0, count: int | None = None,
                   family: str = "v4", threads: int = 1, framelen: bool = False) -> np.ndarray:
    """``ricrc_batch_cpu``: a batch on the host CPU (slice-by-16, ``threads``
    threads) -- no GPU involved, and never used by the GPU batch calls."""
    buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
    if count is None:
        count = len(off) if off is not None else (len(ln) if ln is not None else buf.size // stride)
    out = np.empty(count, dtype=np.uint32)
    rc = cpu.ricrc_batch_cpu(buf.ctypes.data, _ptr(off), _ptr(ln), stride, count, l3_offset, out.ctypes.data,
                             _fam(family) | (F_FRAMELEN if framelen else 0), threads)
    if rc:
        raise ICRCError(rc, "ricrc_batch_cpu")
    return out


class Xfer(ctypes.Structure):
    """One RCCL call of the all-gather plan (``ricrc_xfer``)."""
    _fields_ = [("dev", ctypes.c_int32), ("kind", ctypes.c_int32), ("peer", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("offset", ctypes.c_uint64), ("count", ctypes.c_uint64)]


XFER_ALLGATHER, XFER_SEND, XFER_RECV = 0, 1, 2


def allgather_plan(counts) -> list:
    """``ricrc_allgather_plan``: the RCCL calls ricrc_batch_device_all issues
    for these per-device shard counts, as (dev, kind, peer, offset, count)."""
    cnt = (ctypes.c_uint64 * len(counts))(*[int(c) for c in counts])
    need = cpu.ricrc_allgather_plan(len(counts), cnt, None, 0)
    if need < 0:
        raise ICRCError(need, "ricrc_allgather_plan")
    ops = (Xfer * max(need, 1))()
    cpu.ricrc_allgather_plan(len(counts), cnt, ops, need)
    return [(x.dev, x.kind, x.peer, x.offset, x.count) for x in ops[:need]]


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
        self._lib = lib = hip_lib()
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
            hip_lib().ricrc_destroy(self._h)
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
        return self._lib.ricrc_device_count(self._h)

    def stream(self, dev: int = 0) -> int:
        return self._lib.ricrc_stream(self._h, dev)

    # -- host in, host out ------------------------------------------------
    def batch_host(self, buf, offsets=None, lengths=None, stride: int = 0, l3_offset: int = 0,
                   count: int | None = None, family: str = "v4") -> np.ndarray:
        buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
        off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
        if count is None:
            count = len(off) if off is not None else (len(ln) if ln is not None else buf.size // stride)
        out = np.empty(count, dtype=np.uint32)
        rc = self._lib.ricrc_batch_host_ex(self._h, buf.ctypes.data, _ptr(off), _ptr(ln), stride, count,
                                     l3_offset, out.ctypes.data, _fam(family))
        if rc:
            raise ICRCError(rc, "ricrc_batch_host")
        return out

    def batch_host_st(self, buf, offsets=None, lengths=None, stride: int = 0, l3_offset: int = 0,
                      count: int | None = None, family: str = "v4", strict: bool = False,
                      verify: bool = False, framelen: bool = False):
        """``ricrc_batch_host_st``: ``(out, status)`` -- a status per packet
        (:data:`ST_OK`, :data:`ST_BADLEN`, :data:`ST_NOTROCE`) instead of
        failing the call on a bad descriptor length; with ``strict`` only
        packets the reference's ingress parser accepts as RoCEv2 get an ICRC
        (shuffle_ingress_parser.p4:12-36); ``out[i] = 0`` where status != OK."""
        buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
        off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
        if count is None:
            count = len(off) if off is not None else (len(ln) if ln is not None else buf.size // stride)
        out = np.empty(count, dtype=np.uint32)
        st = np.empty(count, dtype=np.uint8)
        flags = _fam(family) | (F_STRICT if strict else 0) | (F_VERIFY if verify else 0) | (F_FRAMELEN if framelen else 0)
        rc = self._lib.ricrc_batch_host_st(self._h, buf.ctypes.data, _ptr(off), _ptr(ln), stride, count,
                                           l3_offset, out.ctypes.data, st.ctypes.data, flags)
        if rc:
            raise ICRCError(rc, "ricrc_batch_host_st")
        return out, st

    def batch_host_bounded(self, buf, base_bytes: int, offsets=None, lengths=None, stride: int = 0,
                           l3_offset: int = 0, count: int | None = None, family: str = "v4", status: bool = False,
                           strict: bool = False, verify: bool = False, framelen: bool = False):
        """``ricrc_batch_host_bounded``: descriptors checked against the first
        ``base_bytes`` of ``buf`` -- ``out`` (``status=False``: a packet outside
        raises ICRCError -EINVAL) or ``(out, status)`` (outside: ST_BADLEN)."""
        buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
        off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
        if count is None:
            count = len(off) if off is not None else (len(ln) if ln is not None else buf.size // stride)
        out = np.empty(count, dtype=np.uint32)
        st = np.empty(count, dtype=np.uint8) if status else None
        flags = _fam(family) | (F_STRICT if strict else 0) | (F_VERIFY if verify else 0) | (F_FRAMELEN if framelen else 0)
        rc = self._lib.ricrc_batch_host_bounded(self._h, buf.ctypes.data, base_bytes, _ptr(off), _ptr(ln), stride,
                                                count, l3_offset, out.ctypes.data,
                                                st.ctypes.data if st is not None else None, flags)
        if rc:
            raise ICRCError(rc, "ricrc_batch_host_bounded")
        return (out, st) if status else out

    # -- device resident --------------------------------------------------
    def batch_device(self, base, count: int, out, stride: int = 0, offsets=None, lengths=None,
                     l3_offset: int = 0, dev: int = 0, stream=None, verify: bool = False,
                     family: str = "v4") -> None:
        fn = self._lib.ricrc_verify_device_ex if verify else self._lib.ricrc_batch_device_ex
        rc = fn(self._h, dev, _ptr(base), _ptr(offsets), _ptr(lengths), stride, count, l3_offset,
                _ptr(out), _stream_ptr(stream), _fam(family))
        if rc:
            raise ICRCError(rc, "ricrc_verify_device" if verify else "ricrc_batch_device")

    def batch_device_st(self, base, count: int, out, status, stride: int = 0, offsets=None, lengths=None,
                        l3_offset: int = 0, dev: int = 0, stream=None, family: str = "v4",
                        strict: bool = False, verify: bool = False, framelen: bool = False) -> None:
        """``ricrc_batch_device_st``: as :meth:`batch_device`, plus ``status``
        (``count`` uint8 on the device, :data:`ST_OK` / :data:`ST_BADLEN` /
        :data:`ST_NOTROCE`).  ``framelen``: RICRC_F_FRAMELEN (descriptor
        lengths are frame extents past L3; packet lengths from the IP headers)."""
        flags = _fam(family) | (F_STRICT if strict else 0) | (F_VERIFY if verify else 0) | (F_FRAMELEN if framelen else 0)
        rc = self._lib.ricrc_batch_device_st(self._h, dev, _ptr(base), _ptr(offsets), _ptr(lengths), stride, count,
                                             l3_offset, _ptr(out), _ptr(status), _stream_ptr(stream), flags)
        if rc:
            raise ICRCError(rc, "ricrc_batch_device_st")

    def batch_device_bounded(self, base, base_bytes: int, count: int, out, status, stride: int = 0, offsets=None,
                             lengths=None, l3_offset: int = 0, dev: int = 0, stream=None, family: str = "v4",
                             strict: bool = False, verify: bool = False, framelen: bool = False) -> None:
        """``ricrc_batch_device_bounded``: as :meth:`batch_device_st`, packets
        outside ``[base, base + base_bytes)`` never read (ST_BADLEN, out 0)."""
        flags = _fam(family) | (F_STRICT if strict else 0) | (F_VERIFY if verify else 0) | (F_FRAMELEN if framelen else 0)
        rc = self._lib.ricrc_batch_device_bounded(self._h, dev, _ptr(base), base_bytes, _ptr(offsets), _ptr(lengths),
                                                  stride, count, l3_offset, _ptr(out), _ptr(status),
                                                  _stream_ptr(stream), flags)
        if rc:
            raise ICRCError(rc, "ricrc_batch_device_bounded")

    def classify_device(self, base, count: int, cls, stride: int = 0, offsets=None, lengths=None,
                        l3_offset: int = 0, dev: int = 0, stream=None) -> None:
        """``ricrc_classify_device``: ``cls[i]`` = 4 / 6 / 0 (uint8 on the device)."""
        rc = self._lib.ricrc_classify_device(self._h, dev, _ptr(base), _ptr(offsets), _ptr(lengths), stride, count,
                                             l3_offset, _ptr(cls), _stream_ptr(stream))
        if rc:
            raise ICRCError(rc, "ricrc_classify_device")

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
        rc = self._lib.ricrc_repair_device(self._h, dev, _ptr(base), _ptr(offsets), _ptr(lengths), stride, count,
                                     l3_offset, off, ln, _ptr(old_bytes), old_stride, _fam(family),
                                     1 if stamp else 0, _ptr(out), _stream_ptr(stream))
        if rc:
            raise ICRCError(rc, "ricrc_repair_device")

    def synth_device(self, buf, seed: int, first: int, count: int, n: int, stride: int | None = None,
                     dev: int = 0, stream=None) -> None:
        rc = self._lib.ricrc_synth_device(self._h, dev, seed, first, count, n, stride or n, _ptr(buf),
                                    _stream_ptr(stream))
        if rc:
            raise ICRCError(rc, "ricrc_synth_device")

    def synth_ragged_device(self, buf, seed: int, first: int, count: int, offsets, lengths,
                            dev: int = 0, stream=None) -> None:
        """Packet k = global packet ``first + k`` (the bytes :meth:`synth_device`
        makes for that index and length) at ``buf + offsets[k]`` (device arrays)."""
        rc = self._lib.ricrc_synth_ragged_device(self._h, dev, seed, first, count, _ptr(offsets), _ptr(lengths),
                                                 _ptr(buf), _stream_ptr(stream))
        if rc:
            raise ICRCError(rc, "ricrc_synth_ragged_device")

    def pass_times(self, dev: int = 0):
        """``ricrc_pass_times`` (RICRC_PASS_TIMES set at creation): (calls,
        summed ms of the ragged pipeline's bucket, fold, one-line and gather
        passes since the last query)."""
        ms = (ctypes.c_float * 4)()
        rc = self._lib.ricrc_pass_times(self._h, dev, ms, 4)
        if rc < 0:
            raise ICRCError(rc, "ricrc_pass_times")
        return rc, [float(v) for v in ms]

    def launch_info(self, base, count: int, stride: int = 0, offsets=None, lengths=None, l3_offset: int = 0,
                    dev: int = 0) -> dict:
        """``ricrc_launch_info``: how the dispatch would launch this batch on
        ``dev`` -- the main kernel's grid, its per-XCD work-split weights, the
        recorded start XCD, and the ragged passes' shape."""
        info = LaunchInfo()
        rc = self._lib.ricrc_launch_info(self._h, dev, _ptr(base), _ptr(offsets), _ptr(lengths), stride, count,
                                         l3_offset, ctypes.byref(info))
        if rc:
            raise ICRCError(rc, "ricrc_launch_info")
        return _launch_dict(info)

    def prime(self, usec: int = 20000, dev: int = 0) -> None:
        """``ricrc_prime``: bring the device out of its idle power state."""
        rc = self._lib.ricrc_prime(self._h, dev, usec)
        if rc:
            raise ICRCError(rc, "ricrc_prime")

    # -- one process, all context devices, RCCL ---------------------------
    def comm_init(self) -> None:
        rc = self._lib.ricrc_comm_init(self._h)
        if rc:
            raise ICRCError(rc, "ricrc_comm_init")

    def batch_device_all(self, bases, counts, outs, stride: int = 0, offsets=None, lengths=None,
                         l3_offset: int = 0, family: str = "v4") -> None:
        """``ricrc_batch_device_all``: shard k on context device k, every
        ``outs[k]`` (``sum(counts)`` int32 on device k) ends with all ICRCs in
        shard order.  Asynchronous on the context streams: :meth:`sync`."""
        n = len(bases)
        arr = lambda xs: None if xs is None else (ctypes.c_void_p * n)(*[_ptr(x) for x in xs])  # noqa: E731
        cnt = (ctypes.c_uint64 * n)(*[int(c) for c in counts])
        rc = self._lib.ricrc_batch_device_all(self._h, arr(bases), arr(offsets), arr(lengths), stride, cnt,
                                              l3_offset, arr(outs), _fam(family))
        if rc:
            raise ICRCError(rc, "ricrc_batch_device_all")

    def allgather(self, counts, outs) -> None:
        n = len(outs)
        cnt = (ctypes.c_uint64 * n)(*[int(c) for c in counts])
        rc = self._lib.ricrc_allgather(self._h, cnt, (ctypes.c_void_p * n)(*[_ptr(x) for x in outs]))
        if rc:
            raise ICRCError(rc, "ricrc_allgather")

    def sync(self) -> None:
        rc = self._lib.ricrc_sync(self._h)
        if rc:
            raise ICRCError(rc, "ricrc_sync")

    def host_alloc(self, nbytes: int) -> np.ndarray:
        """Pinned host buffer (uint8 array); freed with :meth:`host_free`."""
        p = self._lib.ricrc_host_alloc(self._h, nbytes)
        if not p:
            raise ICRCError(-errno.ENOMEM, "ricrc_host_alloc")
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
        return arr

    def host_free(self, arr: np.ndarray) -> None:
        self._lib.ricrc_host_free(self._h, arr.ctypes.data)

    def host_register(self, arr: np.ndarray) -> None:
        """Pin an existing contiguous host array (a NIC ring) so host batches
        read it by DMA; undo with :meth:`host_unregister`."""
        if not arr.flags["C_CONTIGUOUS"]:
            raise ValueError("host_register needs a contiguous array")
        rc = self._lib.ricrc_host_register(self._h, arr.ctypes.data, arr.nbytes)
        if rc:
            raise ICRCError(rc, "ricrc_host_register")

    def host_unregister(self, arr: np.ndarray) -> None:
        rc = self._lib.ricrc_host_unregister(self._h, arr.ctypes.data)
        if rc:
            raise ICRCError(rc, "ricrc_host_unregister")


def _launch_dict(info: LaunchInfo) -> dict:
    d = {"grid": info.grid, "xcd_weights": list(info.xcd_weights), "start_xcd": info.start_xcd,
         "lanes_per_packet": info.lanes_per_packet}
    if info.pass_grid:
        d.update(pass_grid=info.pass_grid, pass_unroll=info.pass_unroll,
                 one_line_in=("kernel", "gather", "fold")[info.one_line], gather_grid=info.gather_grid)
    elif info.one_line == 2:  # the workgroup-local ragged kernel: one launch, no bucket / gather passes
        d.update(one_line_in="fold", passes=1)
    return d


def launch_info(base, count: int, stride: int = 0, offsets=None, lengths=None, l3_offset: int = 0) -> dict:
    """``ricrc_launch_info`` without a context: how the dispatch launches a
    batch of this shape on a 256-CU MI355X (default knobs; no GPU needed)."""
    info = LaunchInfo()
    rc = hip_lib().ricrc_launch_info(None, 0, _ptr(base), _ptr(offsets), _ptr(lengths), stride, count, l3_offset,
                                     ctypes.byref(info))
    if rc:
        raise ICRCError(rc, "ricrc_launch_info")
    return _launch_dict(info)


def kernel_path(base, count: int, stride: int = 0, offsets=None, lengths=None, l3_offset: int = 0,
                family: str = "v4", ctx: Context | None = None) -> str:
    """``ricrc_kernel_path``: the '+'-joined gfx950 kernel names the batch
    dispatch launches for a batch of this shape (``base`` only for its
    alignment: a tensor, array or integer address).  No GPU needed."""
    addr = _ptr(base)
    r = hip_lib().ricrc_kernel_path(ctx.handle if ctx else None, addr, _ptr(offsets), _ptr(lengths), stride, count,
                                    l3_offset, _fam(family))
    if r is None:
        raise ValueError("ricrc_kernel_path: not a valid batch")
    return r.decode()


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
