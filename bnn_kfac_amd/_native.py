"""ctypes binding of libkfac_hip.so (the C ABI declared in include/kfac_hip.h).

The product path has NO fallback: if the library is missing, fails to load, or a
tensor is not on a HIP device, the calls below raise.  Device buffers are torch
tensors (the caching allocator owns them); the stream is torch's current stream
on the tensor's device, passed to every call explicitly.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BNN_KFAC_AMD_LIB", os.path.join(_HERE, "libkfac_hip.so"))

# enums (include/kfac_hip.h)
KFAC_OK, KFAC_EINVAL, KFAC_ELAUNCH, KFAC_EWORKSPACE = 0, -1, -2, -3
ROWMAJOR, CHANNEL, PATCH = 0, 1, 2
OUT_INV_CHOL, OUT_INVERSE = 0, 1
TRI_SYMMETRIC, TRI_LOWER = 0, 1
(PROF_FACTOR_TILES, PROF_FACTOR_REDUCE, PROF_INVERT, PROF_QUAD_TILES, PROF_FACTOR_SYRK3,
 PROF_FACTOR_X3, PROF_FACTOR_CONV, PROF_FACTOR_CHANNEL_SMALL, PROF_SYEV, PROF_FACTOR_CONV_X3,
 PROF_FACTOR_CONV_X3S, PROF_FACTOR_CONV_X3F, PROF_FACTOR_CHANNEL_X3) = range(13)
# profile slot -> the kernel family rocprofv3 names (kfac_prof_id, include/kfac_hip.h; the
# fp32 SYRK is the template kfac_factor_tiles_t<...>, named without the _t as in profiles/)
PROF_FACTOR_KERNELS = {PROF_FACTOR_TILES: "kfac_factor_tiles", PROF_FACTOR_SYRK3: "kfac_factor_syrk3",
                       PROF_FACTOR_X3: "kfac_factor_tiles_x3", PROF_FACTOR_CONV: "kfac_factor_conv",
                       PROF_FACTOR_CHANNEL_SMALL: "kfac_factor_channel_small",
                       PROF_FACTOR_CONV_X3: "kfac_factor_conv_x3", PROF_FACTOR_CONV_X3S: "kfac_factor_conv_x3s",
                       PROF_FACTOR_CONV_X3F: "kfac_factor_conv_x3f", PROF_FACTOR_CHANNEL_X3: "kfac_factor_channel_x3"}

c_i32, c_i64, c_f32, c_f64, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_void_p


class Operand(ctypes.Structure):
    _fields_ = [("ptr", c_vp), ("layout", c_i32), ("cols", c_i32), ("rows", c_i64),
                ("has_ones", c_i32), ("last_rows", c_i32), ("ld", c_i64), ("L", c_i64),
                ("sB", c_i64)] + [(f, c_i32) for f in
                                  ("C", "H", "W", "kh", "kw", "sh", "sw", "ph", "pw", "Ho", "Wo",
                                   "reserved1")]


class FactorJob(ctypes.Structure):
    _fields_ = [("x", Operand), ("alpha", c_f32), ("beta", c_f32), ("F", c_vp), ("ldF", c_i64),
                ("acc", c_vp), ("acc_splits", c_i32), ("acc_beta", c_f32),
                ("seg_ptrs", c_vp), ("nseg", c_i32), ("acc_stride", c_i32)]


class InvertJob(ctypes.Structure):
    _fields_ = [("F", c_vp), ("ldF", c_i64), ("n", c_i32), ("out_kind", c_i32),
                ("scale", c_f64), ("shift", c_f64), ("out", c_vp), ("ldo", c_i64)]


class EigJob(ctypes.Structure):
    _fields_ = [("F", c_vp), ("ldF", c_i64), ("n", c_i32), ("reserved", c_i32),
                ("evals", c_vp), ("evecs", c_vp), ("ldv", c_i64)]


class QuadJob(ctypes.Structure):
    _fields_ = [("J", c_vp), ("ldJ", c_i64), ("nA", c_i32), ("nG", c_i32), ("K1", c_vp),
                ("ld1", c_i64), ("K2", c_vp), ("ld2", c_i64), ("lower1", c_i32),
                ("lower2", c_i32), ("v", c_vp)]


class SampleJob(ctypes.Structure):
    _fields_ = [("LA", c_vp), ("ldA", c_i64), ("LG", c_vp), ("ldG", c_i64), ("Z", c_vp),
                ("nA", c_i32), ("nG", c_i32), ("W", c_vp), ("ldW", c_i64), ("bias", c_vp),
                ("wcols", c_i32), ("dense", c_i32)]


class EfbJob(ctypes.Structure):
    _fields_ = [("VA", c_vp), ("ldA", c_i64), ("VG", c_vp), ("ldG", c_i64), ("grad", c_vp),
                ("ld_grad", c_i64), ("state", c_vp), ("ld_state", c_i64), ("diag", c_vp),
                ("ld_diag", c_i64), ("nA", c_i32), ("nG", c_i32), ("accumulate", c_i32),
                ("scale", c_f32)]


class GramJob(ctypes.Structure):
    _fields_ = [("UA", c_vp), ("ldA", c_i64), ("UG", c_vp), ("ldG", c_i64), ("c", c_vp),
                ("sigma", c_vp), ("out", c_vp), ("ldo", c_i64), ("nA", c_i32), ("nG", c_i32),
                ("la", c_i32), ("lg", c_i32)]


class TriJob(ctypes.Structure):
    _fields_ = [("F", c_vp), ("ldF", c_i64), ("n", c_i32), ("reserved", c_i32), ("offset", c_i64)]


# symbol -> (restype, argtypes); every symbol include/kfac_hip.h declares
SIGNATURES = {
    "kfac_factor_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(FactorJob), ctypes.c_int]),
    "kfac_factor_update": (ctypes.c_int, [ctypes.POINTER(FactorJob), ctypes.c_int, c_vp,
                                          ctypes.c_size_t, c_vp]),
    "kfac_factor_accum_plan": (ctypes.c_int, [ctypes.POINTER(FactorJob), ctypes.c_int,
                                              ctypes.POINTER(c_i32), ctypes.POINTER(ctypes.c_size_t)]),
    "kfac_factor_flush": (ctypes.c_int, [ctypes.POINTER(FactorJob), ctypes.c_int, c_vp]),
    "kfac_syrk_linear": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, ctypes.c_int, c_f32, c_f32,
                                        c_vp, c_i64, c_vp, ctypes.c_size_t, c_vp]),
    "kfac_syrk_conv": (ctypes.c_int, [c_vp, c_i64] + [ctypes.c_int] * 10 + [c_f32, c_f32, c_vp,
                                                                            c_i64, c_vp,
                                                                            ctypes.c_size_t, c_vp]),
    "kfac_syrk_convgrad": (ctypes.c_int, [c_vp, c_i64, ctypes.c_int, c_i64, c_f32, c_f32, c_vp,
                                          c_i64, c_vp, ctypes.c_size_t, c_vp]),
    "kfac_invert_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(InvertJob), ctypes.c_int]),
    "kfac_invert": (ctypes.c_int, [ctypes.POINTER(InvertJob), ctypes.c_int, c_vp,
                                   ctypes.c_size_t, c_vp, c_vp]),
    "kfac_invert_ex": (ctypes.c_int, [ctypes.POINTER(InvertJob), ctypes.c_int, c_vp,
                                      ctypes.c_size_t, c_vp, c_vp, c_vp]),
    "kfac_damped_inv_chol": (ctypes.c_int, [c_vp, ctypes.c_int, c_i64, c_f64, c_f64, c_vp, c_i64,
                                            c_vp, ctypes.c_size_t, c_vp, c_vp]),
    "kfac_eig_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(EigJob), ctypes.c_int]),
    "kfac_syev": (ctypes.c_int, [ctypes.POINTER(EigJob), ctypes.c_int, c_vp, ctypes.c_size_t,
                                 c_vp, c_vp]),
    "kfac_quadform_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(QuadJob), ctypes.c_int,
                                                        c_i64]),
    "kfac_kron_quadform": (ctypes.c_int, [ctypes.POINTER(QuadJob), ctypes.c_int, c_i64,
                                          ctypes.c_int, c_vp, c_vp, ctypes.c_size_t, c_vp]),
    "kfac_sample_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(SampleJob), ctypes.c_int]),
    "kfac_sample": (ctypes.c_int, [ctypes.POINTER(SampleJob), ctypes.c_int, ctypes.c_int, c_vp,
                                   ctypes.c_size_t, c_vp]),
    "kfac_efb_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(EfbJob), ctypes.c_int]),
    "kfac_efb_update": (ctypes.c_int, [ctypes.POINTER(EfbJob), ctypes.c_int, c_vp, ctypes.c_size_t,
                                       c_vp]),
    "kfac_gram_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(GramJob), ctypes.c_int]),
    "kfac_kron_gram": (ctypes.c_int, [ctypes.POINTER(GramJob), ctypes.c_int, c_vp, ctypes.c_size_t,
                                      c_vp]),
    "kfac_tri_pack": (ctypes.c_int, [ctypes.POINTER(TriJob), ctypes.c_int, c_vp, c_vp]),
    "kfac_tri_unpack": (ctypes.c_int, [ctypes.POINTER(TriJob), ctypes.c_int, c_vp, ctypes.c_int, c_vp]),
    "kfac_profile_enable": (ctypes.c_int, [ctypes.c_int]),
    "kfac_profile_read": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_int64)]),
    "kfac_profile_read_work": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_double)]),
    "kfac_profile_reset": (ctypes.c_int, []),
    "kfac_set_knob": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "kfac_get_knob": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    "kfac_release": (ctypes.c_int, []),
    "kfac_invert_pipelined": (ctypes.c_int, [ctypes.POINTER(InvertJob), ctypes.c_int, c_vp, ctypes.c_size_t,
                                             c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "kfac_event_create": (ctypes.c_int, [ctypes.POINTER(c_vp)]),
    "kfac_event_create_ex": (ctypes.c_int, [ctypes.POINTER(c_vp), ctypes.c_int]),
    "kfac_event_destroy": (ctypes.c_int, [c_vp]),
    "kfac_event_record": (ctypes.c_int, [c_vp, c_vp]),
    "kfac_stream_wait_event": (ctypes.c_int, [c_vp, c_vp]),
    "kfac_event_query": (ctypes.c_int, [c_vp]),
    "kfac_event_synchronize": (ctypes.c_int, [c_vp]),
    "kfac_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "kfac_version": (ctypes.c_char_p, []),
}

_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def lib():
    """Load libkfac_hip.so (after torch, so the process shares torch's HIP runtime)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise NativeError(
                        f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                        f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
                handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
                for name, (res, args) in SIGNATURES.items():
                    fn = getattr(handle, name)
                    fn.restype = res
                    fn.argtypes = args
                _lib = handle
                # the library's cached hipGraphs / events go while the HIP runtime is
                # still up (Python's atexit runs before the C runtime's exit handlers)
                atexit.register(_release_at_exit)
    return _lib


def _release_at_exit():
    try:
        if _lib is not None and torch.cuda.is_initialized():
            for h in list(_raw_events):
                _lib.kfac_event_destroy(h)
            _raw_events.clear()
            _lib.kfac_release()
    except Exception:  # exiting anyway: never mask the process's own status
        pass


_raw_events = set()  # handles of the live RawEvents (what is left is destroyed at exit)


class RawEvent:
    """A HIP event owned through the C ABI (kfac_event_*): record / wait / query /
    synchronize are one ctypes call each, where torch.cuda.Event and Stream objects
    cost the caller's thread 5-10 us per call.  Created on `device` (default: the
    current HIP device), like torch.cuda.Event on its stream's device; destroyed by
    close() or when the last reference goes (the KFAC event pools hold them)."""
    __slots__ = ("handle", "ordering")

    def __init__(self, device=None, ordering=False):
        """`ordering`: the event only orders one stream after another on the device
        (kfac_event_create_ex flag 1: no system-scope fence); the host must not rely
        on it to see device writes after synchronize()."""
        h = ctypes.c_void_p()
        flags = 1 if ordering else 0
        if device is not None and torch.device(device).index is not None:
            with torch.cuda.device(device):
                check(lib().kfac_event_create_ex(ctypes.byref(h), flags), "kfac_event_create_ex")
        else:
            check(lib().kfac_event_create_ex(ctypes.byref(h), flags), "kfac_event_create_ex")
        self.handle = h.value
        self.ordering = ordering
        _raw_events.add(self.handle)

    def close(self):
        h, self.handle = self.handle, None
        if h is not None and h in _raw_events:
            _raw_events.discard(h)
            _lib.kfac_event_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # (interpreter shutdown: _release_at_exit owns what is left)
            pass

    def record(self, stream: int):
        check(_lib.kfac_event_record(self.handle, stream), "kfac_event_record")

    def wait_on(self, stream: int):
        """Order `stream`'s later work after this event's recorded work."""
        check(_lib.kfac_stream_wait_event(stream, self.handle), "kfac_stream_wait_event")

    def query(self) -> bool:
        r = _lib.kfac_event_query(self.handle)
        if r < 0:
            check(r, "kfac_event_query")
        return r == 1

    def synchronize(self):
        check(_lib.kfac_event_synchronize(self.handle), "kfac_event_synchronize")


def check(rc: int, what: str):
    if rc != KFAC_OK:
        msg = lib().kfac_strerror(rc).decode()
        raise NativeError(f"{what} failed: {msg} ({rc})")


def require_device(t: torch.Tensor, what: str, owner=None):
    """HIP device + fp32, or raise (no CPU fallback).  `owner` (e.g. the layer) is
    only formatted into the message on failure: this runs on every update."""
    if t.is_cuda and t.dtype == torch.float32:
        return
    where = f"{what} of {owner}" if owner is not None else what
    if not t.is_cuda:
        raise NativeError(f"bnn_kfac_amd runs on the MI355X only: {where} is on {t.device} "
                          f"(no CPU fallback; move the model/tensors to a HIP device)")
    raise TypeError(f"{where}: expected float32 (the reference computes in fp32), got {t.dtype}")


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(device: torch.device) -> int:
    """hipStream_t of torch's current stream on `device` (the raw query avoids
    building a Stream object per call)."""
    if _raw_stream is not None:
        return _raw_stream(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


class _Workspace:
    """Grow-only device scratch per (device, stream); stream order makes reuse safe."""

    def __init__(self):
        self._bufs = {}

    def get(self, device: torch.device, nbytes: int, stream: int = None, stream_obj=None) -> torch.Tensor:
        """`stream_obj`: the torch stream the work runs on when it is not the current one
        -- a (re)allocation is then made on it, so the caching allocator orders a grown
        buffer's release after that stream's queued work, not the current stream's."""
        key = (device.index, stream_handle(device) if stream is None else stream)
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            if stream_obj is not None:
                with torch.cuda.stream(stream_obj):
                    buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            else:
                buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            self._bufs[key] = buf
        return buf


workspace = _Workspace()
_info_bufs = {}  # (device, stream, jobs) -> the device verdict vector of kfac_invert


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def as_array(ctype, items):
    return (ctype * len(items))(*items)


# ------------------------------------------------------------------ op wrappers
def factor_update(jobs, device: torch.device):
    if not jobs:
        return
    L = lib()
    arr = as_array(FactorJob, jobs)
    need = L.kfac_factor_workspace_bytes(arr, len(jobs))
    stream = stream_handle(device)
    ws = workspace.get(device, need, stream)
    rc = L.kfac_factor_update(arr, len(jobs), ws.data_ptr(), ws.numel(), stream)
    if rc != KFAC_OK:
        check(rc, "kfac_factor_update")


def factor_accum_plan(jobs):
    """[(splits, bytes)] of each job's deferred-reduction accumulator."""
    arr = as_array(FactorJob, jobs)
    splits = (c_i32 * len(jobs))()
    nbytes = (ctypes.c_size_t * len(jobs))()
    check(lib().kfac_factor_accum_plan(arr, len(jobs), splits, nbytes), "kfac_factor_accum_plan")
    return list(zip(splits, nbytes))


def factor_flush(jobs, device: torch.device, stream: int = None):
    """kfac_factor_flush on torch's current stream, or on the raw HIP stream `stream`."""
    if jobs:
        check(lib().kfac_factor_flush(as_array(FactorJob, jobs), len(jobs),
                                      stream_handle(device) if stream is None else stream),
              "kfac_factor_flush")


def invert(jobs, device: torch.device, inputs_read=None) -> torch.Tensor:
    """Launch the grouped inversion on torch's current stream; returns the DEVICE info
    tensor (int32, one per job).  `inputs_read` (a torch.cuda.Event, optional) is
    recorded right after the launches that read the factors (kfac_invert_ex)."""
    L = lib()
    arr = as_array(InvertJob, jobs)
    need = L.kfac_invert_workspace_bytes(arr, len(jobs))
    stream = stream_handle(device)
    ws = workspace.get(device, need, stream)
    # a fresh verdict tensor per call (zeroed by kfac_invert): callers may hold several
    # calls' verdicts at once (the pooled buffer is only invert_pipelined's, whose
    # verdict is copied to host on the same stream before the buffer is written again)
    info = torch.empty(len(jobs), dtype=torch.int32, device=device)
    ev = None
    if inputs_read is not None:
        ev = inputs_read.cuda_event
    check(L.kfac_invert_ex(arr, len(jobs), ws.data_ptr(), ws.numel(), info.data_ptr(), ev, stream),
          "kfac_invert_ex")
    return info


def invert_pipelined(jobs, device: torch.device, info_host: torch.Tensor, order: "RawEvent",
                     inputs_read, done: "RawEvent", main: int, side: int, side_stream=None) -> torch.Tensor:
    """kfac_invert_pipelined: `side` ordered after `main`, the grouped inversion on `side`
    (`inputs_read` recorded after the F-reading launch), the verdict copied into the
    pinned `info_host`, `done` recorded on `side`.  Returns the device verdict vector:
    a buffer pooled per (device, side stream, job count) that the next such call on
    that stream overwrites -- read `info_host` (after `done`), or clone it first."""
    L = lib()
    arr = as_array(InvertJob, jobs)
    need = L.kfac_invert_workspace_bytes(arr, len(jobs))
    ws = workspace.get(device, need, side, side_stream)
    key = (device.index, side, len(jobs))
    info = _info_bufs.get(key)
    if info is None:
        info = _info_bufs[key] = torch.empty(len(jobs), dtype=torch.int32, device=device)
    check(L.kfac_invert_pipelined(arr, len(jobs), ws.data_ptr(), ws.numel(), info.data_ptr(),
                                  info_host.data_ptr(), order.handle,
                                  inputs_read.handle if inputs_read is not None else None,
                                  done.handle, main, side), "kfac_invert_pipelined")
    return info


def tri_jobs(factors):
    """[TriJob] of square row-major factors laid out back to back in a packed
    lower-triangle buffer, and that buffer's length (elements)."""
    jobs, off = [], 0
    for F in factors:
        n = F.shape[0]
        if F.dim() != 2 or F.shape[1] != n or F.stride(1) != 1:
            raise NativeError(f"tri pack: factor must be square with unit column stride, got "
                              f"{tuple(F.shape)} / {F.stride()}")
        jobs.append(TriJob(F.data_ptr(), F.stride(0), n, 0, off))
        off += n * (n + 1) // 2
    return jobs, off


def tri_pack(jobs, packed: torch.Tensor) -> None:
    """kfac_tri_pack on torch's current stream of packed's device."""
    check(lib().kfac_tri_pack(as_array(TriJob, jobs), len(jobs), packed.data_ptr(),
                              stream_handle(packed.device)), "kfac_tri_pack")


def tri_unpack(jobs, packed: torch.Tensor, mode: int) -> None:
    """kfac_tri_unpack (TRI_SYMMETRIC mirrors, TRI_LOWER zeroes the upper triangle)."""
    check(lib().kfac_tri_unpack(as_array(TriJob, jobs), len(jobs), packed.data_ptr(), int(mode),
                                stream_handle(packed.device)), "kfac_tri_unpack")


def syev(jobs, device: torch.device) -> torch.Tensor:
    L = lib()
    arr = as_array(EigJob, jobs)
    need = L.kfac_eig_workspace_bytes(arr, len(jobs))
    ws = workspace.get(device, need)
    info = torch.zeros(len(jobs), dtype=torch.int32, device=device)
    check(L.kfac_syev(arr, len(jobs), ptr(ws), ws.numel(), ptr(info), stream_handle(device)),
          "kfac_syev")
    return info


def kron_quadform(jobs, nb: int, abs_sum: bool, out: torch.Tensor):
    L = lib()
    arr = as_array(QuadJob, jobs)
    need = L.kfac_quadform_workspace_bytes(arr, len(jobs), nb)
    ws = workspace.get(out.device, need)
    check(L.kfac_kron_quadform(arr, len(jobs), nb, int(abs_sum), ptr(out), ptr(ws), ws.numel(),
                               stream_handle(out.device)), "kfac_kron_quadform")


def sample(jobs, device: torch.device, accumulate: bool) -> None:
    """kfac_sample, <= 8 jobs per launch pair (KFAC.sample / sample_and_replace)."""
    L = lib()
    for i in range(0, len(jobs), 8):
        chunk = jobs[i:i + 8]
        arr = as_array(SampleJob, chunk)
        ws = workspace.get(device, L.kfac_sample_workspace_bytes(arr, len(chunk)))
        check(L.kfac_sample(arr, len(chunk), int(accumulate), ptr(ws), ws.numel(),
                            stream_handle(device)), "kfac_sample")


def efb_update(jobs, device: torch.device) -> None:
    """kfac_efb_update, <= 8 layers per launch pair (EFB.update)."""
    L = lib()
    for i in range(0, len(jobs), 8):
        chunk = jobs[i:i + 8]
        arr = as_array(EfbJob, chunk)
        ws = workspace.get(device, L.kfac_efb_workspace_bytes(arr, len(chunk)))
        check(L.kfac_efb_update(arr, len(chunk), ptr(ws), ws.numel(), stream_handle(device)),
              "kfac_efb_update")


def efb_job(VA: torch.Tensor, VG: torch.Tensor, grad: torch.Tensor, state: torch.Tensor,
            diag, accumulate: bool, scale: float) -> EfbJob:
    """One layer of EFB.update: state (+)= (VG^T grad VA)^2, diag (+)= grad^2 * scale."""
    nG, nA = grad.shape
    for t, what in ((VA, "V_A"), (VG, "V_G"), (grad, "grad"), (state, "state")):
        require_device(t, what)
        if t.dim() != 2 or t.stride(1) != 1:
            raise ValueError(f"{what}: expected a 2-D tensor with unit column stride")
    if tuple(VA.shape) != (nA, nA) or tuple(VG.shape) != (nG, nG) or tuple(state.shape) != (nG, nA):
        raise ValueError(f"EFB shapes: V_A {tuple(VA.shape)}, V_G {tuple(VG.shape)}, grad "
                         f"{tuple(grad.shape)}, state {tuple(state.shape)}")
    j = EfbJob()
    j.VA, j.ldA, j.VG, j.ldG = VA.data_ptr(), VA.stride(0), VG.data_ptr(), VG.stride(0)
    j.grad, j.ld_grad = grad.data_ptr(), grad.stride(0)
    j.state, j.ld_state = state.data_ptr(), state.stride(0)
    if diag is not None:
        require_device(diag, "diag")
        if tuple(diag.shape) != (nG, nA) or diag.stride(1) != 1:
            raise ValueError(f"diag: expected ({nG}, {nA}) row-major, got {tuple(diag.shape)}")
        j.diag, j.ld_diag = diag.data_ptr(), diag.stride(0)
    j.nA, j.nG, j.accumulate, j.scale = nA, nG, int(accumulate), float(scale)
    return j


def kron_gram(UA: torch.Tensor, UG: torch.Tensor, c: torch.Tensor, sigma: torch.Tensor) -> torch.Tensor:
    """kfac_kron_gram: (la*lg)^2 = diag(sigma) V^T V diag(sigma), V = c * kron(UA, UG)
    (INF.pre_sampler, curvatures.py:548-580), never forming V."""
    for t, what in ((UA, "U_A"), (UG, "U_G"), (c, "correction"), (sigma, "sigma")):
        require_device(t, what)
    UA = UA if UA.stride(1) == 1 else UA.contiguous()
    UG = UG if UG.stride(1) == 1 else UG.contiguous()
    c, sigma = c.contiguous(), sigma.contiguous()
    nA, la = UA.shape
    nG, lg = UG.shape
    if c.numel() != nA * nG or sigma.numel() != la * lg:
        raise ValueError(f"kron_gram: c has {c.numel()} (want {nA * nG}), sigma {sigma.numel()} "
                         f"(want {la * lg}) elements")
    out = torch.empty(la * lg, la * lg, device=UA.device, dtype=torch.float32)
    j = GramJob()
    j.UA, j.ldA, j.UG, j.ldG = UA.data_ptr(), UA.stride(0), UG.data_ptr(), UG.stride(0)
    j.c, j.sigma, j.out, j.ldo = c.data_ptr(), sigma.data_ptr(), out.data_ptr(), out.stride(0)
    j.nA, j.nG, j.la, j.lg = nA, nG, la, lg
    L = lib()
    arr = as_array(GramJob, [j])
    ws = workspace.get(UA.device, L.kfac_gram_workspace_bytes(arr, 1))
    check(L.kfac_kron_gram(arr, 1, ptr(ws), ws.numel(), stream_handle(UA.device)), "kfac_kron_gram")
    return out


def sample_job(LA: torch.Tensor, LG: torch.Tensor, z: torch.Tensor, W: torch.Tensor, wcols: int,
               bias: torch.Tensor = None, dense: bool = False) -> SampleJob:
    """(LA z LG^T)^T into W (nG rows, columns < wcols) and, when wcols == nA - 1, its
    last column into bias."""
    for t in (LA, LG, z, W) + ((bias,) if bias is not None else ()):
        require_device(t, "sample operand")
        if t.stride(-1) != 1:
            raise NativeError("sample operands need a unit column stride")
    nA, nG = LA.shape[0], LG.shape[0]
    if tuple(z.shape) != (nA, nG) or not z.is_contiguous():
        raise NativeError(f"sample: z must be a contiguous ({nA}, {nG}) tensor")
    if W.dim() != 2 or W.shape[0] != nG or W.shape[1] < wcols:
        raise NativeError(f"sample: output must be ({nG}, >= {wcols})")
    return SampleJob(LA.data_ptr(), LA.stride(0), LG.data_ptr(), LG.stride(0), z.data_ptr(), nA, nG,
                     W.data_ptr(), W.stride(0), bias.data_ptr() if bias is not None else None,
                     wcols, int(dense))


# ---------------------------------------------------------------- job builders
def rowmajor_operand(x: torch.Tensor, has_ones: bool) -> Operand:
    """(rows, cols) row-major matrix, unit column stride (Linear a / g_rec)."""
    rows, cols = x.shape
    ld, unit = x.stride()
    assert unit == 1
    # positional constructor: one ctypes call instead of an attribute write per field
    return Operand(x.data_ptr(), ROWMAJOR, cols, rows, int(has_ones), 0, max(ld, cols))


def channel_operand(g: torch.Tensor) -> Operand:
    """Conv2d output gradient (B, C, Ho, Wo) contiguous: rows = B*Ho*Wo, cols = C."""
    assert g.dim() == 4 and g.is_contiguous()
    B, C, Ho, Wo = g.shape
    op = Operand()
    op.ptr, op.layout, op.cols = g.data_ptr(), CHANNEL, C
    op.L = Ho * Wo
    op.sB = C * Ho * Wo
    op.rows = B * Ho * Wo
    return op


def patch_operand(x: torch.Tensor, kernel, padding, stride, has_ones: bool) -> Operand:
    """Implicit F.unfold(x, kernel, padding=, stride=) of a contiguous (B,C,H,W) input."""
    assert x.dim() == 4 and x.is_contiguous()
    B, C, H, W = x.shape
    kh, kw = kernel
    ph, pw = padding
    sh, sw = stride
    Ho = (H + 2 * ph - kh) // sh + 1
    Wo = (W + 2 * pw - kw) // sw + 1
    if Ho <= 0 or Wo <= 0:
        raise RuntimeError(f"unfold: kernel {kernel} with padding {padding} larger than input {H}x{W}")
    op = Operand()
    op.ptr, op.layout = x.data_ptr(), PATCH
    op.C, op.H, op.W, op.kh, op.kw, op.sh, op.sw, op.ph, op.pw, op.Ho, op.Wo = \
        C, H, W, kh, kw, sh, sw, ph, pw, Ho, Wo
    op.L = Ho * Wo
    op.sB = C * H * W
    op.rows = B * Ho * Wo
    op.cols = C * kh * kw
    op.has_ones = int(has_ones)
    return op


def factor_job(op: Operand, F: torch.Tensor, alpha: float, beta: float) -> FactorJob:
    return FactorJob(op, alpha, beta, F.data_ptr(), F.stride(0))


def segment_table(ptrs):
    """HOST int64 array of batch base pointers for a multi-batch factor job
    (kfac_factor_job.seg_ptrs).  kfac_factor_update reads it during the call and
    passes the bases to the kernel as launch arguments: no device copy, no sync.
    The caller keeps the returned array alive until the call returns."""
    return (ctypes.c_int64 * len(ptrs))(*ptrs)


def table_ptr(table) -> int:
    return ctypes.addressof(table)


def invert_job(F: torch.Tensor, out: torch.Tensor, scale: float, shift: float,
               kind: int = OUT_INV_CHOL) -> InvertJob:
    # (one positional constructor call: field-by-field assignment costs ~4x the host time)
    return InvertJob(F.data_ptr(), F.stride(0), F.shape[0], kind, scale, shift, out.data_ptr(),
                     out.stride(0))


# ------------------------------------------------------------------ profiling
def profile_enable(on: bool = True):
    check(lib().kfac_profile_enable(int(on)), "kfac_profile_enable")


def profile_reset():
    check(lib().kfac_profile_reset(), "kfac_profile_reset")


def profile_read(kid: int):
    """(total milliseconds, launches) of the library's launches of kernel `kid`
    recorded since the last reset (HIP events on the launch stream)."""
    ms, n = ctypes.c_double(), ctypes.c_int64()
    check(lib().kfac_profile_read(kid, ctypes.byref(ms), ctypes.byref(n)), "kfac_profile_read")
    return ms.value, n.value


def profile_read_work(kid: int):
    """(total milliseconds, launches, algorithmic flops, algorithmic bytes) of slot `kid`
    since the last reset (kfac_profile_read_work: a factor slot's flops are sum K_rows *
    n (n + 1), its bytes every operand read once)."""
    ms, n = ctypes.c_double(), ctypes.c_int64()
    w, b = ctypes.c_double(), ctypes.c_double()
    check(lib().kfac_profile_read_work(kid, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(w), ctypes.byref(b)),
          "kfac_profile_read_work")
    return ms.value, n.value, w.value, b.value


# ------------------------------------------------------------------ knobs
def set_knob(name: str, value: int):
    """Change a per-call knob (KFAC_INV_GRAPH, KFAC_INV_LOOKAHEAD, KFAC_EIG_G, KFAC_EIG_RB)
    between calls; the library reads its environment once, at load."""
    check(lib().kfac_set_knob(name.encode(), int(value)), f"kfac_set_knob({name})")


def get_knob(name: str) -> int:
    v = ctypes.c_int()
    check(lib().kfac_get_knob(name.encode(), ctypes.byref(v)), f"kfac_get_knob({name})")
    return v.value
