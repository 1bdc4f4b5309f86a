"""Python mirror of the reference's SIFT interface over libsift_hip.so (C ABI).

Names follow /root/reference/sift_cuda/interface/Detector.hh:24-96 and
/root/reference/sift_cuda/types/CudaSiftConfig.hh:3-14 (including the
reference's field spellings), so host code and parity tests read like the
reference's own callers (/root/reference/tool/*.cc).

The compute path is the HIP library only: if libsift_hip.so is missing this
module raises ImportError-like errors on first use; there is no CPU fallback.

HIP runtime note: PyTorch wheels bundle their own libamdhip64.so.  A process that
uses both torch and this library must load torch's runtime BEFORE
libsift_hip.so, so that the library binds to the already-loaded runtime (one HIP
runtime per process; the other order leaves torch with "No HIP GPUs are
available").  `lib()` therefore imports torch first whenever torch is
installed, so the load order no longer depends on the caller's imports.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import sys
import warnings
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.normpath(os.path.join(_HERE, "..", "lib"))
# SIFT_HIP_LIB: alternative build of the same library (kernel A/B experiments).
LIB_PATH = os.environ.get("SIFT_HIP_LIB") or os.path.join(LIB_DIR, "libsift_hip.so")

SIFT_HIP_OK = 0
SIFT_HIP_F32, SIFT_HIP_U8 = 0, 1  # pixel formats (include/sift_hip.h)
SIFT_HIP_DESC_FAST, SIFT_HIP_DESC_EXACT = 0, 1  # descriptor modes (sift_hip_set_descriptor_mode)
_lib = None


class SiftHipError(RuntimeError):
    pass


class SiftCapacityWarning(RuntimeWarning):
    """A per-frame capacity (candidates, refined, oriented, results) overflowed; see overflow_flags()."""


class _Config(ctypes.Structure):
    _fields_ = [
        ("col_width", ctypes.c_int),
        ("row_width", ctypes.c_int),
        ("numFeatures", ctypes.c_int),
        ("numOctaveLayers", ctypes.c_int),
        ("contrastThreshould", ctypes.c_double),
        ("edgeThreshould", ctypes.c_double),
        ("sigma", ctypes.c_double),
        ("upscale", ctypes.c_int),
        ("numOctaves", ctypes.c_int),
        ("maxKeypoints", ctypes.c_int),
    ]


def lib() -> ctypes.CDLL:
    """Load libsift_hip.so (once).  Fails loudly when the build is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SiftHipError(f"{LIB_PATH} not found: build it with `make` (or __graft_entry__.build())")
    # torch's bundled HIP runtime first (module docstring), so one HIP runtime
    # serves both; importing torch does not touch the GPU.  Only when torch is
    # installed, and a broken torch install (OSError / RuntimeError from its
    # bundled libraries) must not stop callers that never use torch.
    if "torch" not in sys.modules and importlib.util.find_spec("torch") is not None:
        try:
            import torch  # noqa: F401
        except Exception as e:  # noqa: BLE001
            print(f"sift_amd: torch import failed ({e!r}); loading {LIB_PATH} on its own", file=sys.stderr)
    L = ctypes.CDLL(LIB_PATH)
    vp, ip, i, f, d, sz = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_float, ctypes.c_double, ctypes.c_size_t
    sigs = {
        "sift_hip_default_config": (None, [ctypes.POINTER(_Config), i, i]),
        "sift_hip_version": (ctypes.c_char_p, []),
        "sift_hip_last_error": (ctypes.c_char_p, []),
        "sift_hip_create": (i, [ctypes.POINTER(_Config), i, ctypes.POINTER(vp)]),
        "sift_hip_destroy": (i, [vp]),
        "sift_hip_warmup": (i, [vp]),
        "sift_hip_num_octaves": (i, [vp, ip]),
        "sift_hip_octave_dims": (i, [vp, i, ip, ip, ip]),
        "sift_hip_detect": (i, [vp, vp, sz]),
        "sift_hip_detect_device": (i, [vp, vp, sz, vp]),
        "sift_hip_detect_u8": (i, [vp, vp, sz]),
        "sift_hip_detect_device_fmt": (i, [vp, vp, sz, i, vp]),
        "sift_hip_submit": (i, [vp, vp, sz, i, ctypes.POINTER(ctypes.c_longlong)]),
        "sift_hip_wait": (i, [vp, ctypes.c_longlong]),
        "sift_hip_submit_device": (i, [vp, vp, sz, i, vp, ctypes.POINTER(ctypes.c_longlong)]),
        "sift_hip_set_lanes": (i, [vp, i]),
        "sift_hip_lanes": (i, [vp, ip, ip]),
        "sift_hip_set_micro_batch": (i, [vp, i]),
        "sift_hip_micro_batch": (i, [vp, ip]),
        "sift_hip_set_auto_micro_batch": (i, [vp, i]),
        "sift_hip_auto_micro_batch": (i, [vp, ip]),
        "sift_hip_sync": (i, [vp]),
        "sift_hip_set_batch": (i, [vp, i]),
        "sift_hip_batch_capacity": (i, [vp, ip]),
        "sift_hip_set_descriptor_mode": (i, [vp, i]),
        "sift_hip_descriptor_mode": (i, [vp, ip]),
        "sift_hip_capacities": (i, [vp, ip, ip, ip, ip]),
        "sift_hip_detect_batch_device": (i, [vp, vp, i, sz, sz, i, vp]),
        "sift_hip_batch_frames": (i, [vp, ip]),
        "sift_hip_batch_results_device": (i, [vp, i, ip, ip, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp)]),
        "sift_hip_batch_copy_to_host": (i, [vp, i, vp, vp, vp, i, ip]),
        "sift_hip_num_keypoints": (i, [vp, ip]),
        "sift_hip_overflow_flags": (i, [vp, ip]),
        "sift_hip_results_device": (i, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), ip, ip]),
        "sift_hip_copy_to_host": (i, [vp, vp, vp, vp, i]),
        "sift_hip_results_host": (i, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), ip]),
        "sift_hip_copy_descriptors_device": (i, [vp, vp, i, vp]),
        "sift_hip_results_sidecar": (i, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
        "sift_hip_descriptors_written": (i, [vp]),
        "sift_hip_match_codes_batched": (i, [vp, vp, vp, i, vp, vp, vp, vp, vp, vp, f, i, vp, vp, vp, vp]),
        "sift_hip_set_datagen": (i, [vp, ctypes.c_char_p]),
        "sift_hip_replay_stage": (i, [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]),
        "sift_hip_set_timing": (i, [vp, i]),
        "sift_hip_timing_count": (i, [vp, ip]),
        "sift_hip_timing_entry": (i, [vp, i, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(d), ip, ctypes.POINTER(d)]),
        "sift_hip_timing_reset": (i, [vp]),
        "sift_hip_debug_gaussian": (i, [vp, i, i, vp]),
        "sift_hip_debug_candidates": (i, [vp, vp, i, ip]),
        "sift_hip_matcher_create": (i, [i, i, i, i, ctypes.POINTER(vp)]),
        "sift_hip_matcher_destroy": (i, [vp]),
        "sift_hip_matcher_set_sidecars": (i, [vp, i]),
        "sift_hip_match_device": (i, [vp, vp, i, vp, i, f, i, vp, vp, vp, vp]),
        "sift_hip_match_batched": (i, [vp, i, vp, vp, vp, vp, f, i, vp, vp, vp, vp]),
        "sift_hip_match_host": (i, [vp, vp, i, vp, i, f, i, vp]),
        "sift_hip_match_plan": (i, [i, i, i, ip, ip]),
        "sift_synth_frame": (i, [ctypes.c_uint, i, i, vp]),
        "sift_hip_device_count": (i, [ip]),
        "sift_hip_set_device": (i, [i]),
        "sift_hip_memcpy_d2d": (i, [vp, vp, sz, vp]),
        "sift_hip_comm_create": (i, [i, ip, ctypes.POINTER(vp)]),
        "sift_hip_comm_destroy": (i, [vp]),
        "sift_hip_comm_size": (i, [vp, ip]),
        "sift_hip_comm_allgather": (i, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), sz, ctypes.POINTER(vp)]),
        "sift_hip_malloc": (i, [ctypes.POINTER(vp), sz]),
        "sift_hip_free": (i, [vp]),
        "sift_hip_memcpy_h2d": (i, [vp, vp, sz]),
        "sift_hip_memcpy_d2h": (i, [vp, vp, sz]),
        "sift_hip_device_sync": (i, []),
    }
    for name, (res, args) in sigs.items():
        if os.environ.get("SIFT_HIP_LIB") and not hasattr(L, name):
            continue  # an older A/B build (tools/ab_build.sh) may predate an entry point
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != SIFT_HIP_OK:
        msg = lib().sift_hip_last_error().decode(errors="replace")
        raise SiftHipError(f"{what} failed ({rc}): {msg}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def version() -> str:
    """'abi=<n> arch=gfx950 hip=<ver> build=default' or 'build=ab <A/B macros>'."""
    return lib().sift_hip_version().decode()


def is_default_build() -> bool:
    """False for a library built with kernel A/B or instrumentation macros
    (tools/ab_variant.sh): bench.py and smoke() refuse to report from one."""
    return "build=default" in version()


def device_count() -> int:
    n = ctypes.c_int(0)
    lib().sift_hip_device_count(ctypes.byref(n))
    return n.value


def synth_frame(index: int, width: int, height: int) -> np.ndarray:
    """Deterministic synthetic frame: float32 HxW, integers 0..255."""
    out = np.empty((height, width), np.float32)
    _check(lib().sift_synth_frame(index, width, height, _ptr(out)), "sift_synth_frame")
    return out


@dataclass
class CudaSiftConfig:
    """/root/reference/sift_cuda/types/CudaSiftConfig.hh:3-14 (+ numOctaves, maxKeypoints)."""

    col_width: int = 0
    row_width: int = 0
    numFeatures: int = 5000
    numOctaveLayers: int = 3
    contrastThreshould: float = 0.04
    edgeThreshould: float = 10.0
    sigma: float = 1.6
    upscale: bool = False
    numOctaves: int = 0
    maxKeypoints: int = 0

    def _abi(self) -> _Config:
        c = _Config()
        for name, _ in _Config._fields_:
            setattr(c, name, int(getattr(self, name)) if name == "upscale" else getattr(self, name))
        return c


class DeviceBuffer:
    """Non-owning device array view (stands in for thrust::device_vector).
    data() is for reading; a caller that writes into a detector's descriptor
    buffer takes mutable_data(), which drops the buffer's matcher sidecar
    (sift_hip_descriptors_written) so matches convert the written rows."""

    def __init__(self, ptr: int, size: int, descriptors: bool = False):
        self.ptr, self._size, self._desc = int(ptr or 0), int(size), descriptors

    def data(self) -> int:
        return self.ptr

    def mutable_data(self) -> int:
        if self._desc and self.ptr:
            _check(lib().sift_hip_descriptors_written(self.ptr), "descriptors_written")
        return self.ptr

    def size(self) -> int:
        return self._size


class Detector:
    """sift_cuda::Detector (Detector.hh:24-96) over the C ABI."""

    def __init__(self, config: CudaSiftConfig, device: int = -1, batch: int = 1, exact_descriptors: bool = False,
                 lanes: Optional[int] = None, micro_batch: int = 1, auto_micro_batch: Optional[int] = None):
        """batch > 1: frame-batch handle (sift_hip_set_batch): detectBatchDevice runs up to `batch`
        frames per launch; the single-frame methods keep working (frame 0's arena).
        exact_descriptors: OpenCV's sequential float histogram (SIFT_HIP_DESC_EXACT), descriptors
        bit-identical to the oracle; default the fixed-point histogram (+-1 on a byte).
        lanes: compute lanes for frames in flight (sift_hip_set_lanes, 1..4, library default 2):
        frames submitted before the previous one completes run concurrently on another lane.
        micro_batch > 1: frames of submitDevice queue until that many run as one launch group on a
        lane (sift_hip_set_micro_batch; a wait on a queued frame launches the partial group).
        auto_micro_batch: automatic launch groups of up to that many frames once every lane is busy
        (sift_hip_set_auto_micro_batch; library default 8, 0 = off)."""
        self.config = config
        self.batch = int(batch)
        self.exact_descriptors = bool(exact_descriptors)
        self._h = ctypes.c_void_p()
        _check(lib().sift_hip_create(ctypes.byref(config._abi()), device, ctypes.byref(self._h)), "sift_hip_create")
        if self.batch != 1:
            _check(lib().sift_hip_set_batch(self._h, self.batch), "set_batch")
        if lanes is not None:
            _check(lib().sift_hip_set_lanes(self._h, int(lanes)), "set_lanes")
        if micro_batch != 1:
            _check(lib().sift_hip_set_micro_batch(self._h, int(micro_batch)), "set_micro_batch")
        if auto_micro_batch is not None:
            _check(lib().sift_hip_set_auto_micro_batch(self._h, int(auto_micro_batch)), "set_auto_micro_batch")
        if self.exact_descriptors:
            _check(lib().sift_hip_set_descriptor_mode(self._h, SIFT_HIP_DESC_EXACT), "set_descriptor_mode")
        n = ctypes.c_int()
        lib().sift_hip_num_octaves(self._h, ctypes.byref(n))
        self.nOctaves = n.value
        self.total_size = 0
        self.prev_size = 0
        self.final_kpts = np.zeros((0, 3), np.float32)
        self.final_features = np.zeros((0, 4), np.float32)
        self.descriptors = np.zeros((0, 128), np.float16)
        self.device_kpts = self.device_features = self.device_descriptor = self.prev_descriptor = DeviceBuffer(0, 0)
        self._ready = False
        self._rb = None     # _refresh's ctypes holders
        self._views = None  # the pointers the result views were built from

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and h.value and _lib is not None:
            _lib.sift_hip_destroy(h)
            self._h = None

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def gpuWarmUpAndAllocate(self) -> bool:
        if not self._ready:
            _check(lib().sift_hip_warmup(self._h), "gpuWarmUpAndAllocate")
            self._ready = True
            self._refresh()
        return True

    def octave_dims(self, o: int):
        w, h, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().sift_hip_octave_dims(self._h, o, ctypes.byref(w), ctypes.byref(h), ctypes.byref(p)), "octave_dims")
        return w.value, h.value, p.value

    def _refresh(self) -> None:
        # Called after every frame: the ctypes holders are made once per
        # detector and the result views are rebuilt only when a pointer changed
        # (each ctypes call and object here is ~1 us of a ~0.23 ms frame).
        if self._rb is None:
            vals = [ctypes.c_void_p() for _ in range(4)] + [ctypes.c_int() for _ in range(4)]
            self._rb = (vals, [ctypes.byref(v) for v in vals])
        (k3, f4, d, pd, pc, cap, n, flags), refs = self._rb
        L = lib()
        _check(L.sift_hip_results_device(self._h, refs[0], refs[1], refs[2], refs[3], refs[4], refs[5]), "results")
        key = (k3.value, f4.value, d.value, pd.value, cap.value)
        if key != self._views:
            self._views = key
            self.device_kpts = DeviceBuffer(k3.value, cap.value)
            self.device_features = DeviceBuffer(f4.value, cap.value)
            self.device_descriptor = DeviceBuffer(d.value, cap.value * 128, descriptors=True)
            self.prev_descriptor = DeviceBuffer(pd.value, cap.value * 128, descriptors=True)
        self.prev_size = pc.value
        L.sift_hip_num_keypoints(self._h, refs[6])
        self.total_size = n.value
        L.sift_hip_overflow_flags(self._h, refs[7])
        self._warn_overflow(flags.value)

    def _warn_overflow(self, flags: Optional[int] = None) -> None:
        """A stage that hit its capacity clamps and sets a bit (keypoints the reference would keep are
        dropped): warned once per detector and flag (SiftCapacityWarning)."""
        if flags is None:
            flags = self.overflow_flags()
        new = flags & ~getattr(self, "_overflow_warned", 0)
        if new:
            self._overflow_warned = getattr(self, "_overflow_warned", 0) | flags
            warnings.warn(f"capacity overflow (flags {flags:#x}: 1 candidates, 2 refined, 4 oriented, 8 results); "
                          f"keypoints were dropped -- raise CudaSiftConfig.maxKeypoints", SiftCapacityWarning, stacklevel=3)

    def _host_frame(self, image: np.ndarray):
        """(array, format): uint8 frames stay 8-bit (Image8U); anything else is float32 (Imagef)."""
        if image.dtype == np.uint8:
            img, fmt = np.ascontiguousarray(image), SIFT_HIP_U8
        else:
            img, fmt = np.ascontiguousarray(image, dtype=np.float32), SIFT_HIP_F32
        if img.shape != (self.config.row_width, self.config.col_width):
            raise SiftHipError(f"image shape {img.shape} != configured {(self.config.row_width, self.config.col_width)}")
        return img, fmt

    def detectAndCompute(self, image: np.ndarray) -> None:
        """Detector.cu:133-233.  `image`: (rows, cols) float32 0..255 (Imagef) or uint8 (Image8U)."""
        self.gpuWarmUpAndAllocate()
        img, fmt = self._host_frame(image)
        if fmt == SIFT_HIP_U8:
            _check(lib().sift_hip_detect_u8(self._h, _ptr(img), img.strides[0]), "detectAndCompute")
        else:
            _check(lib().sift_hip_detect(self._h, _ptr(img), img.strides[0]), "detectAndCompute")
        self._refresh()

    def submit(self, image: np.ndarray) -> int:
        """Pipelined input (sift_hip_submit): stage + upload + enqueue, no wait.  Returns the frame ticket."""
        self.gpuWarmUpAndAllocate()
        img, fmt = self._host_frame(image)
        t = ctypes.c_longlong()
        _check(lib().sift_hip_submit(self._h, _ptr(img), img.strides[0], fmt, ctypes.byref(t)), "submit")
        return t.value

    def submitDevice(self, dev_ptr: int, row_stride_bytes: int = 0, stream: Optional[int] = None, u8: bool = False) -> int:
        """Pipelined device input (sift_hip_submit_device): the frame at dev_ptr is enqueued on a free lane
        after `stream`; returns the ticket for wait().  The buffer must stay unchanged until wait(ticket)."""
        self.gpuWarmUpAndAllocate()
        t = ctypes.c_longlong()
        _check(lib().sift_hip_submit_device(self._h, dev_ptr, row_stride_bytes, SIFT_HIP_U8 if u8 else SIFT_HIP_F32,
                                            stream, ctypes.byref(t)), "submitDevice")
        return t.value

    def lanes(self) -> tuple:
        """(lane limit, lanes created so far)."""
        m, c = ctypes.c_int(), ctypes.c_int()
        _check(lib().sift_hip_lanes(self._h, ctypes.byref(m), ctypes.byref(c)), "lanes")
        return m.value, c.value

    def micro_batch(self) -> int:
        """Frames per submitDevice launch group (sift_hip_micro_batch)."""
        m = ctypes.c_int()
        _check(lib().sift_hip_micro_batch(self._h, ctypes.byref(m)), "micro_batch")
        return m.value

    def auto_micro_batch(self) -> int:
        """Largest automatic launch group (sift_hip_auto_micro_batch; 0: automatic groups off)."""
        m = ctypes.c_int()
        _check(lib().sift_hip_auto_micro_batch(self._h, ctypes.byref(m)), "auto_micro_batch")
        return m.value

    def wait(self, ticket: int) -> None:
        """Block until frame `ticket` is complete and expose its results (prev = frame ticket-1)."""
        _check(lib().sift_hip_wait(self._h, ticket), "wait")
        self._refresh()

    def detectAndComputeDevice(self, dev_ptr: int, row_stride_bytes: int, stream: Optional[int] = None, sync: bool = True,
                               u8: bool = False) -> None:
        self.gpuWarmUpAndAllocate()
        fmt = SIFT_HIP_U8 if u8 else SIFT_HIP_F32
        _check(lib().sift_hip_detect_device_fmt(self._h, dev_ptr, row_stride_bytes, fmt, stream), "detectAndComputeDevice")
        if sync:
            self.sync()

    def sync(self) -> None:
        _check(lib().sift_hip_sync(self._h), "sync")
        self._refresh()

    # --- frame batches ----------------------------------------------------------
    def detectBatchDevice(self, dev_ptr: int, n: int, row_stride_bytes: int = 0, frame_stride_bytes: int = 0,
                          stream: Optional[int] = None, sync: bool = True, u8: bool = False) -> None:
        """n (<= batch) device frames at dev_ptr + i * frame_stride_bytes, one launch per stage for all."""
        self.gpuWarmUpAndAllocate()
        fmt = SIFT_HIP_U8 if u8 else SIFT_HIP_F32
        _check(lib().sift_hip_detect_batch_device(self._h, dev_ptr, n, row_stride_bytes, frame_stride_bytes, fmt, stream),
               "detectBatchDevice")
        if sync:
            self.sync()

    def results_sidecar(self):
        """(codes, keys) device pointers of the current frame's matcher sidecar (sift_hip_results_sidecar):
        int8 codes v - 128 per descriptor row (128 B) and int32 key biases -(256 |c|^2 + (row & 255))."""
        c, k = ctypes.c_void_p(), ctypes.c_void_p()
        _check(lib().sift_hip_results_sidecar(self._h, ctypes.byref(c), ctypes.byref(k)), "results_sidecar")
        return c.value, k.value

    def batch_frames(self) -> int:
        n = ctypes.c_int()
        _check(lib().sift_hip_batch_frames(self._h, ctypes.byref(n)), "batch_frames")
        return n.value

    def batch_results(self, i: int):
        """(count, overflow flags, device kpts3 / feats4 / descriptor pointers) of frame i of the current batch."""
        c, o = ctypes.c_int(), ctypes.c_int()
        k3, f4, d = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        _check(lib().sift_hip_batch_results_device(self._h, i, ctypes.byref(c), ctypes.byref(o), ctypes.byref(k3),
                                                   ctypes.byref(f4), ctypes.byref(d)), "batch_results")
        return c.value, o.value, k3.value, f4.value, d.value

    def batch_copy_to_host(self, i: int, descriptor: bool = True):
        """Host copies (kpts3 (n,3), feats4 (n,4), descriptors (n,128) fp16 or None) of frame i of the current batch."""
        n = self.batch_results(i)[0]
        k3 = np.zeros((n, 3), np.float32)
        f4 = np.zeros((n, 4), np.float32)
        d = np.zeros((n, 128), np.uint16) if descriptor else None
        got = ctypes.c_int()
        _check(lib().sift_hip_batch_copy_to_host(self._h, i, _ptr(k3), _ptr(f4), _ptr(d) if d is not None else None, n,
                                                 ctypes.byref(got)), "batch_copy_to_host")
        return k3, f4, (d.view(np.float16) if d is not None else None)

    def copyToHost(self, descriptor: bool = True) -> None:
        """Detector.cu:606-634."""
        n = self.total_size
        k3 = np.empty((n, 3), np.float32)
        f4 = np.empty((n, 4), np.float32)
        d = np.empty((n, 128), np.uint16) if descriptor else None
        _check(lib().sift_hip_copy_to_host(self._h, _ptr(k3), _ptr(f4), _ptr(d) if d is not None else None, n), "copyToHost")
        self.final_kpts, self.final_features = k3, f4
        if d is not None:
            self.descriptors = d.view(np.float16)

    def results_host(self, descriptor: bool = True):
        """(kpts3 (n,3), feats4 (n,4), descriptors (n,128) fp16 or None) of the
        current frame as read-only views of the handle's pinned host results
        (sift_hip_results_host: no copy into Python memory).  They stay valid
        while the frame is the current or the previous one; copy what must
        outlive that."""
        k3, f4, d, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int()
        _check(lib().sift_hip_results_host(self._h, ctypes.byref(k3), ctypes.byref(f4),
                                           ctypes.byref(d) if descriptor else None, ctypes.byref(n)), "results_host")

        def view(ptr, ctype, cols, dtype):
            if n.value == 0:
                return np.zeros((0, cols), dtype)
            a = np.ctypeslib.as_array((ctype * (n.value * cols)).from_address(ptr)).reshape(n.value, cols)
            a.flags.writeable = False
            return a

        kp = view(k3.value, ctypes.c_float, 3, np.float32)
        ft = view(f4.value, ctypes.c_float, 4, np.float32)
        ds = view(d.value, ctypes.c_uint16, 128, np.uint16).view(np.float16) if descriptor else None
        return kp, ft, ds

    def capacities(self) -> dict:
        """Per-frame buffer capacities (sift_hip_capacities; host-only)."""
        v = [ctypes.c_int() for _ in range(4)]
        _check(lib().sift_hip_capacities(self._h, *[ctypes.byref(x) for x in v]), "capacities")
        return dict(zip(("candidates", "refined", "oriented", "results"), (x.value for x in v)))

    def overflow_flags(self) -> int:
        v = ctypes.c_int()
        lib().sift_hip_overflow_flags(self._h, ctypes.byref(v))
        return v.value

    # --- parity/debug helpers -------------------------------------------------
    def debug_gaussian(self, octave: int, layer: int) -> np.ndarray:
        w, h, _ = self.octave_dims(octave)
        out = np.empty((h, w), np.float32)
        _check(lib().sift_hip_debug_gaussian(self._h, octave, layer, _ptr(out)), "debug_gaussian")
        return out

    def debug_candidates(self, cap: int = 1 << 20) -> np.ndarray:
        q = np.zeros((cap, 4), np.int32)
        cnt = ctypes.c_int()
        _check(lib().sift_hip_debug_candidates(self._h, _ptr(q), cap, ctypes.byref(cnt)), "debug_candidates")
        return q[: min(cnt.value, cap)]

    def setDataGen(self, path: str) -> None:
        """Detector.hh:48-51: from now on every single-frame detect writes its stage
        dumps into `path` (sift_hip_set_datagen; "" switches them off)."""
        _check(lib().sift_hip_set_datagen(self._h, (path or "").encode()), "setDataGen")

    STAGES = ("pyramid", "extrema", "refine", "orientation", "order", "descriptor")

    def replayStage(self, dump_dir: str, stage: str, out_dir: str) -> None:
        """tool/perf.cu:43-100: run ONE pipeline stage on a setDataGen dump's
        recorded input (sift_hip_replay_stage); outputs go to out_dir in the
        dump's file formats.  The handle's current results are discarded."""
        self.gpuWarmUpAndAllocate()
        _check(lib().sift_hip_replay_stage(self._h, dump_dir.encode(), stage.encode(), out_dir.encode()),
               f"replayStage({stage})")
        self._refresh()

    # --- stage timing (roofline) ---------------------------------------------
    def set_timing(self, enable, blur_reps: int = 1) -> None:
        mode = (blur_reps if blur_reps > 1 else 1) if enable else 0
        _check(lib().sift_hip_set_timing(self._h, mode), "set_timing")

    def timing(self) -> dict:
        n = ctypes.c_int()
        lib().sift_hip_timing_count(self._h, ctypes.byref(n))
        out = {}
        for k in range(n.value):
            name, ms, nl, by = ctypes.c_char_p(), ctypes.c_double(), ctypes.c_int(), ctypes.c_double()
            _check(lib().sift_hip_timing_entry(self._h, k, ctypes.byref(name), ctypes.byref(ms), ctypes.byref(nl), ctypes.byref(by)), "timing")
            out[name.value.decode()] = {"ms": ms.value, "launches": nl.value, "bytes": by.value}
        return out

    def timing_reset(self) -> None:
        lib().sift_hip_timing_reset(self._h)


class Matcher:
    """Brute-force L2 matcher (replaces Match.cu:8-177) with preallocated scratch."""

    @staticmethod
    def plan(max_query: int, max_train: int, pairs: int = 1) -> tuple:
        """(train splits per query block, waves per workgroup) a call of this
        shape launches with (sift_hip_match_plan; host-only)."""
        S, nw = ctypes.c_int(), ctypes.c_int()
        _check(lib().sift_hip_match_plan(max_query, max_train, pairs, ctypes.byref(S), ctypes.byref(nw)), "match_plan")
        return S.value, nw.value

    def __init__(self, max_query: int, max_train: int, max_pairs: int = 1, device: int = -1):
        self._m = ctypes.c_void_p()
        self.max_query, self.max_train, self.max_pairs = max_query, max_train, max_pairs
        _check(lib().sift_hip_matcher_create(device, max_query, max_train, max_pairs, ctypes.byref(self._m)), "matcher_create")

    def __del__(self):
        m = getattr(self, "_m", None)
        if m and m.value and _lib is not None:
            _lib.sift_hip_matcher_destroy(m)
            self._m = None

    def set_sidecars(self, enable: bool) -> None:
        """Single pairs of detector-produced buffers match their sidecar codes (default on; sift_hip_matcher_set_sidecars)."""
        _check(lib().sift_hip_matcher_set_sidecars(self._m, int(bool(enable))), "matcher_set_sidecars")

    def match_device(self, q_ptr: int, nq: int, t_ptr: int, nt: int, ratio: float = 0.8, ratio_on_squared: bool = False,
                     idx2_ptr: int = 0, d2_ptr: int = 0, match_ptr: int = 0, stream: Optional[int] = None) -> None:
        _check(lib().sift_hip_match_device(self._m, q_ptr, nq, t_ptr, nt, ratio, int(ratio_on_squared),
                                           idx2_ptr or None, d2_ptr or None, match_ptr or None, stream), "match_device")

    def match_batched(self, q_ptrs: Sequence[int], nqs: Sequence[int], t_ptrs: Sequence[int], nts: Sequence[int],
                      ratio: float = 0.8, ratio_on_squared: bool = False, idx2_ptr: int = 0, d2_ptr: int = 0,
                      match_ptr: int = 0, stream: Optional[int] = None) -> None:
        P = len(q_ptrs)
        qa = (ctypes.c_void_p * P)(*q_ptrs)
        ta = (ctypes.c_void_p * P)(*t_ptrs)
        na = (ctypes.c_int * P)(*nqs)
        ma = (ctypes.c_int * P)(*nts)
        _check(lib().sift_hip_match_batched(self._m, P, qa, na, ta, ma, ratio, int(ratio_on_squared),
                                            idx2_ptr or None, d2_ptr or None, match_ptr or None, stream), "match_batched")

    def match_codes_batched(self, codes_ptr: int, keys_ptr: int, pairs: Sequence, ratio: float = 0.8,
                            ratio_on_squared: bool = False, idx2_ptr: int = 0, d2_ptr: int = 0, match_ptr: int = 0,
                            stream: Optional[int] = None) -> None:
        """Pairs (qrow0, qkey0, nq, trow0, tkey0, nt) of ready code sets -- int8 codes (128 B rows from code row
        qrow0 / trow0) and int32 key biases (from key index qkey0 / tkey0), e.g. every rank's sidecar all-gathered
        (multi.all_gather_codes / multi.code_pairs) -- in ONE launch, no conversion
        (sift_hip_match_codes_batched).  Outputs packed per pair as match_batched."""
        P = len(pairs)
        qr, qk, nq, tr, tk, nt = ((ctypes.c_int * P)(*[p[k] for p in pairs]) for k in range(6))
        _check(lib().sift_hip_match_codes_batched(self._m, codes_ptr, keys_ptr, P, qr, qk, nq, tr, tk, nt, ratio,
                                                  int(ratio_on_squared), idx2_ptr or None, d2_ptr or None,
                                                  match_ptr or None, stream), "match_codes_batched")

    def match_host(self, q_ptr: int, nq: int, t_ptr: int, nt: int, ratio: float = 0.8, ratio_on_squared: bool = True) -> np.ndarray:
        out = np.full(max(nq, 0), -1, np.int32)
        _check(lib().sift_hip_match_host(self._m, q_ptr, nq, t_ptr, nt, ratio, int(ratio_on_squared), _ptr(out)), "match_host")
        return out


_default_matcher: Optional[Matcher] = None


def matchBruteForce(des: DeviceBuffer, num_des: int, src: DeviceBuffer, num_src: int) -> np.ndarray:
    """Match.cuh:9-14: nearest src row per des row if d1^2 < 0.8 d2^2, else -1."""
    global _default_matcher
    if _default_matcher is None or num_des > _default_matcher.max_query or num_src > _default_matcher.max_train:
        mq = max(num_des, _default_matcher.max_query if _default_matcher else 0, 1)
        mt = max(num_src, _default_matcher.max_train if _default_matcher else 0, 1)
        _default_matcher = Matcher(mq, mt)
    if num_des <= 0:
        return np.zeros(0, np.int32)
    return _default_matcher.match_host(des.data(), num_des, src.data(), num_src, 0.8, True)


class DeviceArray:
    """Minimal owning device allocation for callers without torch (tests)."""

    def __init__(self, nbytes: int):
        self.ptr = ctypes.c_void_p()
        self.nbytes = nbytes
        _check(lib().sift_hip_malloc(ctypes.byref(self.ptr), max(nbytes, 1)), "malloc")

    @classmethod
    def from_numpy(cls, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        d = cls(a.nbytes)
        _check(lib().sift_hip_memcpy_h2d(d.ptr, _ptr(a), a.nbytes), "h2d")
        return d

    def to_numpy(self, dtype, shape) -> np.ndarray:
        out = np.empty(shape, dtype)
        _check(lib().sift_hip_memcpy_d2h(_ptr(out), self.ptr, out.nbytes), "d2h")
        return out

    @property
    def value(self) -> int:
        return self.ptr.value

    def __del__(self):
        if getattr(self, "ptr", None) is not None and self.ptr.value and _lib is not None:
            _lib.sift_hip_free(self.ptr)
            self.ptr = None
