"""ctypes binding of ``libprotoseg_hip.so`` (C ABI: ``include/protoseg_hip.h``).

The library is the only compute path of this package: there is no CPU or eager-PyTorch
fallback. If the shared object is missing, every entry point raises ``ProtosegError``.

``torch`` is imported first on purpose: torch ships its own ``libamdhip64.so`` (SONAME
``libamdhip64.so.7``), and loading it before our library makes the dynamic linker bind our
HIP calls to that same runtime, so stream handles from ``torch.cuda`` are valid for us.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PACKAGE_ROOT = pathlib.Path(__file__).resolve().parent.parent
CSRC_DIR = PACKAGE_ROOT / "csrc"
LIB_PATH = pathlib.Path(os.environ.get("PROTOSEG_HIP_LIB", CSRC_DIR / "libprotoseg_hip.so"))

# status codes (enum protoseg_status)
OK, ERR_INVALID, ERR_UNSUPPORTED, ERR_HIP = 0, 1, 2, 3
# enum protoseg_dtype
F32, BF16, I64, I32, U8, F16 = 0, 1, 2, 3, 4, 5
# enum protoseg_act
ACT_LOG, ACT_LINEAR, ACT_IDENTITY = 0, 1, 2
X_SIGMOID = 0x100  # OR-ed into the layer's act_kind: sigmoid of the pre-activation on load
OPERANDS_READY = 0x200  # OR-ed into protoseg_l2_fwd_ex's act_kind: operands hold these parameters' images
# enum protoseg_precision
PREC_BF16X3, PREC_BF16X6, PREC_F32 = 0, 1, 2
PRECISIONS = {"bf16x3": PREC_BF16X3, "bf16x6": PREC_BF16X6, "f32": PREC_F32}

_vp, _i, _f, _sz, _i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_int64

# name -> (restype, argtypes); exactly the symbols declared in include/protoseg_hip.h
SIGNATURES = {
    "protoseg_version": (_i, []),
    "protoseg_last_error": (ctypes.c_char_p, []),
    "protoseg_timing_events": (_i, [ctypes.c_char_p, _vp, _vp]),
    "protoseg_timing_kernel": (ctypes.c_char_p, []),
    "protoseg_timing_events_n": (_i, [ctypes.c_char_p, _vp, _vp, _i]),
    "protoseg_timing_launches": (_i, []),
    "protoseg_l2_supported": (_i, [_i, _i, _i]),
    "protoseg_l2_x_dtype_supported": (_i, [_i, _i, _i, _i]),
    "protoseg_l2_bwd_reads_dist": (_i, [_i, _i, _i, _i]),
    "protoseg_l2_bwd_saved": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _i, _f, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _sz, _vp]),
    "protoseg_adam_step": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _f, _f, _f, _f, _f, _vp]),
    "protoseg_l2_adam_prep_supported": (_i, [_i, _i, _i, _i]),
    "protoseg_l2_adam_prep": (_i, [_i, _i, _i, _f, _i, _i, _vp, _vp, _vp, _vp, _vp, _f, _f, _vp, _vp, _vp, _vp, _vp, _f,
                                   _f, _f, _f, _f, _vp, _sz, _vp]),
    "protoseg_l2_max_protos": (_i, [_i, _i]),
    "protoseg_l2_x_sigmoid_supported": (_i, [_i, _i, _i, _i, _i, _i, _i]),
    "protoseg_l2_fwd": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _i, _f, _i, _i, _vp, _vp, _vp, _vp]),
    "protoseg_l2_bwd_workspace_size": (_sz, [_i, _i, _i, _i, _i, _i]),
    "protoseg_l2_bwd": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _i, _f, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp,
                             _sz, _vp]),
    "protoseg_l2_bwd_kld": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _i, _f, _i, _i, _vp, _vp, _vp, _vp, _i, _vp,
                                 _vp, _vp, _vp, _sz, _vp]),
    "protoseg_l2_bwd_kld_supported": (_i, [_i, _i, _i, _i, _i, _i, _i, _i, _i]),
    "protoseg_set_backward_kernel": (_i, [ctypes.c_char_p]),
    "protoseg_l2_train_operands_bytes": (_sz, [_i, _i, _i, _i]),
    "protoseg_l2_fwd_ex": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _i, _f, _i, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    "protoseg_l2_bwd_ex": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _i, _f, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp,
                                _sz, _vp, _sz, _vp]),
    "protoseg_l2_bwd_kld_ex": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _i, _f, _i, _i, _vp, _vp, _vp, _vp, _i,
                                    _vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp]),
    "protoseg_patch_class_mask": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp]),
    "protoseg_push_argmin": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "protoseg_push_distances": (_i, [_vp, _i, _i, _i, _vp, _i, _vp, _vp]),
    "protoseg_patch_class_mask_words": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp]),
    "protoseg_push_argmin_words": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp]),
    "protoseg_push_distances_words": (_i, [_vp, _i, _i, _i, _vp, _i, _i, _vp, _vp]),
    "protoseg_push_merge": (_i, [_vp, _vp, _i, _i64, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "protoseg_push_update": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _vp, _i, _i, _i, _vp, _i, _vp, _i64, _vp, _vp,
                                  _vp, _vp, _vp, _vp]),
    "protoseg_kld_workspace_size": (_sz, [_i, _i, _i, _i]),
    "protoseg_kld_forward": (_i, [_vp, _i, _i, _i, _vp, _i, _vp, _i, _i, _vp, _vp, _vp, _sz, _vp]),
    "protoseg_kld_backward": (_i, [_vp, _i, _i, _i, _vp, _i, _vp, _i, _i, _vp, _vp, _sz, _vp, _vp]),
    "protoseg_kld_coef_bytes": (_sz, [_i, _i]),
    "protoseg_kld_backward_ex": (_i, [_vp, _i, _i, _i, _vp, _i, _vp, _i, _i, _vp, _vp, _sz, _vp, _sz, _vp, _vp]),
    "protoseg_kld_backward_compact": (_i, [_vp, _i, _i, _i, _vp, _i, _vp, _i, _i, _vp, _vp, _sz, _vp, _vp, _vp,
                                           _vp]),
    "protoseg_kld_expand": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "protoseg_eval_counts": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _vp, _i, _vp, _vp, _vp]),
    "protoseg_resize_label": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp]),
    "protoseg_knn_image_min": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "protoseg_knn_patch_label": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _vp, _i, _vp, _vp, _vp, _vp]),
    "protoseg_knn_heap_push": (_i, [_vp, _vp, _vp, _i, _i64, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "protoseg_knn_finalize": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "protoseg_act_upsample": (_i, [_vp, _i, _i, _i, _i, _i, _i, _f, _f, _vp, _vp, _vp]),
    "protoseg_bound_boxes": (_i, [_vp, _i, _i, _i, _vp, _i, _i, _vp, _vp, _i, _vp, _vp, _f, _i, _vp, _vp, _vp]),
}


class ProtosegError(RuntimeError):
    """A libprotoseg_hip call failed, or the library / a ROCm device is unavailable."""


_lock = threading.Lock()
_handle: ctypes.CDLL | None = None


def load() -> ctypes.CDLL:
    """Loads the library once and declares every exported symbol."""
    global _handle
    if _handle is not None:
        return _handle
    with _lock:
        if _handle is None:
            if not LIB_PATH.exists():
                raise ProtosegError(
                    f"{LIB_PATH} is missing: build it with `make -C {CSRC_DIR}` or __graft_entry__.build(); "
                    "the prototype layer has no fallback path")
            handle = ctypes.CDLL(str(LIB_PATH))
            for name, (restype, argtypes) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = restype
                fn.argtypes = argtypes
            _handle = handle
    return _handle


def call(name: str, *args) -> None:
    """Calls an int-status entry point and raises ProtosegError on failure."""
    lib = load()
    status = getattr(lib, name)(*args)
    if status != OK:
        msg = lib.protoseg_last_error()
        raise ProtosegError(f"{name} failed with status {status}: {msg.decode() if msg else ''}")


def version() -> int:
    return load().protoseg_version()


def ptr(t: torch.Tensor | None) -> ctypes.c_void_p:
    """Device pointer of a tensor, or NULL for None / an empty placeholder."""
    if t is None or t.numel() == 0:
        return ctypes.c_void_p(None)
    return ctypes.c_void_p(t.data_ptr())


def stream_of(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(*tensors: torch.Tensor) -> torch.device:
    """All tensors on one ROCm device; the HIP path refuses CPU tensors loudly."""
    dev = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise ProtosegError("protoseg HIP kernels need ROCm device tensors; got a tensor on "
                                f"{t.device} (there is no CPU path)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ProtosegError(f"tensors on different devices: {dev} and {t.device}")
    return dev
