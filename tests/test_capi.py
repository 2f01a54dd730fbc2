"""CPU: the C-ABI library loads and exports every symbol include/protoseg_hip.h declares;
the pure-host entry points (no GPU call) behave as documented."""
import ctypes
import os
import re

import pytest

from protoseg_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "protoseg_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(protoseg_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_symbols()
    assert len(names) >= 9
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(_lib.SIGNATURES), "ctypes signatures out of sync with the header"


def test_version_and_supported_shapes():
    lib = _lib.load()
    assert lib.protoseg_version() == 10000
    assert lib.protoseg_l2_supported(64, 190, 19) == 1
    assert lib.protoseg_l2_supported(64, 361, 19) == 1
    assert lib.protoseg_l2_supported(32, 38, 3) == 1
    assert lib.protoseg_l2_supported(128, 64, 32) == 1
    assert lib.protoseg_l2_supported(64, 570, 19) == 1    # 30 prototypes/class: bf16 prototype chunks
    assert lib.protoseg_l2_supported(128, 1000, 19) == 1  # f32 family over prototype chunks
    # the wide family (l2_wide.hip): any depth, any class count, P beyond the chunked bound
    assert lib.protoseg_l2_supported(48, 190, 19) == 1
    assert lib.protoseg_l2_supported(64, 190, 33) == 1
    assert lib.protoseg_l2_supported(64, 5000, 19) == 1
    assert lib.protoseg_l2_supported(256, 2000, 200) == 1  # construct_PPNet's default, model.py:394
    assert lib.protoseg_l2_supported(512, 2000, 200) == 1
    assert lib.protoseg_l2_supported(0, 190, 19) == 0
    assert lib.protoseg_l2_supported(8192, 190, 19) == 0
    assert lib.protoseg_l2_supported(64, 100000, 19) == 0
    for C in (48, 64, 128, 512):
        assert lib.protoseg_l2_max_protos(C, _lib.PREC_BF16X3) == 65536
    assert lib.protoseg_l2_max_protos(0, _lib.PREC_F32) == 0
    assert lib.protoseg_l2_max_protos(64, 9) == 0
    for C in (32, 64, 128):
        m = lib.protoseg_l2_max_protos(C, _lib.PREC_F32)
        assert lib.protoseg_l2_supported(C, m, 19) == 1
    # on-load sigmoid of the add-on pre-activation: bf16x3 at C = 64, any P <= 4096
    assert lib.protoseg_l2_x_sigmoid_supported(32, 64, 65, 65, 361, 19, _lib.PREC_BF16X3) == 1
    assert lib.protoseg_l2_x_sigmoid_supported(32, 64, 65, 65, 190, 19, _lib.PREC_BF16X6) == 0
    assert lib.protoseg_l2_x_sigmoid_supported(32, 64, 65, 65, 190, 19, _lib.PREC_F32) == 0
    assert lib.protoseg_l2_x_sigmoid_supported(2, 128, 9, 9, 38, 19, _lib.PREC_BF16X3) == 0
    assert lib.protoseg_l2_x_sigmoid_supported(4096, 64, 256, 256, 190, 19, _lib.PREC_BF16X3) == 0  # > 2^31 B
    # native feature-map dtypes: f32 / bf16 everywhere, fp16 in the wide family only
    for dt in (_lib.F32, _lib.BF16):
        assert lib.protoseg_l2_x_dtype_supported(64, 361, 19, dt) == 1
    assert lib.protoseg_l2_x_dtype_supported(1024, 570, 19, _lib.F16) == 1   # configs[4] depth
    assert lib.protoseg_l2_x_dtype_supported(512, 2000, 200, _lib.F16) == 1  # construct_PPNet default
    assert lib.protoseg_l2_x_dtype_supported(64, 190, 19, _lib.F16) == 0     # bf16 family: widened
    assert lib.protoseg_l2_x_dtype_supported(64, 190, 19, _lib.I64) == 0
    assert lib.protoseg_l2_x_dtype_supported(0, 190, 19, _lib.F32) == 0


def test_workspace_size_is_host_only_and_aligned():
    lib = _lib.load()
    n = lib.protoseg_l2_bwd_workspace_size(32, 64, 65, 65, 190, 19)
    assert n > 0 and n % 256 == 0
    assert lib.protoseg_l2_bwd_workspace_size(0, 64, 65, 65, 190, 19) == 0


def test_argument_validation_returns_status_without_gpu():
    lib = _lib.load()
    null = ctypes.c_void_p(None)
    st = lib.protoseg_l2_fwd(null, 0, 1, 64, 2, 2, null, 19, null, 19, 1e-4, 0, 0, null, null, null, null)
    assert st == _lib.ERR_INVALID
    assert b"non-null" in lib.protoseg_last_error()
    dummy = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    st = lib.protoseg_l2_fwd(dummy, 7, 1, 64, 2, 2, dummy, 19, dummy, 19, 1e-4, 0, 0, null, null, null, null)
    assert st == _lib.ERR_UNSUPPORTED
    st = lib.protoseg_l2_fwd(dummy, 0, 1, 8192, 2, 2, dummy, 19, dummy, 19, 1e-4, 0, 0, null, null, null, null)
    assert st == _lib.ERR_UNSUPPORTED
    st = lib.protoseg_l2_fwd(dummy, _lib.F16, 1, 64, 2, 2, dummy, 19, dummy, 19, 1e-4, 0, 0, null, null, null, null)
    assert st == _lib.ERR_UNSUPPORTED and b"f16" in lib.protoseg_last_error()  # fp16 x: wide family only
    st = lib.protoseg_l2_fwd(dummy, 0, 1, 64, 2, 2, dummy, 19, dummy, 19, 1e-4, 0, 9, null, null, null, null)
    assert st == _lib.ERR_UNSUPPORTED and b"precision" in lib.protoseg_last_error()
    st = lib.protoseg_l2_fwd(dummy, 0, 1, 64, 2, 2, dummy, 19, dummy, 19, 1e-4, _lib.X_SIGMOID, _lib.PREC_F32,
                             null, null, null, null)
    assert st == _lib.ERR_UNSUPPORTED and b"X_SIGMOID" in lib.protoseg_last_error()
    st = lib.protoseg_adam_step(0, null, null, null, null, null, null, 1e-3, 0.9, 0.999, 1e-8, 0.0, null)
    assert st == _lib.ERR_INVALID
    # the fused update + prep: the bf16x3 one-chunk shapes only, refused before any launch
    bf3 = _lib.PRECISIONS["bf16x3"]
    assert lib.protoseg_l2_adam_prep_supported(64, 361, 19, bf3) == 1
    assert lib.protoseg_l2_adam_prep_supported(64, 190, 19, bf3) == 1
    assert lib.protoseg_l2_adam_prep_supported(64, 570, 19, bf3) == 0  # prototype chunks
    assert lib.protoseg_l2_adam_prep_supported(128, 361, 19, bf3) == 0
    assert lib.protoseg_l2_adam_prep_supported(64, 361, 19, _lib.PREC_F32) == 0
    assert lib.protoseg_l2_adam_prep_supported(64, 361, 200, bf3) == 0
    args = [dummy] * 5 + [1e-3, 0.0] + [dummy] * 5 + [1e-3, 0.0, 0.9, 0.999, 1e-8, dummy, 1 << 20, null]
    st = lib.protoseg_l2_adam_prep(64, 570, 19, 1e-4, 0, bf3, *args)
    assert st == _lib.ERR_UNSUPPORTED and b"adam_prep" in lib.protoseg_last_error()
    st = lib.protoseg_l2_adam_prep(64, 361, 19, 1e-4, 0, bf3, *args[:-3], null, 0, null)
    assert st == _lib.ERR_INVALID and b"operands" in lib.protoseg_last_error()
    st = lib.protoseg_l2_fwd_ex(dummy, 0, 1, 64, 2, 2, dummy, 570, dummy, 19, 1e-4, _lib.OPERANDS_READY, bf3,
                                dummy, null, null, null, 0, null)
    assert st == _lib.ERR_INVALID and b"OPERANDS_READY" in lib.protoseg_last_error()
    st = lib.protoseg_patch_class_mask(null, 2, 1, 4, 4, 2, 2, null, 0, null, null)
    assert st == _lib.ERR_INVALID
    st = lib.protoseg_push_argmin(dummy, 1, 8192, 2, 2, dummy, 3, dummy, dummy, dummy, null, null)
    assert st == _lib.ERR_UNSUPPORTED
    st = lib.protoseg_push_argmin_words(dummy, 1, 64, 2, 2, dummy, 3, dummy, dummy, 0, dummy, null, null)
    assert st == _lib.ERR_INVALID
    with pytest.raises(_lib.ProtosegError, match="status 1"):
        _lib.call("protoseg_push_merge", null, null, 1, 0, null, 64, 4, 3, null, null, null, null, null, null)
