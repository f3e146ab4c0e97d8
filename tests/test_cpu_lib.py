"""libupr.so loads on a GPU-less host and exports exactly the C ABI declared in
include/upr.h; host-side tables agree with the numpy oracle.  No device calls."""
import ctypes
import os
import re

import numpy as np

from conftest import REPO
from oracle import cv_u8
from upr import _lib as L
from upr import runtime


def header_functions(headers=("upr.h", "upr_train.h")):
    names = set()
    for h in headers:
        src = open(os.path.join(REPO, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(upr_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_library_builds_and_loads():
    assert os.path.exists(L.LIB_PATH), "run __graft_entry__.build() first"
    assert L.lib() is not None


def test_exports_every_header_symbol():
    names = header_functions()
    assert len(names) >= 60
    cdll = ctypes.CDLL(L.LIB_PATH)
    for n in names:
        assert hasattr(cdll, n), f"{n} declared in include/upr.h but not exported"
    # the ctypes binding covers exactly the header
    assert sorted(L.SIGNATURES) == names


def test_status_strings():
    assert L.status_string(0) == "ok"
    assert "shape" in L.status_string(L.UPR_ERR_SHAPE)
    assert "workspace" in L.status_string(L.UPR_ERR_WORKSPACE)


def test_lab_tables_match_oracle():
    a = cv_u8.lab_tables()
    b = runtime.lab_tables()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_null_args_rejected_without_device():
    lib = L.lib()
    assert lib.upr_model_workspace(None, 1, 64, 64) == 0
    assert lib.upr_model_forward(None, None, 1, 64, 64, None, None, None, None, 0, None) == L.UPR_ERR_ARG
    assert lib.upr_quantize_u8(None, None, 10, 0, None) == L.UPR_ERR_ARG
    assert lib.upr_clahe_u8(None, None, None, 1, 8, 8, 2.0, 8, 8, None) == L.UPR_ERR_ARG
    assert lib.upr_conv2d_nhwc(None, 1, 8, 8, 32, None, None, 32, 3, 3, 1, 1, 1, None, 0, None, 0, None) \
        == L.UPR_ERR_ARG
    out = ctypes.c_void_p()
    assert lib.upr_model_create(None, 0, 0, 0, 7, 0, ctypes.byref(out)) == L.UPR_ERR_ARG
    # flags: at most one of IENET_ONLY (1) / HEAD_ONLY (2), no unknown bits -- refused
    # before the (empty) state_dict is even looked at, so before any device call
    for bad in (3, 4, 8, 1 << 20, -1):
        assert lib.upr_model_create(None, 0, 0, 0, 0, bad, ctypes.byref(out)) == L.UPR_ERR_ARG, bad
        assert not out.value
    # training entries (include/upr_train.h) validate before touching the device
    assert lib.upr_t_conv_mfma(None, 1, 8, 8, 32, 32, 0, None, None, 32, 3, 3, 1, 1, 1, None, 0, 0, None, 32, 0, 0,
                               None) == L.UPR_ERR_ARG
    assert lib.upr_t_conv_wgrad(None, 1, 8, 8, 31, 31, 0, None, 8, 8, 32, 32, 0, 3, 3, 1, 1, 1, None,
                                None) == L.UPR_ERR_ARG
    assert lib.upr_t_adam(None, None, None, None, 10, None, 1.0, 1e-4, 0.9, 0.999, 1e-8, 0.0, 1, None,
                          None) == L.UPR_ERR_ARG
    assert lib.upr_t_loss_workspace(2, 64, 64) > 0
    assert lib.upr_t_loss_workspace(2, 8, 8) == 0
    assert lib.upr_t_pointwise(None, None, None, 4, 0, None, None, 0.0, 0, None) == L.UPR_ERR_ARG
