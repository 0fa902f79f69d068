"""The C ABI library: builds in-tree, loads, exports every symbol the header
declares, and reports errors through yh_last_error. No GPU compute here."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "yolo_hip.h")


def header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(yh_\w+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = header_symbols()
    for s in ("yh_create", "yh_destroy", "yh_load_conv", "yh_forward", "yh_forward_u8", "yh_nms", "yh_last_error"):
        assert s in syms


def test_library_exports_every_header_symbol():
    from yolo_hip import _lib
    lib = _lib.lib()
    for s in header_symbols():
        assert hasattr(lib, s), f"{s} declared in include/yolo_hip.h but not exported"
    assert set(header_symbols()) == set(_lib._PROTOS), "ctypes prototypes out of sync with the header"


def test_abi_version_and_error_path():
    from yolo_hip import _lib
    lib = _lib.lib()
    assert lib.yh_abi_version() == _lib.ABI_VERSION
    h = ctypes.c_void_p()
    v = _lib.YhVariant()
    v.num_classes = 0  # invalid on purpose: rejected before any device call
    rc = lib.yh_create(ctypes.byref(v), 0, 0, ctypes.byref(h))
    assert rc != 0
    assert b"num_classes" in lib.yh_last_error()
    with pytest.raises(RuntimeError, match="num_classes"):
        _lib.check(rc)


def test_nms_workspace_bytes():
    from yolo_hip import _lib
    lib = _lib.lib()
    def al(v):
        return (v + 255) // 256 * 256
    # counts | histograms | per image: state (64 B), gathered first batch (4096 keys), decoded
    # first batch (3 x 4096 x 16 B), triangular IoU mask (64 x 64 x 65 / 2 words); no
    # per-candidate key list (the keys are made from the scores where needed, nms.hip)
    hist = al(2 * 4)
    state = al(hist + 2 * 2048 * 4)
    gk = al(state + 2 * 64)
    ents = al(gk + 2 * 4096 * 8)
    mask = al(ents + 2 * 3 * 4096 * 16)
    assert lib.yh_nms_workspace_bytes(2, 80, 8400) == mask + 2 * 64 * 64 * 65 // 2 * 8
    assert lib.yh_nms_workspace_bytes(0, 80, 8400) == 0


def test_nms_rejects_bad_arguments_without_touching_the_device():
    from yolo_hip import _lib
    lib = _lib.lib()
    rc = lib.yh_nms(0, None, 1, 80, 8400, 0.001, 0.65, 300, 30000, 7680.0, None, 0, None, None, None)
    assert rc != 0 and b"null" in lib.yh_last_error()
