"""CPU: the C-ABI library (librsvd_hip.so) builds for gfx950, loads, and exports exactly what
include/rsvd_c.h declares; host-only entry points behave like the reference's arithmetic; the
product path fails loudly (no CPU fallback) where no GPU is present."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO

import rsvd_kamaneh_raganato_terrana_amd as R
from rsvd_kamaneh_raganato_terrana_amd import _capi

HEADER = os.path.join(REPO, "include", "rsvd_c.h")


@pytest.fixture(scope="module")
def lib():
    R.build(force=False)
    return _capi.lib()


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = set(re.findall(r"\b(rsvd_[a-z0-9_]+)\s*\(", src))
    names.discard("rsvd_allreduce_fn")  # callback typedef, not an export
    return names


def test_header_declares_the_binding_list():
    assert _declared() == set(_capi.EXPORTS)


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], check=True, capture_output=True,
                         text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = _declared() - exported
    assert not missing, missing
    for name in _declared():
        assert hasattr(lib, name)


def test_library_is_gfx950_code_object(lib):
    blob = open(_capi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"sm_" not in blob.split(b"amdgcn")[0][-64:]  # no foreign offload targets


def test_status_strings_and_version(lib):
    for k in range(7):
        assert lib.rsvd_status_string(k)
    assert lib.rsvd_abi_version() >= 1


@pytest.mark.parametrize("rows,world", [(100, 1), (100, 3), (7, 4), (4096 * 8, 8), (5, 8)])
def test_row_partition_matches_reference_split(lib, rows, world):
    """src/rSVD.cpp:20-23: rows/P each, the remainder to the first ranks, contiguous offsets."""
    off_expected = 0
    for r in range(world):
        n, off = R.row_partition(rows, world, r)
        per, rem = divmod(rows, world)
        assert n == (per + 1 if r < rem else per)
        assert off == r * per + min(r, rem) == off_expected
        off_expected += n
    assert off_expected == rows
    with pytest.raises(ValueError):
        R.row_partition(rows, world, world)


def _desc(**kw):
    d = dict(m=4096, n=4096, lda=4096, l=64, q=2, dtype=_capi.F32, method=0, qr_mode=0, flags=0, seed=0)
    d.update(kw)
    return _capi.Desc(**d)


def test_workspace_bytes_and_argument_checks(lib):
    import ctypes

    nb = ctypes.c_size_t(0)
    assert lib.rsvd_workspace_bytes(ctypes.byref(_desc()), ctypes.byref(nb)) == 0
    # A is never copied: the workspace holds l-wide panels and slabs only (<< m n)
    assert 0 < nb.value < 4096 * 4096 * 4
    nb64 = ctypes.c_size_t(0)
    assert lib.rsvd_workspace_bytes(ctypes.byref(_desc(dtype=_capi.F64)), ctypes.byref(nb64)) == 0
    assert nb64.value > nb.value
    # 1 = RSVD_ERR_INVALID_ARG, 2 = RSVD_ERR_UNSUPPORTED
    for bad, code in ((dict(l=0), 1), (dict(q=-1), 1), (dict(lda=100), 1), (dict(l=4097), 2), (dict(n=10, l=16), 2),
                      (dict(dtype=7), 2), (dict(method=7), 2), (dict(flags=4), 1)):
        assert lib.rsvd_workspace_bytes(ctypes.byref(_desc(**bad)), ctypes.byref(nb)) == code, bad
    # m < l is a valid row SHARD (the reference partitions the global m, src/rSVD.cpp:20-23): the size
    # query accepts it; rsvd_run refuses it on a one-rank handle (tests/test_gpu_big_l.py)
    assert lib.rsvd_workspace_bytes(ctypes.byref(_desc(m=10, lda=10, l=16)), ctypes.byref(nb)) == 0
    assert lib.rsvd_workspace_bytes(ctypes.byref(_desc(flags=_capi.FLAG_LOWP_INTERMEDIATES)), ctypes.byref(nb)) == 0
    # the wide engine (l > 64, bf16 / e4m3 A): l-wide panels, bf16 hi/lo copies, slabs -- O((m + n) l)
    for dt, l in ((_capi.F32, 128), (_capi.BF16, 256), (_capi.FP8_E4M3, 512), (_capi.F64, 100)):
        assert lib.rsvd_workspace_bytes(ctypes.byref(_desc(dtype=dt, l=l)), ctypes.byref(nb)) == 0, (dt, l)
        assert 0 < nb.value < 80 * 4096 * 512 * 8, (dt, l, nb.value)


def test_status_mapping():
    with pytest.raises(R.RSVDError):
        _capi.check(1, None)
    _capi.check(0, None)


def test_no_cpu_fallback_without_gpu(lib):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import ctypes

    h = ctypes.c_void_p()
    assert lib.rsvd_create(0, ctypes.byref(h)) == 4  # RSVD_ERR_NO_DEVICE
    with pytest.raises(R.RSVDError):
        R.rSVD(np.eye(8), 4)


def test_empty_colmajor_padded_pitch():
    """empty_colmajor(pad=) (INTEGRATION.md "Layout"): a column-major view whose leading dimension is
    rows + pad -- what Engine.desc() passes as lda (max(stride(1), rows))."""
    import torch

    import rsvd_kamaneh_raganato_terrana_amd as R

    for pad in (0, 64):
        A = R.empty_colmajor(7, 3, torch.float32, "cpu", pad=pad)
        assert A.shape == (7, 3) and A.stride() == (1, 7 + pad)
        B = torch.arange(21, dtype=torch.float32).reshape(7, 3)
        A.copy_(B)
        assert torch.equal(A, B)
        C, ld = R.colmajor(A)
        assert C.data_ptr() == A.data_ptr() and ld == 7 + pad  # no copy: the padded view is accepted as is
