"""ctypes binding of the C ABI in include/rsvd_c.h (librsvd_hip.so, gfx950).

The shared library is built in-tree (``build()``) so it travels with the repository; importing
the package never falls back to a CPU implementation: if the library is missing or the GPU
runtime is absent, the calls raise.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "librsvd_hip.so")
REPO = os.path.dirname(PKG_DIR)

RSVD_OK = 0
STATUS = {
    0: "ok",
    1: "invalid argument",
    2: "unsupported",
    3: "HIP error",
    4: "no HIP device",
    5: "numerical failure",
    6: "communication failure",
}

F64, F32, BF16, FP8_E4M3 = 0, 1, 2, 3
SVD_JACOBI, SVD_POWER, SVD_PARALLEL_JACOBI, SVD_POWER_IC = 0, 1, 2, 3
QR_AUTO, QR_GS2, QR_CHOLQR2 = 0, 1, 2
FLAG_LOWP_INTERMEDIATES = 1
FLAG_FORCE_NSHARD = 2  # test/diagnostic: the n-side sharded path (RCCL calls) at world 1
COMM_ID_BYTES = 128

# Every symbol include/rsvd_c.h declares (checked by tests/test_capi_exports.py).
EXPORTS = (
    "rsvd_status_string", "rsvd_abi_version", "rsvd_create", "rsvd_destroy", "rsvd_set_stream",
    "rsvd_last_error", "rsvd_sync", "rsvd_get_info", "rsvd_set_comm", "rsvd_set_collectives", "rsvd_row_partition",
    "rsvd_workspace_bytes", "rsvd_set_workspace", "rsvd_set_timing", "rsvd_get_timing", "rsvd_run", "rsvd_range_finder",
    "rsvd_generate_omega", "rsvd_run_host_f64", "rsvd_range_finder_host_f64",
    "rsvd_generate_omega_host_f64", "rsvd_qr", "rsvd_svd", "rsvd_qr_workspace_bytes",
    "rsvd_svd_workspace_bytes", "rsvd_qr_host_f64", "rsvd_svd_host_f64",
    "rsvd_comm_unique_id", "rsvd_comm_init", "rsvd_comm_destroy",
)


class Desc(ctypes.Structure):
    _fields_ = [
        ("m", ctypes.c_int64), ("n", ctypes.c_int64), ("lda", ctypes.c_int64),
        ("l", ctypes.c_int32), ("q", ctypes.c_int32), ("dtype", ctypes.c_int32),
        ("method", ctypes.c_int32), ("qr_mode", ctypes.c_int32), ("flags", ctypes.c_int32),
        ("seed", ctypes.c_uint64), ("a_scale", ctypes.c_double),
    ]


class Info(ctypes.Structure):
    _fields_ = [
        ("cholqr_fallbacks", ctypes.c_int32), ("jacobi_sweeps", ctypes.c_int32),
        ("splits_nn", ctypes.c_int32), ("splits_tn", ctypes.c_int32), ("power_kept", ctypes.c_int32),
        ("n_shard_rows", ctypes.c_int32),
    ]


class Timing(ctypes.Structure):
    _fields_ = [
        ("nn_launches", ctypes.c_int32), ("tn_launches", ctypes.c_int32),
        ("nn_ms", ctypes.c_double), ("tn_ms", ctypes.c_double),
        ("sketch_launches", ctypes.c_int32), ("reserved", ctypes.c_int32), ("sketch_ms", ctypes.c_double),
    ]


ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                ctypes.c_void_p, ctypes.c_void_p)
# rsvd_collective_fn(op, send, recv, count, dtype, stream, user) -- ABI 5
COLLECTIVE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p)
COLL_REDUCE_SCATTER, COLL_ALL_GATHER = 1, 2


def _sources():
    """The files librsvd_hip.so is built from, in the order the Makefile hashes them."""
    hip = "util.hip proj.hip qr.hip jacobi.hip wide_proj.hip wide_qr.hip wide_svd.hip wide_eig.hip dense.hip gemm.hip".split()
    cpp = "driver.cpp wide.cpp dense_api.cpp comm.cpp dense_big.cpp".split()
    hdr = "common.hpp kernels.hpp wide.hpp dense.hpp handle.hpp".split()
    return ([os.path.join(CSRC, f) for f in hip + cpp + hdr] + [os.path.join(REPO, "include", "rsvd_c.h")]
            + [os.path.join(CSRC, "Makefile")])


def source_hash() -> str:
    """sha256 of the library's sources (the Makefile writes the same digest next to the .so)."""
    import hashlib

    h = hashlib.sha256()
    for p in _sources():
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def built_hash():
    try:
        with open(LIB_PATH + ".sha256") as f:
            return f.read().split()[0]
    except (OSError, IndexError):
        return None


def build(jobs: int = 8, force: bool = True) -> str:
    """Compile librsvd_hip.so for gfx950 with hipcc (cross-compiles without a GPU).

    force=True (what __graft_entry__.build() uses) recompiles every object from scratch; otherwise
    the library is rebuilt unless its recorded source digest matches the current sources."""
    if not force and os.path.exists(LIB_PATH) and built_hash() == source_hash():
        return LIB_PATH
    if force:
        subprocess.run(["make", "-C", CSRC, "clean"], check=True, capture_output=True)
    subprocess.run(["make", "-C", CSRC, f"-j{jobs}"], check=True)
    if built_hash() != source_hash():
        raise RuntimeError("librsvd_hip.so was built but its source digest does not match the sources")
    return LIB_PATH


_LIB = None


def lib():
    """Load librsvd_hip.so (raises if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run rsvd_kamaneh_raganato_terrana_amd.build()")
    if built_hash() != source_hash():
        raise RuntimeError(f"{LIB_PATH} is stale (its recorded source digest differs from csrc/): rebuild it")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    dp = ctypes.POINTER(ctypes.c_double)
    L.rsvd_status_string.restype = ctypes.c_char_p
    L.rsvd_status_string.argtypes = [ctypes.c_int]
    L.rsvd_last_error.restype = ctypes.c_char_p
    L.rsvd_last_error.argtypes = [vp]
    L.rsvd_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.rsvd_destroy.argtypes = [vp]
    L.rsvd_set_stream.argtypes = [vp, vp]
    L.rsvd_sync.argtypes = [vp]
    L.rsvd_get_info.argtypes = [vp, ctypes.POINTER(Info)]
    L.rsvd_set_comm.argtypes = [vp, ctypes.c_int, ctypes.c_int, ALLREDUCE_FN, vp]
    L.rsvd_set_collectives.argtypes = [vp, COLLECTIVE_FN, vp]
    L.rsvd_row_partition.restype = i64
    L.rsvd_row_partition.argtypes = [i64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(i64)]
    L.rsvd_workspace_bytes.argtypes = [ctypes.POINTER(Desc), ctypes.POINTER(ctypes.c_size_t)]
    L.rsvd_set_workspace.argtypes = [vp, vp, ctypes.c_size_t]
    L.rsvd_set_timing.argtypes = [vp, ctypes.c_int]
    L.rsvd_get_timing.argtypes = [vp, ctypes.POINTER(Timing)]
    L.rsvd_run.argtypes = [vp, ctypes.POINTER(Desc), vp, vp, i64, vp, i64, vp, vp, i64]
    L.rsvd_range_finder.argtypes = [vp, ctypes.POINTER(Desc), vp, vp, i64, vp, i64]
    L.rsvd_generate_omega.argtypes = [vp, i64, i32, u64, i32, vp]
    L.rsvd_run_host_f64.argtypes = [vp, i64, i64, dp, i64, i32, i32, i32, dp, u64, dp, dp, dp]
    L.rsvd_range_finder_host_f64.argtypes = [vp, i64, i64, dp, i64, dp, i32, i32, dp]
    L.rsvd_generate_omega_host_f64.argtypes = [vp, i64, i32, u64, dp]
    ip = ctypes.POINTER(i32)
    L.rsvd_qr.argtypes = [vp, i64, i64, vp, i64, i32, i32, vp, i64, vp, i64]
    L.rsvd_svd.argtypes = [vp, i64, i64, vp, i64, i32, i32, i32, u64, vp, i64, vp, vp, i64, ip]
    szp = ctypes.POINTER(ctypes.c_size_t)
    L.rsvd_qr_workspace_bytes.argtypes = [i64, i64, i32, i32, szp]
    L.rsvd_svd_workspace_bytes.argtypes = [i64, i64, i32, i32, szp]
    L.rsvd_qr_host_f64.argtypes = [vp, i64, i64, dp, i64, i32, dp, dp]
    L.rsvd_svd_host_f64.argtypes = [vp, i64, i64, dp, i64, i32, i32, u64, dp, dp, dp, ip]
    L.rsvd_comm_unique_id.argtypes = [vp]
    L.rsvd_comm_init.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.rsvd_comm_destroy.argtypes = [vp]
    _LIB = L
    return L


class RSVDError(RuntimeError):
    def __init__(self, status: int, detail: str = ""):
        self.status = status
        super().__init__(f"{STATUS.get(status, status)}: {detail}")


def check(status: int, handle=None) -> None:
    if status != RSVD_OK:
        detail = ""
        if handle:
            detail = (lib().rsvd_last_error(handle) or b"").decode()
        if status == 2 and "Unsupported SVD method" in detail:
            raise ValueError("Unsupported SVD method")  # std::invalid_argument, src/rSVD.cpp:123
        raise RSVDError(status, detail)


def row_partition(rows: int, world: int, rank: int):
    """(local_rows, offset) per src/rSVD.cpp:20-23 -- host arithmetic, no GPU needed."""
    off = ctypes.c_int64(0)
    n = lib().rsvd_row_partition(rows, world, rank, ctypes.byref(off))
    if n < 0:
        raise ValueError("bad partition arguments")
    return int(n), int(off.value)
