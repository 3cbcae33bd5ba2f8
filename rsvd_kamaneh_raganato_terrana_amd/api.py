"""Python host mirror of the reference's rSVD interface, running on the MI355X engine.

Reference signatures mirrored (AMSC22-23/rSVD_Kamaneh_Raganato_Terrana):

* ``rSVD(A, l, method=SVDMethod.Jacobi)`` -> ``(U, S, V)``
      void rSVD(Mat_m& A, Mat_m& U, Vec_v& S, Mat_m& V, int l, SVDMethod)  include/rSVD.hpp:14
* ``intermediate_step(A, Omega, l, q)`` -> ``Q``
      void intermediate_step(const Mat_m&, Mat_m& Q, const Mat_m& Omega, int l, int q)  :13
* ``generateOmega(n, l)`` -> ``Omega``                    Mat_m generateOmega(int, int)  :15
* ``SVDMethod`` (Jacobi, Power, ParallelJacobi)           include/SVD_class.hpp:28-32

numpy float64 inputs take the synchronous fp64 host path (the drop-in the reference's Eigen
callers see); torch CUDA tensors (float64 / float32 / bfloat16 / float8_e4m3fn) take the
asynchronous device path on the current torch stream, with A resident in HBM (bf16 / fp8 A return
fp32 U, S, V; fp8 A carries a per-tensor scale, A = a_scale * stored).  There is no CPU fallback: without the HIP
library or a GPU these functions raise.
"""
from __future__ import annotations

import ctypes
import enum
from typing import Optional

import numpy as np

from . import _capi
from ._capi import Desc, Info, Timing, check, lib


class SVDMethod(enum.IntEnum):
    Jacobi = 0
    Power = 1
    ParallelJacobi = 2


class QRMode(enum.IntEnum):
    Auto = 0      # CholeskyQR(2) + predicated CGS2 fallback
    GS2 = 1       # always CGS2 (robust, slow: one workgroup)
    CholQR2 = 2   # two CholeskyQR passes on every panel


def _dp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _torch():
    import torch  # plumbing only: device memory, streams, torch.distributed

    return torch


def colmajor(t):
    """A column-major (Fortran-order) view/copy of a 2-D torch tensor and its leading dim."""
    if t.dim() != 2:
        raise ValueError("expected a matrix")
    if t.stride(0) == 1 and t.stride(1) >= max(1, t.shape[0]):
        return t, t.stride(1)
    c = t.t().contiguous().t()
    return c, max(1, c.shape[0])


def empty_colmajor(rows: int, cols: int, dtype, device, pad: int = 0):
    """An uninitialised column-major rows x cols matrix; pad > 0 gives it the leading dimension
    rows + pad.  For a tall A whose row count is a large power of two, a pad of 64 elements keeps the
    columns of one k-step off a common HBM address pattern: C3's A^T Q 0.66 -> 0.54 ms per launch
    (profiles/r06_ldapad_ab.txt; no effect at C4 / C5).  Eigen callers pass lda = m."""
    torch = _torch()
    buf = torch.empty((cols, rows + max(0, pad)), dtype=dtype, device=device)
    return buf[:, :rows].t()


def make_allreduce_hook(get_buffer, group=None):
    """The C ABI's rsvd_allreduce_fn (include/rsvd_c.h) over torch.distributed.

    The engine only ever exchanges slices of its workspace (the Gram matrix of a CholeskyQR pass
    and the n x l panel Z = A^T Q); ``get_buffer()`` returns that workspace as a
    uint8 tensor and the hook sums the (pointer, count, dtype) slice in place across ranks.  It
    returns non-zero (never raises through C) for a slice outside the buffer or a failed
    collective.  With a CUDA workspace and the "nccl" backend this is an RCCL all-reduce over
    xGMI; with a CPU buffer and "gloo" it is the same code path the CPU tests exercise.
    """
    torch = _torch()
    import torch.distributed as dist

    def _hook(buf, count, dtype, stream, user):
        try:
            ws = get_buffer()
            if ws is None or buf is None:
                return 1
            base = ws.data_ptr()
            tdt = torch.float64 if dtype == _capi.F64 else torch.float32
            esz = 8 if dtype == _capi.F64 else 4
            off = buf - base
            if count < 0 or off < 0 or off % esz or off + count * esz > ws.numel():
                return 1
            view = ws[off: off + count * esz].view(tdt)
            dist.all_reduce(view, op=dist.ReduceOp.SUM, group=group)
            return 0
        except Exception:  # never unwind through C
            return 1

    return _capi.ALLREDUCE_FN(_hook)


def make_collective_hook(get_buffer, group=None):
    """The C ABI's rsvd_collective_fn (include/rsvd_c.h, ABI 5) over torch.distributed: the
    reduce-scatter of A^T Q and the all-gathers of the next skinny operand and of V that the
    n-side sharding needs.  Like the all-reduce hook it only ever touches
    slices of the handle's workspace and returns non-zero instead of raising through C.  RCCL
    ("nccl") and gloo on CPU buffers run reduce_scatter_tensor / all_gather_into_tensor, in place
    when the engine aliases recv = send + rank count (RS) or send = recv + rank count (AG) -- so the
    CPU gloo tests run the very branch RCCL runs.  gloo on CUDA buffers (two ranks sharing one GPU
    in the GPU tests) lacks those and gets the same result from one all_reduce (reduce-scatter: sum
    everything, keep this rank's chunk; all-gather: zero the other chunks, sum)."""
    torch = _torch()
    import torch.distributed as dist

    sizes = {_capi.F64: (torch.float64, 8), _capi.F32: (torch.float32, 4), _capi.BF16: (torch.bfloat16, 2)}
    # the tensor collectives (RCCL, and gloo on CPU tensors -- so the CPU tests run this same
    # branch, in-place aliasing included); gloo on CUDA tensors has only all_reduce
    legacy = {}

    def _hook(op, send, recv, count, dtype, stream, user):
        try:
            ws = get_buffer()
            if ws is None or send is None or recv is None or dtype not in sizes or count < 0:
                return 1
            tdt, esz = sizes[dtype]
            world = dist.get_world_size(group)
            rank = dist.get_rank(group)
            base = ws.data_ptr()

            def view(ptr, n):
                off = ptr - base
                if off < 0 or off % esz or off + n * esz > ws.numel():
                    raise ValueError("slice outside the workspace")
                return ws[off: off + n * esz].view(tdt)

            if "v" not in legacy:
                legacy["v"] = dist.get_backend(group) == "gloo" and ws.is_cuda
            if op == _capi.COLL_REDUCE_SCATTER:
                full, part = view(send, world * count), view(recv, count)
                if not legacy["v"]:
                    dist.reduce_scatter_tensor(part, full, op=dist.ReduceOp.SUM, group=group)
                else:
                    dist.all_reduce(full, op=dist.ReduceOp.SUM, group=group)
                    if recv != send + rank * count * esz:
                        part.copy_(full[rank * count:(rank + 1) * count])
                return 0
            if op == _capi.COLL_ALL_GATHER:
                full, part = view(recv, world * count), view(send, count)
                if not legacy["v"]:
                    dist.all_gather_into_tensor(full, part, group=group)
                else:
                    mine = full[rank * count:(rank + 1) * count]
                    if send != recv + rank * count * esz:
                        mine.copy_(part)
                    keep = mine.clone()
                    full.zero_()
                    mine.copy_(keep)
                    if tdt == torch.bfloat16:  # exact: every element is non-zero on one rank only
                        f = full.float()
                        dist.all_reduce(f, op=dist.ReduceOp.SUM, group=group)
                        full.copy_(f)
                    else:
                        dist.all_reduce(full, op=dist.ReduceOp.SUM, group=group)
                return 0
            return 1
        except Exception:  # never unwind through C
            return 1

    return _capi.COLLECTIVE_FN(_hook)


class Engine:
    """One GPU handle (HIP stream + workspace); mirrors what a C++ caller gets from librsvd_hip."""

    def __init__(self, device: int = 0):
        self.device = device
        h = ctypes.c_void_p()
        check(lib().rsvd_create(device, ctypes.byref(h)))
        self.h = h
        self._ws = None
        self._hook = None

    def close(self):
        if getattr(self, "h", None):
            lib().rsvd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- plumbing --------------------------------------------------------------------------
    def _bind_stream(self):
        torch = _torch()
        s = torch.cuda.current_stream(self.device)
        check(lib().rsvd_set_stream(self.h, ctypes.c_void_p(s.cuda_stream)), self.h)

    def reserve(self, desc: Desc):
        """Allocate the workspace from torch's allocator (outside any timed region)."""
        nbytes = ctypes.c_size_t(0)
        check(lib().rsvd_workspace_bytes(ctypes.byref(desc), ctypes.byref(nbytes)))
        return self._reserve_bytes(nbytes.value)

    def _reserve_bytes(self, nbytes: int):
        torch = _torch()
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = None
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{self.device}")
            check(lib().rsvd_set_workspace(self.h, ctypes.c_void_p(self._ws.data_ptr()), nbytes), self.h)
        return self._ws

    def set_comm(self, rank: int, world: int, group=None, shard_n: bool = True):
        """Row-sharded runs: bind the exchange hooks to torch.distributed over RCCL -- the
        all-reduce (m-side Grams; A^T Q when the n side is replicated) and, with shard_n, the
        reduce-scatter / all-gather hook that shards the n side across ranks as well.  At world 1
        the collective hook is still bound with shard_n, for runs with force_nshard=True (the
        sharded code path and its collectives on one GPU)."""
        self._hook = make_allreduce_hook(lambda: self._ws, group)
        check(lib().rsvd_set_comm(self.h, rank, world, self._hook, None), self.h)
        self._coll = make_collective_hook(lambda: self._ws, group) if shard_n else None
        check(lib().rsvd_set_collectives(self.h, self._coll if self._coll is not None else _capi.COLLECTIVE_FN(), None),
              self.h)

    def emulate_world(self, rank: int, world: int):
        """Diagnostics (bench.py --emulate-world): run rank `rank` of a `world`-rank row-sharded rSVD
        on this one handle -- the kernels a rank of the N-GPU job runs, at its shapes (its rows of A,
        its n shard, the fp64 Grams of sharded panels) -- with every collective a no-op.  The
        exchanged values are then not the other ranks' (the outputs are not the SVD of any matrix), so
        this only prices the per-rank kernels; the collectives are priced apart."""
        self._hook = _capi.ALLREDUCE_FN(lambda buf, count, dt, stream, user: 0)
        self._coll = _capi.COLLECTIVE_FN(lambda op, send, recv, count, dt, stream, user: 0)
        check(lib().rsvd_set_comm(self.h, rank, world, self._hook, None), self.h)
        check(lib().rsvd_set_collectives(self.h, self._coll, None), self.h)

    @staticmethod
    def comm_unique_id() -> bytes:
        """rsvd_comm_unique_id: the RCCL id one rank draws and every rank passes to comm_init."""
        buf = ctypes.create_string_buffer(_capi.COMM_ID_BYTES)
        check(lib().rsvd_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, uid: bytes, rank: int, world: int, shard_n: bool = True):
        """rsvd_comm_init: the library-owned RCCL communicator (no Python hooks on the data path;
        what a C / C++ caller uses, include/rsvd_c.h ABI 6)."""
        if len(uid) != _capi.COMM_ID_BYTES:
            raise ValueError("bad RCCL unique id")
        buf = ctypes.create_string_buffer(uid, _capi.COMM_ID_BYTES)
        # the handle may still hold set_comm's trampolines if the call fails (librccl missing):
        # drop the Python references only once the library owns the collectives
        check(lib().rsvd_comm_init(self.h, buf, rank, world, int(shard_n)), self.h)
        self._hook = self._coll = None

    def comm_destroy(self):
        check(lib().rsvd_comm_destroy(self.h), self.h)

    def set_timing(self, enable: bool = True):
        """hipEvent timing of every projection GEMM launch (benchmarking only)."""
        check(lib().rsvd_set_timing(self.h, int(enable)), self.h)

    def timing(self) -> dict:
        t = Timing()
        check(lib().rsvd_get_timing(self.h, ctypes.byref(t)), self.h)
        return {k: getattr(t, k) for k, _ in Timing._fields_}

    def sync(self):
        """rsvd_sync: wait for the queued runs and raise what they could not report at enqueue time
        (a timed-out in-kernel hand-off, an unrepairable rank deficiency, non-finite S)."""
        check(lib().rsvd_sync(self.h), self.h)

    def info(self) -> dict:
        inf = Info()
        check(lib().rsvd_get_info(self.h, ctypes.byref(inf)), self.h)
        return {k: getattr(inf, k) for k, _ in Info._fields_}

    # -- device path -----------------------------------------------------------------------
    @staticmethod
    def abi_dtype(t_dtype) -> int:
        torch = _torch()
        dt = {torch.float64: _capi.F64, torch.float32: _capi.F32, torch.bfloat16: _capi.BF16,
              torch.float8_e4m3fn: _capi.FP8_E4M3}.get(t_dtype)
        if dt is None:
            raise TypeError(f"unsupported dtype {t_dtype}")
        return dt

    @staticmethod
    def out_dtype(t_dtype):
        """Element type of U, S, V, Omega and Q for an A of this dtype (fp32 for bf16 / fp8)."""
        torch = _torch()
        return t_dtype if t_dtype in (torch.float64, torch.float32) else torch.float32

    def desc(self, A, l: int, q: int = 2, method: int = SVDMethod.Jacobi, seed: int = 0,
             qr_mode: int = QRMode.Auto, a_scale: float = 1.0, flags: int = 0) -> Desc:
        dt = self.abi_dtype(A.dtype)
        lda = A.stride(1) if A.stride(0) == 1 else None
        if lda is None:
            raise ValueError("A must be column-major (use colmajor())")
        return Desc(m=A.shape[0], n=A.shape[1], lda=max(lda, A.shape[0]), l=l, q=q, dtype=dt,
                    method=int(method), qr_mode=int(qr_mode), flags=int(flags), seed=seed, a_scale=a_scale)

    def rsvd(self, A, l: int, q: int = 2, method: int = SVDMethod.Jacobi, omega=None, seed: int = 0,
             qr_mode: int = QRMode.Auto, out=None, a_scale: float = 1.0, check_errors: bool = True,
             lowp_intermediates: bool = False, force_nshard: bool = False):
        """Device rSVD: A (m x n, CUDA, column-major f64/f32/bf16/e4m3) -> U (m x l), S (l), V (n x l).

        check_errors=True synchronises and raises on the run's device-side failures (rsvd_sync);
        False leaves the run queued (asynchronous) -- call sync() later to check.
        lowp_intermediates: RSVD_FLAG_LOWP_INTERMEDIATES (include/rsvd_c.h; bf16 / e4m3 A, q >= 2).
        force_nshard: RSVD_FLAG_FORCE_NSHARD (tests: the n-side sharded path at world 1)."""
        torch = _torch()
        A, _ = colmajor(A)
        flags = (_capi.FLAG_LOWP_INTERMEDIATES if lowp_intermediates else 0) | (
            _capi.FLAG_FORCE_NSHARD if force_nshard else 0)
        d = self.desc(A, l, q, method, seed, qr_mode, a_scale, flags)
        self.reserve(d)
        self._bind_stream()
        m, n = A.shape
        dd = min(l, n)
        odt = self.out_dtype(A.dtype)
        if out is None:
            U = empty_colmajor(m, dd, odt, A.device)
            S = torch.empty(dd, dtype=odt, device=A.device)
            V = empty_colmajor(n, dd, odt, A.device)
        else:
            U, S, V = out
        om, ldo = (None, 0)
        if omega is not None:
            om, ldo = colmajor(omega.to(device=A.device, dtype=odt))
        check(lib().rsvd_run(self.h, ctypes.byref(d), ctypes.c_void_p(A.data_ptr()),
                             ctypes.c_void_p(om.data_ptr() if om is not None else 0), ldo,
                             ctypes.c_void_p(U.data_ptr()), U.stride(1),
                             ctypes.c_void_p(S.data_ptr()),
                             ctypes.c_void_p(V.data_ptr()), V.stride(1)), self.h)
        if check_errors:
            self.sync()
        return U, S, V

    def range_finder(self, A, omega, q: int = 2, qr_mode: int = QRMode.Auto):
        A, _ = colmajor(A)
        odt = self.out_dtype(A.dtype)
        om, ldo = colmajor(omega.to(device=A.device, dtype=odt))
        l = om.shape[1]
        d = self.desc(A, l, q, SVDMethod.Jacobi, 0, qr_mode)
        self.reserve(d)
        self._bind_stream()
        Q = empty_colmajor(A.shape[0], l, odt, A.device)
        check(lib().rsvd_range_finder(self.h, ctypes.byref(d), ctypes.c_void_p(A.data_ptr()),
                                      ctypes.c_void_p(om.data_ptr()), ldo, ctypes.c_void_p(Q.data_ptr()),
                                      Q.stride(1)), self.h)
        self.sync()
        return Q

    def generate_omega(self, n: int, l: int, seed: int = 0, dtype=None):
        """Omega on the device.  dtype bfloat16 / float8_e4m3fn: the Omega those A types draw
        (Philox values rounded to bf16 / e4m3), returned as float32."""
        torch = _torch()
        dtype = dtype or torch.float64
        lp = 16
        while lp < l:
            lp *= 2
        self._reserve_bytes(n * lp * 8)
        self._bind_stream()
        Om = empty_colmajor(n, l, self.out_dtype(dtype), f"cuda:{self.device}")
        check(lib().rsvd_generate_omega(self.h, n, l, seed, self.abi_dtype(dtype),
                                        ctypes.c_void_p(Om.data_ptr())), self.h)
        return Om

    # -- host fp64 path (the Eigen-callers' drop-in) ----------------------------------------
    def rsvd_host(self, A: np.ndarray, l: int, q: int = 2, method: int = SVDMethod.Jacobi,
                  omega: Optional[np.ndarray] = None, seed: int = 0):
        A = np.asfortranarray(A, dtype=np.float64)
        m, n = A.shape
        dd = min(l, n)
        U = np.zeros((m, dd), order="F")
        S = np.zeros(dd)
        V = np.zeros((n, dd), order="F")
        om = None if omega is None else np.asfortranarray(omega, dtype=np.float64)
        self.reserve(Desc(m=m, n=n, lda=m, l=l, q=q, dtype=_capi.F64, method=int(method)))
        self._bind_stream()
        check(lib().rsvd_run_host_f64(self.h, m, n, _dp(A), m, l, q, int(method),
                                      _dp(om) if om is not None else None, seed, _dp(U), _dp(S), _dp(V)),
              self.h)
        return U, S, V

    def range_finder_host(self, A: np.ndarray, omega: np.ndarray, q: int = 2) -> np.ndarray:
        A = np.asfortranarray(A, dtype=np.float64)
        om = np.asfortranarray(omega, dtype=np.float64)
        m, n = A.shape
        l = om.shape[1]
        Q = np.zeros((m, l), order="F")
        self.reserve(Desc(m=m, n=n, lda=m, l=l, q=q, dtype=_capi.F64))
        self._bind_stream()
        check(lib().rsvd_range_finder_host_f64(self.h, m, n, _dp(A), m, _dp(om), l, q, _dp(Q)), self.h)
        return Q

    def generate_omega_host(self, n: int, l: int, seed: int = 0) -> np.ndarray:
        om = np.zeros((n, l), order="F")
        self._reserve_bytes(n * ((l + 15) // 16 * 16) * 8)
        self._bind_stream()
        check(lib().rsvd_generate_omega_host_f64(self.h, n, l, seed, _dp(om)), self.h)
        return om

    # -- QR() and SVD<method> drop-ins (dense_api.cpp) ------------------------------------------
    def _reserve_dense(self, fn, m, n, dt, arg):
        nbytes = ctypes.c_size_t(0)
        check(fn(m, n, dt, int(arg), ctypes.byref(nbytes)))
        self._reserve_bytes(nbytes.value)
        self._bind_stream()

    def qr(self, A, full: bool = False):
        """Device QR of A (CUDA f64/f32): (Q, R), reduced (m x n, n x n) or full (m x m, m x n)."""
        A, lda = colmajor(A)
        dt = self.abi_dtype(A.dtype)
        m, n = A.shape
        kq = m if full else n
        self._reserve_dense(lib().rsvd_qr_workspace_bytes, m, n, dt, full)
        Q = empty_colmajor(m, kq, A.dtype, A.device)
        R = empty_colmajor(kq, n, A.dtype, A.device)
        check(lib().rsvd_qr(self.h, m, n, ctypes.c_void_p(A.data_ptr()), lda, dt, int(full),
                            ctypes.c_void_p(Q.data_ptr()), Q.stride(1), ctypes.c_void_p(R.data_ptr()),
                            max(1, R.stride(1))), self.h)
        self.sync()
        return Q, R

    def svd(self, A, method: int = SVDMethod.Jacobi, r: int = 0, seed: int = 0):
        """Device SVD<method> of A (CUDA): (U m x k, S k, V n x k), k = min(m, n) (Power: the
        triplets kept; V's columns are the right singular vectors)."""
        torch = _torch()
        A, lda = colmajor(A)
        dt = self.abi_dtype(A.dtype)
        m, n = A.shape
        k = min(m, n)
        self._reserve_dense(lib().rsvd_svd_workspace_bytes, m, n, dt, method)
        U = empty_colmajor(m, k, A.dtype, A.device)
        S = torch.empty(k, dtype=A.dtype, device=A.device)
        V = empty_colmajor(n, k, A.dtype, A.device)
        kept = ctypes.c_int32(0)
        check(lib().rsvd_svd(self.h, m, n, ctypes.c_void_p(A.data_ptr()), lda, dt, int(method), r, seed,
                             ctypes.c_void_p(U.data_ptr()), U.stride(1), ctypes.c_void_p(S.data_ptr()),
                             ctypes.c_void_p(V.data_ptr()), V.stride(1), ctypes.byref(kept)), self.h)
        self.sync()
        kk = kept.value
        return U[:, :kk], S[:kk], V[:, :kk]

    def qr_host(self, A: np.ndarray, full: bool = False):
        A = np.asfortranarray(A, dtype=np.float64)
        m, n = A.shape
        kq = m if full else n
        Q = np.zeros((m, kq), order="F")
        R = np.zeros((kq, n), order="F")
        self._reserve_dense(lib().rsvd_qr_workspace_bytes, m, n, _capi.F64, full)
        check(lib().rsvd_qr_host_f64(self.h, m, n, _dp(A), m, int(full), _dp(Q), _dp(R)), self.h)
        return Q, R

    def svd_host(self, A: np.ndarray, method: int = SVDMethod.Jacobi, r: int = 0, seed: int = 0):
        A = np.asfortranarray(A, dtype=np.float64)
        m, n = A.shape
        k = min(m, n)
        U = np.zeros((m, k), order="F")
        S = np.zeros(k)
        V = np.zeros((n, k), order="F")
        kept = ctypes.c_int32(0)
        self._reserve_dense(lib().rsvd_svd_workspace_bytes, m, n, _capi.F64, method)
        check(lib().rsvd_svd_host_f64(self.h, m, n, _dp(A), m, int(method), r, seed, _dp(U), _dp(S), _dp(V),
                                      ctypes.byref(kept)), self.h)
        kk = kept.value
        return U[:, :kk].copy(order="F"), S[:kk].copy(), V[:, :kk].copy(order="F")


_DEFAULT: Optional[Engine] = None


def default_engine() -> Engine:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = Engine(0)
    return _DEFAULT


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


# ---- reference-named free functions ------------------------------------------------------------
def rSVD(A, l: int, method: SVDMethod = SVDMethod.Jacobi, q: int = 2, omega=None, seed: int = 0):
    """rSVD (src/rSVD.cpp:72-133). Returns (U, S, V); q defaults to the reference's hard-coded 2.

    SVDMethod.Power returns the reference's layouts (src/rSVD.cpp:106-113): U m x l, S l and V the
    n x n V_ of SVD<Power> (v_i in row i, identity rows beyond), cut to the triplets kept on an
    early stop (SVD_class.hpp:198-208).  Engine.rsvd returns V as columns instead."""
    eng = default_engine()
    if _is_torch(A):
        U, S, V = eng.rsvd(A, l, q=q, method=method, omega=omega, seed=seed)
    else:
        U, S, V = eng.rsvd_host(A, l, q=q, method=method, omega=omega, seed=seed)
    if int(method) != SVDMethod.Power:
        return U, S, V
    kept = eng.info()["power_kept"]
    xp = _torch() if _is_torch(A) else np
    n = V.shape[0]
    Vf = xp.eye(n, dtype=V.dtype, **({"device": V.device} if _is_torch(A) else {}))
    Vf[:kept, :] = V[:, :kept].T
    if kept >= S.shape[0]:
        return U, S, Vf
    if kept == 0:
        z = xp.zeros
        return z((U.shape[0], 1), dtype=U.dtype), z(1, dtype=S.dtype), z((n, 1), dtype=V.dtype)
    return U[:, :kept], S[:kept], Vf[:, :kept]


def rSVD_image_compression(A, l: int, omega=None, seed: int = 0):
    """image_compression's 5-argument rSVD(A, U, S, V, l) (image_compression/src/rSVD.cpp:77-118): q = 1,
    its own power-method SVD of B (image_compression/src/SVD.cpp:30-55 -- B = A^T A recomputed after
    every deflation, no sigma < 1e-12 stop) and V = VT^T with the right singular vectors in columns.
    Returns (U m x d, S d, V n x d), d = min(l, n)."""
    eng = default_engine()
    if _is_torch(A):
        return eng.rsvd(A, l, q=1, method=_capi.SVD_POWER_IC, omega=omega, seed=seed)
    return eng.rsvd_host(A, l, q=1, method=_capi.SVD_POWER_IC, omega=omega, seed=seed)


def intermediate_step(A, Omega, l: int, q: int):
    """intermediate_step (src/rSVD.cpp:57-70): the orthonormal range basis Q (m x l)."""
    eng = default_engine()
    if _is_torch(A):
        return eng.range_finder(A, Omega[:, :l], q=q)
    return eng.range_finder_host(A, np.asarray(Omega)[:, :l], q=q)


def generateOmega(n: int, l: int, seed: int = 0):
    """generateOmega (src/rSVD.cpp:12-55): n x l N(0,1), reproducible from `seed`."""
    return default_engine().generate_omega_host(n, l, seed)


def qr_decomposition_reduced(A):
    """qr_decomposition_reduced (src/QR.cpp:43-80): (Q m x n, R n x n); requires m >= n."""
    eng = default_engine()
    return eng.qr(A, full=False) if _is_torch(A) else eng.qr_host(A, full=False)


def qr_decomposition_full(A):
    """qr_decomposition_full (src/QR.cpp:22-41): (Q m x m, R m x n)."""
    eng = default_engine()
    return eng.qr(A, full=True) if _is_torch(A) else eng.qr_host(A, full=True)


class SVD:
    """template<SVDMethod method> class SVD (include/SVD_class.hpp:35-71) on the GPU engine.

    ``SVD(data, r=0, method=SVDMethod.Jacobi)``; ``compute()``; ``getU/getS/getV``; ``setData``.
    Output shapes follow the reference: Jacobi / ParallelJacobi U m x k, S k, V n x k
    (k = min(m, n), :107-108); Power U m x m and V n x n initialised to the identity with u_i in
    column i of U and v_i in ROW i of V (:82-83, :213-214), S of length min(m, n); when the
    power method stops early at sigma < 1e-12 after i triplets the three are cut to their first i
    columns as conservativeResize does (:198-208).  ``compute()`` prints nothing (the reference
    writes progress to stdout, :80-95).  ``seed`` replaces the power method's random_device start
    vectors (src/PM.cpp:15-16) with Philox(seed + i).
    """

    def __init__(self, data, r: int = 0, method: SVDMethod = SVDMethod.Jacobi, seed: int = 0):
        self._data = np.array(data, dtype=np.float64, order="F", copy=True)
        self._r = int(r)
        self._method = SVDMethod(method)
        self._seed = seed
        self._U = self._S = self._V = None

    def setData(self, data):
        self._data = np.array(data, dtype=np.float64, order="F", copy=True)

    def compute(self):
        m, n = self._data.shape
        eng = default_engine()
        if self._method != SVDMethod.Power:
            self._U, self._S, self._V = eng.svd_host(self._data, self._method)
            return
        dim = self._r if self._r else min(m, n)
        u, s, v = eng.svd_host(self._data, SVDMethod.Power, r=self._r, seed=self._seed)
        k = s.shape[0]
        if k == 0:
            self._U, self._S, self._V = np.zeros((m, 1)), np.zeros(1), np.zeros((n, 1))
            return
        U = np.eye(m, order="F")
        V = np.eye(n, order="F")
        S = np.zeros(min(m, n))
        U[:, :k] = u
        V[:k, :] = v.T
        S[:k] = s
        if k < dim:
            U, S, V = U[:, :k].copy(order="F"), S[:k].copy(), V[:, :k].copy(order="F")
        self._U, self._S, self._V = U, S, V

    def getU(self):
        return self._U

    def getS(self):
        return self._S

    def getV(self):
        return self._V
