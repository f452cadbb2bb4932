"""Corrected gap-affine WFA — a separately labelled
engine, NOT reference parity.

The reference's ``wfa_align`` (src/wfa.rs:23-42; ``sequencealigning_amd.wfa``
reproduces it exactly) defines no output for realistic inputs: Ocean::trim
panics at s = 20.  This module computes what a gap-affine
WFA is meant to compute with the reference's penalties (wfa.rs:14-21,
x = 4 mismatch, o = 2 gap open, e = 6 gap extend; a gap of length L costs
o + L*e): the minimum penalty of a global alignment, on the GPU
(wfa_affine_kernels.hip).  The checker is the Gotoh DP in
``oracle/refaffine.c``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .nw import pack_csr

DEFAULT_PENALTIES = (4, 2, 6)
OVER_MAX_SCORE = -1   # penalty above max_score
OVER_WIDTH = -2       # wavefront wider than the widest ring (2,048 diagonals)


def _pen(penalties):
    x, o, e = penalties if penalties is not None else DEFAULT_PENALTIES
    return _lib.WfaPenalties(int(x), int(o), int(e))


def wfa_affine_batch(queries, dbs, pairs=None, *, penalties=None, max_score: int = 0,
                     device: int = 0) -> np.ndarray:
    """Minimum gap-affine penalty per pair (int32; negative codes above).
    pairs: None (all-vs-all, db outer / query inner like main.rs:61-62) or
    (n, 2) (query index, db index)."""
    qs, qo = pack_csr(queries)
    ds, do = pack_csr(dbs)
    if pairs is None:
        n = (len(qo) - 1) * (len(do) - 1)
        pq = pd = None
    else:
        pairs = np.asarray(pairs, np.uint32).reshape(-1, 2)
        n = len(pairs)
        pq = np.ascontiguousarray(pairs[:, 0])
        pd = np.ascontiguousarray(pairs[:, 1])
    out = np.zeros(n, np.int32)
    if n == 0:
        return out
    vp = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None  # noqa: E731
    pen = _pen(penalties)
    _lib.check(_lib.lib().saln_wfa_affine_batch(
        _lib.context(device), vp(qs), vp(qo), len(qo) - 1, vp(ds), vp(do), len(do) - 1, vp(pq),
        vp(pd), n, C.byref(pen), int(max_score), vp(out)), "saln_wfa_affine_batch")
    return out


def wfa_affine(seq1: bytes, seq2: bytes, *, penalties=None, max_score: int = 0,
               device: int = 0) -> int:
    """Minimum gap-affine penalty of one pair (seq1 = query, seq2 = db)."""
    return int(wfa_affine_batch([seq1], [seq2], [(0, 0)], penalties=penalties,
                                max_score=max_score, device=device)[0])


class WfaAffinePlan:
    """Device-resident corrected-WFA batch: plan from host offsets and a pair
    list once, execute on device (torch) sequence buffers into a device int32
    score tensor."""

    def __init__(self, q_off, db_off, pairs=None, *, penalties=None, max_score: int = 0,
                 device: int = 0):
        L = _lib.lib()
        self._L = L
        qo = np.ascontiguousarray(q_off, np.uint64)
        do = np.ascontiguousarray(db_off, np.uint64)
        if pairs is None:
            n = (len(qo) - 1) * (len(do) - 1)
            pq = pd = None
        else:
            pairs = np.asarray(pairs, np.uint32).reshape(-1, 2)
            n = len(pairs)
            pq = np.ascontiguousarray(pairs[:, 0])
            pd = np.ascontiguousarray(pairs[:, 1])
        self.n_pairs = n
        vp = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None  # noqa: E731
        self._h = C.c_void_p()
        pen = _pen(penalties)
        _lib.check(L.saln_wfa_affine_plan_create(_lib.context(device), vp(qo), len(qo) - 1,
                                                 vp(do), len(do) - 1, vp(pq), vp(pd), n,
                                                 C.byref(pen), int(max_score), C.byref(self._h)),
                   "saln_wfa_affine_plan_create")

    def execute(self, d_q, d_db, d_scores, stream=None):
        """d_q / d_db: device uint8 tensors (CSR bytes), d_scores: device int32[n_pairs]."""
        assert d_scores.numel() >= self.n_pairs and d_scores.dtype.itemsize == 4
        if stream is None:  # torch's current stream, like NwPlan.execute
            stream = _lib.torch_stream(d_scores.device)
        _lib.check(self._L.saln_wfa_affine_execute(
            self._h, C.c_void_p(d_q.data_ptr()), C.c_void_p(d_db.data_ptr()),
            C.c_void_p(d_scores.data_ptr()), C.c_void_p(stream)), "saln_wfa_affine_execute")

    def close(self):
        if self._h:
            self._L.saln_wfa_affine_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
