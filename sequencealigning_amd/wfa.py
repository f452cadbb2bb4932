"""WFA engine, Python face of the C ABI.

Mirrors ``pub fn wfa_align(seq1: &Record, seq2: &Record, mode: Mode)``
(src/wfa.rs:23-42) with the reference's exact semantics, run by libsaln's HIP
kernel: the score loop of WaveFrontTensor::new / extend / Ocean::trim, the
convergence test and the rec_tr traceback.  The reference's panics become
statuses (``REF_PANIC_TRIM``, ``REF_PANIC_SLICE``); a run that the
reference would never finish stops at ``max_steps`` (``NONCONVERGED``).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .nw import _bytes, pack_csr
from .records import AlignmentError, Mode

STATES = "MDI"  # enum State { M, D, I } (wfa.rs:44-50)


@dataclass
class WfaAlignment:
    score: int       # printed score wfs.len()
    status: int
    steps: int
    seq1: bytes      # Alignment rows in display order (reversed push order)
    seq2: bytes


def render(seq1, seq2, mode: Mode = Mode.Global, *, max_steps: int = 64, max_width: int = 64,
           device: int = 0) -> tuple[str, int]:
    """The reference's stdout for wfa_align(seq1, seq2, mode) (up to its
    panic point): (text, status)."""
    q, d = _bytes(seq1), _bytes(seq2)
    L = _lib.lib()
    ctx = _lib.context(device)
    qb = C.create_string_buffer(q, len(q)) if q else None
    db = C.create_string_buffer(d, len(d)) if d else None
    n = C.c_uint64()
    res = _lib.WfaResult()
    _lib.check(L.saln_wfa_render(ctx, qb, len(q), db, len(d), int(mode), max_steps, max_width,
                                 None, 0, C.byref(n), C.byref(res)), "saln_wfa_render")
    buf = C.create_string_buffer(n.value + 1)
    _lib.check(L.saln_wfa_render(ctx, qb, len(q), db, len(d), int(mode), max_steps, max_width,
                                 buf, n.value + 1, C.byref(n), C.byref(res)), "saln_wfa_render")
    return buf.raw[:n.value].decode("latin-1"), res.status


def render_batch(queries, dbs, pairs=None, mode: Mode = Mode.Global, *, max_steps: int = 64,
                 max_width: int = 64, device: int = 0) -> list[tuple[str, int]]:
    """The reference's stdout per pair of a batch (saln_wfa_render_batch: one
    GPU run, every pair computed once): [(text, status)] in pair order
    (pairs=None: all-vs-all, db outer / query inner, main.rs:61-62)."""
    qs, qo = pack_csr(queries)
    ds, do = pack_csr(dbs)
    if pairs is None:
        pq = pd = None
        n = len(queries) * len(dbs)
    else:
        pa = np.asarray(pairs, np.uint32).reshape(-1, 2)
        pq, pd = np.ascontiguousarray(pa[:, 0]), np.ascontiguousarray(pa[:, 1])
        n = len(pa)
    L = _lib.lib()
    h = C.c_void_p()
    ptr = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None  # noqa: E731
    _lib.check(L.saln_wfa_render_batch(_lib.context(device), ptr(qs), ptr(qo), len(queries),
                                       ptr(ds), ptr(do), len(dbs), ptr(pq), ptr(pd), n,
                                       int(mode), max_steps, max_width, C.byref(h)),
               "saln_wfa_render_batch")
    try:
        out = []
        for k in range(L.saln_wfa_text_count(h)):
            tp, tn, res = C.c_void_p(), C.c_uint64(), _lib.WfaResult()
            _lib.check(L.saln_wfa_text_get(h, k, C.byref(tp), C.byref(tn), C.byref(res)),
                       "saln_wfa_text_get")
            out.append((C.string_at(tp.value, tn.value).decode("latin-1") if tn.value else "",
                        res.status))
        return out
    finally:
        L.saln_wfa_text_free(h)


def wfa_align(seq1, seq2, mode: Mode = Mode.Global, *, max_steps: int = 64, max_width: int = 64,
              device: int = 0) -> WfaAlignment:
    """wfa.rs:23 — seq1 = query, seq2 = db."""
    res, rows = wfa_align_batch([seq1], [seq2], [(0, 0)], mode, max_steps=max_steps,
                                max_width=max_width, device=device, with_alignment=True)
    if int(res["status"][0]) == _lib.NOT_IMPLEMENTED:
        raise AlignmentError("not implemented")
    return WfaAlignment(int(res["score"][0]), int(res["status"][0]), int(res["steps"][0]),
                        rows[0][0], rows[0][1])


def wfa_align_batch(queries, dbs, pairs=None, mode: Mode = Mode.Global, *, max_steps: int = 64,
                    max_width: int = 64, device: int = 0, with_alignment: bool = False):
    """Batched wfa_align (pairs: None = all-vs-all db-outer/query-inner, or
    (query, db) index pairs).  Returns (results structured array, rows or None)."""
    qs, qo = pack_csr(queries)
    ds, do = pack_csr(dbs)
    if pairs is None:
        n_pairs = (len(qo) - 1) * (len(do) - 1)
        pq = pd = None
    else:
        pairs = np.asarray(pairs, np.uint32).reshape(-1, 2)
        n_pairs = len(pairs)
        pq = np.ascontiguousarray(pairs[:, 0])
        pd = np.ascontiguousarray(pairs[:, 1])
    res = np.zeros(n_pairs, dtype=_lib.WFA_RESULT_DTYPE)
    if n_pairs == 0:
        return res, ([] if with_alignment else None)
    cap = int(2 * (int(np.diff(qo).max(initial=0)) + int(np.diff(do).max(initial=0))) + 64)
    aln = np.zeros(2 * cap * n_pairs, np.uint8) if with_alignment else None
    aoff = (np.arange(n_pairs, dtype=np.uint64) * np.uint64(2 * cap)) if with_alignment else None
    vp = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None  # noqa: E731
    _lib.check(_lib.lib().saln_wfa_align_batch(
        _lib.context(device), vp(qs), vp(qo), len(qo) - 1, vp(ds), vp(do), len(do) - 1, vp(pq),
        vp(pd), n_pairs, int(mode), max_steps, max_width, vp(res), vp(aln), vp(aoff), cap),
        "saln_wfa_align_batch")
    rows = None
    if with_alignment:
        rows = []
        for k in range(n_pairs):
            base = 2 * cap * k
            n1, n2 = min(int(res["aln_len1"][k]), cap), min(int(res["aln_len2"][k]), cap)
            rows.append((aln[base:base + n1].tobytes()[::-1],
                         aln[base + cap:base + cap + n2].tobytes()[::-1]))
    return res, rows


class WfaPlan:
    """Device-resident WFA batch (include/saln.h saln_wfa_plan_*): plan once
    from host offsets and a pair list, execute on device sequences into a
    device results buffer (uint8[n_pairs * 32] or int32[n_pairs * 8]).  Used
    for the configs[2] (C3) measurement."""

    def __init__(self, q_off, db_off, pairs=None, mode: Mode = Mode.Global, *,
                 max_steps: int = 64, max_width: int = 64, device: int = 0):
        self._L = _lib.lib()
        self.device = device
        qo = np.ascontiguousarray(q_off, np.uint64)
        do = np.ascontiguousarray(db_off, np.uint64)
        n_q, n_db = len(qo) - 1, len(do) - 1
        if pairs is None:
            self.n_pairs = n_q * n_db
            pq = pd = None
        else:
            pairs = np.asarray(pairs, np.uint32).reshape(-1, 2)
            self.n_pairs = len(pairs)
            pq = np.ascontiguousarray(pairs[:, 0])
            pd = np.ascontiguousarray(pairs[:, 1])
        vp = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None  # noqa: E731
        self._h = C.c_void_p()
        _lib.check(self._L.saln_wfa_plan_create(_lib.context(device), vp(qo), n_q, vp(do), n_db,
                                                vp(pq), vp(pd), self.n_pairs, int(mode),
                                                max_steps, max_width, C.byref(self._h)),
                   "saln_wfa_plan_create")

    def execute(self, q_seq, db_seq, results, stream=None) -> None:
        ptr = lambda t: t if isinstance(t, int) else t.data_ptr()  # noqa: E731
        if stream is None:
            stream = _lib.torch_stream(self.device)
        _lib.check(self._L.saln_wfa_execute(self._h, ptr(q_seq), ptr(db_seq), ptr(results),
                                            stream), "saln_wfa_execute")

    def close(self) -> None:
        if self._h:
            self._L.saln_wfa_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
