"""ORACLE — test infrastructure only.

ctypes front-end for the C restatement in ``oracle/refcpu.c`` (reference:
``src/needleman_wunsch_affine.rs``, ``src/parse.rs``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import
this module, and only as the checker.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "librefcpu.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class _Mats(C.Structure):
    _fields_ = [("lq", C.c_size_t), ("ld", C.c_size_t),
                ("M", C.POINTER(C.c_int32)), ("I", C.POINTER(C.c_int32)),
                ("D", C.POINTER(C.c_int32)),
                ("pM", C.POINTER(C.c_uint8)), ("pI", C.POINTER(C.c_uint8)),
                ("pD", C.POINTER(C.c_uint8))]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        u8p = C.POINTER(C.c_uint8)
        L.ref_nw_fill.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t, C.POINTER(_Mats)]
        L.ref_nw_free.argtypes = [C.POINTER(_Mats)]
        L.ref_nw_dense_mask.argtypes = [C.POINTER(_Mats), u8p]
        L.ref_nw_score.argtypes = [C.POINTER(_Mats), u8p]
        L.ref_nw_score.restype = C.c_int32
        L.ref_nw_traceback_dfs.argtypes = [u8p, u8p, C.POINTER(_Mats), C.c_char_p, C.c_size_t,
                                           C.POINTER(C.c_size_t), C.c_uint64,
                                           C.POINTER(C.c_uint64)]
        L.ref_nw_dag_summary.argtypes = [u8p, u8p, C.POINTER(_Mats), C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_int), C.c_char_p, C.c_size_t,
                                         C.POINTER(C.c_int64)]
        L.ref_nw_run_pairs.argtypes = [u8p, C.POINTER(C.c_uint64), u8p, C.POINTER(C.c_uint64),
                                       C.c_uint64, C.c_uint64]
        L.ref_nw_run_pairs.restype = C.c_uint64
        L.ref_nw_run_pairs_mt.argtypes = [u8p, C.POINTER(C.c_uint64), u8p, C.POINTER(C.c_uint64),
                                          C.c_uint64, C.c_uint64, C.c_int]
        L.ref_nw_run_pairs_mt.restype = C.c_uint64
        L.ref_nw_run_pairs_capped.argtypes = [u8p, C.POINTER(C.c_uint64), u8p,
                                              C.POINTER(C.c_uint64), C.c_uint64, C.c_uint64,
                                              C.c_uint64, C.POINTER(C.c_uint64)]
        L.ref_nw_run_pairs_capped.restype = C.c_uint64
        L.ref_nw_run_pairs_mt_capped.argtypes = [u8p, C.POINTER(C.c_uint64), u8p,
                                                 C.POINTER(C.c_uint64), C.c_uint64, C.c_uint64,
                                                 C.c_uint64, C.c_int, C.POINTER(C.c_uint64)]
        L.ref_nw_traceback_dfs_blocks.argtypes = [u8p, u8p, C.POINTER(_Mats), C.c_char_p,
                                                  C.c_size_t, C.POINTER(C.c_size_t), C.c_uint64,
                                                  C.c_uint64, C.POINTER(C.c_uint64)]
        L.ref_nw_run_pairs_mt_capped.restype = C.c_uint64
        L.ref_nw_run_pairs_text_mt.argtypes = [u8p, C.POINTER(C.c_uint64), u8p,
                                               C.POINTER(C.c_uint64), C.c_uint64, C.c_uint64,
                                               C.c_uint64, C.c_int, C.c_int, C.c_uint64,
                                               C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.ref_nw_run_pairs_text_mt.restype = C.c_uint64
        L.ref_nw_check_pairs_mt.argtypes = [u8p, C.POINTER(C.c_uint64), u8p,
                                            C.POINTER(C.c_uint64), C.c_uint64,
                                            C.POINTER(C.c_uint64), C.POINTER(C.c_int32), u8p, u8p,
                                            C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.c_int]
        L.ref_nw_first_linear.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t, C.c_int,
                                          C.POINTER(C.c_int32), u8p, C.POINTER(C.c_int),
                                          C.c_char_p, C.c_size_t, C.POINTER(C.c_int64),
                                          C.POINTER(C.c_uint64)]
        L.ref_nw_score_linear.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t, C.c_int,
                                          C.POINTER(C.c_int32), u8p, C.POINTER(C.c_int)]
        L.ref_parse_fasta.argtypes = [u8p, C.c_size_t, C.c_int, u8p, C.c_size_t,
                                      C.POINTER(C.c_size_t), u8p, C.c_size_t,
                                      C.POINTER(C.c_size_t)]
        L.ref_parse_fasta.restype = C.c_int64
        i32p = C.POINTER(C.c_int32)
        L.ref_affine_penalty.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t, C.c_int32, C.c_int32,
                                         C.c_int32]
        L.ref_affine_penalty.restype = C.c_int64
        L.ref_affine_run_pairs.argtypes = [u8p, C.POINTER(C.c_uint64), u8p, C.POINTER(C.c_uint64),
                                           C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                           C.c_uint64, C.c_int32, C.c_int32, C.c_int32, C.c_int,
                                           C.POINTER(C.c_int64)]
        L.ref_wfa_align.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t, C.c_int, C.c_uint64,
                                    C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.ref_wfa_tensor_new.argtypes = [i32p, i32p, i32p, i32p, C.c_char_p, C.c_size_t]
        L.ref_wfa_tensor_new.restype = C.c_int64
        L.ref_wfa_initial_converged.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t]
        _lib = L
    return _lib


def _u8(b: bytes):
    buf = (C.c_uint8 * max(1, len(b))).from_buffer_copy(b if b else b"\0")
    return buf


@dataclass
class NwOracle:
    score: int
    end_states: int          # bit0 M, bit1 I, bit2 D
    dense_mask: np.ndarray   # (ld+1, lq+1) uint8, same bit meaning as the product export
    M: np.ndarray
    I: np.ndarray
    D: np.ndarray
    stdout: str | None       # literal DFS output (None when not requested)
    dfs_rc: int | None       # 0 finished, 1 panic, 2 pop cap, 3 block cap (max_blocks)
    dfs_blocks: int | None
    n_blocks: int            # memoised DFS: blocks printed before the first panic
    panics: bool
    first_ops: str | None    # first printed alignment ('=','X','I','D'), None if none printed


def nw(query: bytes, db: bytes, *, literal_dfs: bool = True, max_pops: int = 2_000_000,
       out_cap: int = 1 << 22, max_blocks: int = 0) -> NwOracle:
    L = lib()
    q, d = _u8(query), _u8(db)
    m = _Mats()
    if L.ref_nw_fill(q, len(query), d, len(db), C.byref(m)) != 0:
        raise MemoryError("oracle fill")
    try:
        H, W = len(db) + 1, len(query) + 1
        dense = np.zeros((H, W), np.uint8)
        L.ref_nw_dense_mask(C.byref(m), dense.ctypes.data_as(C.POINTER(C.c_uint8)))
        es = C.c_uint8(0)
        score = L.ref_nw_score(C.byref(m), C.byref(es))
        Mv = np.ctypeslib.as_array(m.M, shape=(H * W,)).reshape(H, W).copy()
        Iv = np.ctypeslib.as_array(m.I, shape=(H * W,)).reshape(H, W).copy()
        Dv = np.ctypeslib.as_array(m.D, shape=(H * W,)).reshape(H, W).copy()
        text = rc = blocks = None
        if literal_dfs:
            out = C.create_string_buffer(out_cap)
            olen = C.c_size_t(0)
            nb = C.c_uint64(0)
            rc = L.ref_nw_traceback_dfs_blocks(q, d, C.byref(m), out, out_cap, C.byref(olen),
                                               max_pops, max_blocks, C.byref(nb))
            text = out.raw[:min(olen.value, out_cap)].decode("latin-1")
            blocks = nb.value
        nbk = C.c_uint64(0)
        pan = C.c_int(0)
        cap = len(query) + len(db) + 1
        ops = C.create_string_buffer(cap)
        olen2 = C.c_int64(0)
        L.ref_nw_dag_summary(q, d, C.byref(m), C.byref(nbk), C.byref(pan), ops, cap,
                             C.byref(olen2))
        first = ops.raw[:olen2.value].decode() if olen2.value >= 0 else None
        return NwOracle(score, es.value, dense, Mv, Iv, Dv, text, rc, blocks, nbk.value,
                        bool(pan.value), first)
    finally:
        L.ref_nw_free(C.byref(m))


def nw_score_linear(query: bytes, db: bytes, threads: int = 0) -> tuple[int, int, bool]:
    """(score, end_states, panics) of one pair in linear memory (reflinear.c),
    for pairs too large for the full-matrix oracle (configs[3])."""
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    sc, es, pan = C.c_int32(0), C.c_uint8(0), C.c_int(0)
    if lib().ref_nw_score_linear(_u8(query), len(query), _u8(db), len(db), threads,
                                 C.byref(sc), C.byref(es), C.byref(pan)) != 0:
        raise MemoryError("oracle linear fill")
    return sc.value, es.value, bool(pan.value)


def nw_first_linear(query: bytes, db: bytes, threads: int = 0):
    """(score, end_states, panics, first_ops or None, dead_nodes) of one pair:
    the linear-memory fill keeping 1 B of parent sets per cell and the
    reference DFS's first event over them (reflinear.c), for pairs too large
    for the full-matrix oracle; dead_nodes > 0 means the DFS backtracked out
    of sentinel-rooted subtrees before its first event."""
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    sc, es, pan = C.c_int32(0), C.c_uint8(0), C.c_int(0)
    cap = len(query) + len(db) + 1
    ops = C.create_string_buffer(cap)
    olen, dead = C.c_int64(0), C.c_uint64(0)
    if lib().ref_nw_first_linear(_u8(query), len(query), _u8(db), len(db), threads, C.byref(sc),
                                 C.byref(es), C.byref(pan), ops, cap, C.byref(olen),
                                 C.byref(dead)) != 0:
        raise MemoryError("oracle linear first alignment")
    first = ops.raw[:olen.value].decode() if olen.value >= 0 else None
    return sc.value, es.value, bool(pan.value), first, dead.value


def run_pairs(qs: bytes, q_off: np.ndarray, ds: bytes, d_off: np.ndarray, n_pairs: int,
              max_pops: int = 100_000) -> int:
    """Timed CPU baseline body: literal fill + DFS over n_pairs (CSR inputs)."""
    L = lib()
    qo = np.ascontiguousarray(q_off, np.uint64)
    do = np.ascontiguousarray(d_off, np.uint64)
    return L.ref_nw_run_pairs(_u8(qs), qo.ctypes.data_as(C.POINTER(C.c_uint64)), _u8(ds),
                              do.ctypes.data_as(C.POINTER(C.c_uint64)), n_pairs, max_pops)


def run_pairs_capped(qs: bytes, q_off: np.ndarray, ds: bytes, d_off: np.ndarray, n_pairs: int,
                     max_pops: int = 100_000, threads: int = 1,
                     max_blocks: int = 0) -> tuple[int, int]:
    """(cells, pairs whose DFS stopped at max_pops) of run_pairs / run_pairs_mt
    (max_blocks > 0: each DFS also stops before its (max_blocks+1)-th block)."""
    L = lib()
    qo = np.ascontiguousarray(q_off, np.uint64)
    do = np.ascontiguousarray(d_off, np.uint64)
    nc = C.c_uint64(0)
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint64))  # noqa: E731
    if threads <= 1:
        cells = L.ref_nw_run_pairs_capped(_u8(qs), P(qo), _u8(ds), P(do), n_pairs, max_pops,
                                          max_blocks, C.byref(nc))
    else:
        cells = L.ref_nw_run_pairs_mt_capped(_u8(qs), P(qo), _u8(ds), P(do), n_pairs, max_pops,
                                             max_blocks, threads, C.byref(nc))
    return int(cells), int(nc.value)


def run_pairs_text(qs: bytes, q_off: np.ndarray, ds: bytes, d_off: np.ndarray, n_pairs: int,
                   fd: int, max_pops: int = 100_000, threads: int = 1, max_blocks: int = 0,
                   chunk: int = 4096) -> tuple[int, int, int]:
    """(cells, text bytes, capped pairs): the pair loop with the reference's
    text of every pair written to file descriptor `fd` in pair order
    (refmt.c ref_nw_run_pairs_text_mt; the CLI's text-inclusive CPU baseline)."""
    L = lib()
    qo = np.ascontiguousarray(q_off, np.uint64)
    do = np.ascontiguousarray(d_off, np.uint64)
    nb, nc = C.c_uint64(0), C.c_uint64(0)
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint64))  # noqa: E731
    cells = L.ref_nw_run_pairs_text_mt(_u8(qs), P(qo), _u8(ds), P(do), n_pairs, max_pops,
                                       max_blocks, threads, fd, chunk, C.byref(nb), C.byref(nc))
    return int(cells), int(nb.value), int(nc.value)


def run_pairs_mt(qs: bytes, q_off: np.ndarray, ds: bytes, d_off: np.ndarray, n_pairs: int,
                 max_pops: int = 100_000, threads: int = 1) -> int:
    """run_pairs over contiguous slices of the pairs on `threads` threads."""
    L = lib()
    qo = np.ascontiguousarray(q_off, np.uint64)
    do = np.ascontiguousarray(d_off, np.uint64)
    return L.ref_nw_run_pairs_mt(_u8(qs), qo.ctypes.data_as(C.POINTER(C.c_uint64)), _u8(ds),
                                 do.ctypes.data_as(C.POINTER(C.c_uint64)), n_pairs, max_pops,
                                 threads)


@dataclass
class BatchCheck:
    score: np.ndarray       # int32[n]
    end_states: np.ndarray  # uint8[n]
    panics: np.ndarray      # bool[n]
    cig_len: np.ndarray     # int32[n], -1 = nothing printed
    cig_off: np.ndarray     # uint64[n+1]
    cig: np.ndarray         # uint32 CIGAR words, pair p at cig_off[p]

    def cigar_words(self, p: int) -> np.ndarray | None:
        n = int(self.cig_len[p])
        return None if n < 0 else self.cig[int(self.cig_off[p]):int(self.cig_off[p]) + n]


def check_pairs(qs, q_off, ds, d_off, threads: int = 0) -> BatchCheck:
    """Reference results of every pair (k-th query slice vs k-th db slice of
    the CSR inputs): literal fill + memoised DFS (refcheck.c), on threads."""
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    qs = np.ascontiguousarray(np.frombuffer(bytes(qs), np.uint8) if isinstance(qs, (bytes, bytearray)) else qs, np.uint8)
    ds = np.ascontiguousarray(np.frombuffer(bytes(ds), np.uint8) if isinstance(ds, (bytes, bytearray)) else ds, np.uint8)
    qo = np.ascontiguousarray(q_off, np.uint64)
    do = np.ascontiguousarray(d_off, np.uint64)
    n = len(qo) - 1
    span = (qo[1:] - qo[:-1]) + (do[1:] - do[:-1])
    co = np.zeros(n + 1, np.uint64)
    co[1:] = np.cumsum(span)
    out = BatchCheck(np.zeros(n, np.int32), np.zeros(n, np.uint8), np.zeros(n, np.uint8),
                     np.zeros(n, np.int32), co, np.zeros(max(1, int(co[-1])), np.uint32))
    P = lambda a, t: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    rc = lib().ref_nw_check_pairs_mt(P(qs if len(qs) else np.zeros(1, np.uint8), C.c_uint8),
                                      P(qo, C.c_uint64),
                                      P(ds if len(ds) else np.zeros(1, np.uint8), C.c_uint8),
                                      P(do, C.c_uint64), n, P(co, C.c_uint64),
                                      P(out.score, C.c_int32), P(out.end_states, C.c_uint8),
                                      P(out.panics, C.c_uint8), P(out.cig_len, C.c_int32),
                                      P(out.cig, C.c_uint32), threads)
    if rc != 0:
        raise MemoryError("oracle check_pairs")
    out.panics = out.panics.astype(bool)
    return out


def parse_fasta_bytes(data: bytes, valid_ext: bool = True):
    """Returns (records [(name, seq)], bad_chars bytes) or None for FastaError."""
    L = lib()
    cap = len(data) * 2 + 64
    out = (C.c_uint8 * cap)()
    rl = C.c_size_t(0)
    bad = (C.c_uint8 * (len(data) + 1))()
    nb = C.c_size_t(0)
    n = L.ref_parse_fasta(_u8(data), len(data), int(valid_ext), out, cap, C.byref(rl), bad,
                          len(data) + 1, C.byref(nb))
    if n < 0:
        return None
    raw = bytes(out)[:rl.value]
    recs, o = [], 0
    for _ in range(n):
        nl = int.from_bytes(raw[o:o + 4], "little"); o += 4
        name = raw[o:o + nl]; o += nl
        sl = int.from_bytes(raw[o:o + 4], "little"); o += 4
        seq = raw[o:o + sl]; o += sl
        recs.append((name, seq))
    return recs, bytes(bad)[:nb.value]


# ----------------------------------------------------------------------- WFA
class _WfaRes(C.Structure):
    _fields_ = [("status", C.c_int32), ("steps", C.c_uint64), ("score", C.c_int64),
                ("aln_len1", C.c_uint64), ("aln_len2", C.c_uint64)]


WFA_OK, WFA_NOT_IMPLEMENTED, WFA_PANIC_TRIM, WFA_PANIC_SLICE, WFA_NONCONVERGED = 0, 1, 3, 4, 5
_STATES = "MDI"  # enum State { M, D, I } (wfa.rs:44-50)


@dataclass
class WfaOracle:
    status: int
    steps: int
    score: int            # printed score: wfs.len()
    stdout: str
    aln_len1: int
    aln_len2: int


def wfa(query: bytes, db: bytes, *, mode: int = 0, max_steps: int = 0) -> WfaOracle:
    """wfa_align(seq1=query, seq2=db, mode) (wfa.rs:23-42), release semantics."""
    L = lib()
    res = _WfaRes()
    n = C.c_size_t()
    L.ref_wfa_align(_u8(query), len(query), _u8(db), len(db), mode, max_steps, C.byref(res),
                    None, 0, C.byref(n))
    buf = C.create_string_buffer(n.value + 1)
    L.ref_wfa_align(_u8(query), len(query), _u8(db), len(db), mode, max_steps, C.byref(res),
                    buf, n.value + 1, C.byref(n))
    return WfaOracle(res.status, res.steps, res.score, buf.raw[:n.value].decode("latin-1"),
                     res.aln_len1, res.aln_len2)


def _enc_front(f):
    if f is None:
        return [0, 0, 0, 0]
    out = [1, f["lo"], f["hi"], len(f["elements"])]
    for e in f["elements"]:
        if e is None:
            out += [0] * 7
        else:
            off, st, par = e
            p = [_STATES.index(x) for x in par] + [0, 0, 0]
            out += [1, off, _STATES.index(st), len(par)] + p[:3]
    return out


def _enc_tensor(t):
    if t is None:
        return None
    arr = [1] + _enc_front(t.get("i")) + _enc_front(t.get("d")) + _enc_front(t.get("m"))
    return (C.c_int32 * len(arr))(*arr)


def _dec_front(a, k):
    some, lo, hi, n = a[k:k + 4]
    k += 4
    els = []
    for _ in range(n):
        s, off, st, np_, p0, p1, p2 = a[k:k + 7]
        k += 7
        els.append((off, _STATES[st], [_STATES[x] for x in (p0, p1, p2)[:np_]]) if s else None)
    return ({"lo": lo, "hi": hi, "elements": els} if some else None), k


def wfa_tensor_new(o=None, e=None, x=None):
    """WaveFrontTensor::new(o, e, x) (wfa.rs:225-420) on tensors given as
    {'i'|'d'|'m': None | {'lo', 'hi', 'elements': [None | (offset, state,
    [parents])]}} -> (tensor or None, printed text)."""
    L = lib()
    out = (C.c_int32 * 65536)()
    txt = C.create_string_buffer(256)
    L.ref_wfa_tensor_new(_enc_tensor(o), _enc_tensor(e), _enc_tensor(x), out, txt, 256)
    a = list(out)
    if not a[0]:
        return None, txt.value.decode()
    i, k = _dec_front(a, 1)
    d, k = _dec_front(a, k)
    m, k = _dec_front(a, k)
    return {"i": i, "d": d, "m": m}, txt.value.decode()


def wfa_initial_converged(query: bytes, db: bytes) -> bool:
    """Ocean::global().is_converged(query, db) (test_converge, wfa.rs:1289-1294)."""
    return bool(lib().ref_wfa_initial_converged(_u8(query), len(query), _u8(db), len(db)))


def affine_penalty(query: bytes, db: bytes, x: int = 4, o: int = 2, e: int = 6) -> int:
    """Minimum gap-affine penalty of a global alignment (oracle/refaffine.c):
    the value the corrected gap-affine WFA computes."""
    return int(lib().ref_affine_penalty(_u8(query), len(query), _u8(db), len(db), x, o, e))


def affine_run_pairs(qs: np.ndarray, q_off: np.ndarray, ds: np.ndarray, d_off: np.ndarray,
                     pair_q: np.ndarray, pair_d: np.ndarray, x: int = 4, o: int = 2, e: int = 6,
                     threads: int = 1) -> np.ndarray:
    """affine_penalty over (query, db) index pairs on `threads` threads."""
    qs = np.ascontiguousarray(qs, np.uint8)
    ds = np.ascontiguousarray(ds, np.uint8)
    qo = np.ascontiguousarray(q_off, np.uint64)
    do = np.ascontiguousarray(d_off, np.uint64)
    pq = np.ascontiguousarray(pair_q, np.uint32)
    pd = np.ascontiguousarray(pair_d, np.uint32)
    out = np.zeros(len(pq), np.int64)
    P = lambda a, t: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    lib().ref_affine_run_pairs(P(qs, C.c_uint8), P(qo, C.c_uint64), P(ds, C.c_uint8),
                               P(do, C.c_uint64), P(pq, C.c_uint32), P(pd, C.c_uint32), len(pq),
                               x, o, e, threads, P(out, C.c_int64))
    return out
