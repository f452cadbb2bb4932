"""Input types and errors, mirroring ``src/parse.rs`` and ``src/errors.rs``.

``Record``/``Records`` (parse.rs:107-139), ``Mode``/``Algo`` (parse.rs:36-50),
``parse_fasta`` (parse.rs:54-99, implemented natively in ``libsaln.so``) and
the ``AlignerError`` family (errors.rs:7-15).
"""
from __future__ import annotations

import ctypes as C
import enum
import os
from dataclasses import dataclass, field

from . import _lib


class AlignerError(Exception):
    """errors.rs:8 ``AlignerError``."""


class FastaError(AlignerError):
    """``FastaError(io::Error)``: "Fasta could not be opened with err: {0}"."""

    def __init__(self, err: str):
        self.err = err
        super().__init__(f"Fasta could not be opened with err: {err}")


class AlignmentError(AlignerError):
    """``AlignmentError(&str)``: "Error in alignment: {0}"."""

    def __init__(self, msg: str):
        self.msg = msg
        super().__init__(f"Error in alignment: {msg}")


class CharError(AlignerError):
    """``CharError{res, chars}``: records parsed with the invalid bytes dropped."""

    def __init__(self, res: "Records", chars: list[str]):
        self.res = res
        self.chars = chars
        super().__init__(f"Invalid character: {chars!r}")


class Mode(enum.IntEnum):  # parse.rs:44-50; clap value names global/local/semi-global
    Global = 0
    Local = 1
    SemiGlobal = 2

    @classmethod
    def parse(cls, s: str) -> "Mode":
        return {"global": cls.Global, "local": cls.Local, "semi-global": cls.SemiGlobal}[s]


class Algo(enum.IntEnum):  # parse.rs:36-42; a-star is out of scope for this engine
    AStar = 0
    NeedlemanWunsch = 1
    Wfa = 2

    @classmethod
    def parse(cls, s: str) -> "Algo":
        return {"a-star": cls.AStar, "needleman-wunsch": cls.NeedlemanWunsch,
                "wfa": cls.Wfa}[s]


@dataclass
class Record:  # parse.rs:135-139
    seq: bytes = b""
    name: bytes = b""


@dataclass
class Records:  # parse.rs:107-110
    records: list[Record] = field(default_factory=list)

    def __len__(self):
        return len(self.records)

    def __iter__(self):
        return iter(self.records)


def _records_from_handle(h: C.c_void_p) -> Records:
    L = _lib.lib()
    out = Records()
    n = L.saln_records_count(h)
    name_p, seq_p = C.c_void_p(), C.c_void_p()
    nl, sl = C.c_uint64(), C.c_uint64()
    for i in range(n):
        _lib.check(L.saln_records_get(h, i, C.byref(name_p), C.byref(nl), C.byref(seq_p),
                                      C.byref(sl)), "saln_records_get")
        name = C.string_at(name_p, nl.value) if nl.value else b""
        seq = C.string_at(seq_p, sl.value) if sl.value else b""
        out.records.append(Record(seq=seq, name=name))
    L.saln_records_free(h)
    return out


def _finish(rc: int, h: C.c_void_p, bad, nbad: C.c_uint64) -> Records:
    if rc == _lib.E_FASTA:
        raise FastaError(_lib.last_error().replace("Fasta could not be opened with err: ", ""))
    if rc not in (_lib.OK, _lib.E_FASTA_CHARS):
        raise _lib.SalnError(rc, "saln_parse_fasta")
    recs = _records_from_handle(h)
    if rc == _lib.E_FASTA_CHARS:
        chars = [chr(b) for b in bytes(bad)[:min(nbad.value, len(bad))]]
        raise CharError(recs, chars)
    return recs


def parse_fasta(path: str | os.PathLike) -> Records:
    """parse.rs:54-99. Raises FastaError / CharError like the reference's Err."""
    L = _lib.lib()
    h = C.c_void_p()
    size = os.path.getsize(path) if os.path.exists(path) else 0
    bad = (C.c_uint8 * (size + 1))()
    nbad = C.c_uint64(0)
    rc = L.saln_parse_fasta(os.fsencode(path), C.byref(h), bad, size + 1, C.byref(nbad))
    return _finish(rc, h, bad, nbad)


def parse_fasta_bytes(data: bytes) -> Records:
    """Same parser on an in-memory buffer (no extension check)."""
    L = _lib.lib()
    h = C.c_void_p()
    bad = (C.c_uint8 * (len(data) + 1))()
    nbad = C.c_uint64(0)
    buf = C.create_string_buffer(data, len(data)) if data else None
    rc = L.saln_parse_fasta_buffer(buf, len(data), C.byref(h), bad, len(data) + 1, C.byref(nbad))
    return _finish(rc, h, bad, nbad)
