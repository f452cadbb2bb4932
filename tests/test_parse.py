"""CPU: FASTA parser (libsaln, parse.rs:54-99) against the reference's own
tests (parse.rs:166-251) and against the oracle restatement."""
import os

import numpy as np
import pytest


def _write(tmp_path, name, data: bytes):
    p = tmp_path / name
    p.write_bytes(data)
    return str(p)


def test_parse_good_fasta(saln, tmp_path):  # parse.rs:166-186
    p = _write(tmp_path, "x.fa", b">Record1\nATGCATGCATGCATGCATGCATGCATGC\n>Record2\nATGCATGCGTGCAGTGACCACA")
    r = saln.parse_fasta(p)
    assert len(r.records) == 2
    assert len(r.records[0].name) == 8
    assert len(r.records[0].seq) == 28


def test_parse_bad_header(saln, tmp_path):  # parse.rs:188-215
    p = _write(tmp_path, "x.fa", b">Record1\nATGCATGCATGCATGCATGCATGCATGC\nRecord2\nATGCATGCGTGCAGTGACCACA")
    with pytest.raises(saln.CharError) as e:
        saln.parse_fasta(p)
    assert e.value.chars == ["R", "e", "c", "o", "r", "d", "2"]
    rec = e.value.res.records[0]
    assert rec.name == b">Record1"
    assert rec.seq == b"ATGCATGCATGCATGCATGCATGCATGCATGCATGCGTGCAGTGACCACA"


def test_parse_bad_nt(saln, tmp_path):  # parse.rs:217-238
    p = _write(tmp_path, "x.fa", b">Record1\nATGCATGCAKGCATGCATGCANNNGCATGC")
    with pytest.raises(saln.CharError) as e:
        saln.parse_fasta(p)
    assert e.value.chars == ["K"]
    assert e.value.res.records[0].seq == b"ATGCATGCAGCATGCATGCANNNGCATGC"


def test_parse_false_file(saln, tmp_path):  # parse.rs:240-251
    p = _write(tmp_path, "x.txt", b">a\nACGT\n")
    with pytest.raises(saln.FastaError):
        saln.parse_fasta(p)


@pytest.mark.parametrize("name,ok", [("a.fa", True), ("a.fasta", True), ("a.fna", True),
                                     ("a.FA", False), ("a.fa.gz", False), (".fa", False),
                                     ("a", False), ("a.fastq", False)])
def test_extensions(saln, tmp_path, name, ok):
    p = _write(tmp_path, name, b">a\nACGT\n")
    if ok:
        assert saln.parse_fasta(p).records[0].seq == b"ACGT"
    else:
        with pytest.raises(saln.FastaError):
            saln.parse_fasta(p)


def test_missing_file(saln, tmp_path):
    with pytest.raises(saln.FastaError):
        saln.parse_fasta(str(tmp_path / "nope.fa"))


def test_fuzz_vs_oracle(saln, oracle):
    rng = np.random.default_rng(9)
    alphabet = np.frombuffer(b"ACGTNacgtn>\n\rXK ", np.uint8)
    for _ in range(300):
        n = int(rng.integers(0, 200))
        data = alphabet[rng.integers(0, len(alphabet), n)].tobytes()
        ref = oracle.parse_fasta_bytes(data)
        assert ref is not None
        ref_recs, ref_bad = ref
        try:
            got = saln.parse_fasta_bytes(data)
            got_bad = b""
        except saln.CharError as e:
            got = e.res
            got_bad = bytes(ord(c) for c in e.chars)
        assert [(r.name, r.seq) for r in got.records] == ref_recs
        assert got_bad == ref_bad
