"""CPU: deterministic generators, CSR packing, mask geometry."""
import numpy as np

from sequencealigning_amd import synth
from sequencealigning_amd.nw import alignment_rows, pack_csr


def test_splitmix64_matches_oracle(oracle):
    import ctypes
    L = oracle.lib()
    L.ref_splitmix64.restype = ctypes.c_uint64
    st = ctypes.c_uint64(0x5EED0002)
    ref = [L.ref_splitmix64(ctypes.byref(st)) for _ in range(16)]
    assert synth.splitmix64(0x5EED0002, 16).tolist() == ref


def test_iid_pairs_shape_and_determinism():
    a = synth.iid_pairs(10, 150, 150, seed=1)
    b = synth.iid_pairs(10, 150, 150, seed=1)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    q, qo, d, do = a
    assert len(q) == 1500 and qo[-1] == 1500 and set(q.tobytes()) <= set(b"ACGT")


def test_mutate_rate():
    q, d = synth.mut_pair(20000, 0.05, 7)
    assert len(q) == 20000
    assert abs(len(d) - len(q)) < 400
    assert set(d) <= set(b"ACGT")


def test_pack_csr():
    buf, off = pack_csr([b"AC", b"", b"GGT"])
    assert off.tolist() == [0, 2, 2, 5]
    assert buf.tobytes() == b"ACGGT"


def test_alignment_rows():
    assert alignment_rows(b"AAA", b"AA", [(1, "="), (1, "I"), (1, "=")]) == ("AAA", "| |", "A-A")


def test_mutate_matches_per_base_definition():
    """synth.mutate (vectorised) == the per-base G-mut(delta) definition of
    SURVEY.md §8(d)."""
    from sequencealigning_amd import synth

    def slow(seq, delta, seed):
        s = np.frombuffer(bytes(seq), np.uint8)
        n = len(s)
        r = synth.splitmix64(seed, 3 * n)
        u = (r[:n] >> np.uint64(11)).astype(np.float64) / float(1 << 53)
        ev = (r[n:2 * n] >> np.uint64(62)).astype(np.int64)
        rb = (r[2 * n:] >> np.uint64(60)).astype(np.int64)
        out = []
        for k in range(n):
            c = int(np.searchsorted(synth.BASES, s[k]))
            if u[k] >= delta:
                out.append(int(s[k]))
            elif ev[k] <= 1:
                out.append(int(synth.BASES[(c + 1 + (rb[k] % 3)) % 4]))
            elif ev[k] == 2:
                out.append(int(s[k]))
                out.append(int(synth.BASES[rb[k] & 3]))
        return bytes(out)

    for seed, n, delta in [(1, 0, 0.1), (2, 1, 0.9), (3, 2000, 0.05), (4, 3000, 0.5)]:
        q = synth.random_bases(seed, n).tobytes()
        assert synth.mutate(q, delta, seed) == slow(q, delta, seed)


def test_torch_mut_pairs_equal_numpy_generators():
    """synth.mut_pairs_torch (bench's configs[2] generator, run on the GPU
    there) is bit-identical to the numpy random_bases + mutate pairs."""
    from sequencealigning_amd import synth
    n, L = 23, 300
    qs, qo, ds, do = synth.mut_pairs_torch(n, L, 0.05, 0x5EED0003, "cpu", chunk=7)
    allq = synth.random_bases(0x5EED0003, n * L).tobytes()
    for k in range(n):
        q = allq[k * L:(k + 1) * L]
        assert bytes(qs[int(qo[k]):int(qo[k + 1])].numpy()) == q
        assert bytes(ds[int(do[k]):int(do[k + 1])].numpy()) == synth.mutate(q, 0.05, seed=k)
