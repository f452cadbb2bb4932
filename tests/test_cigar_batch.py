"""CPU: the Python batch API's lazily decoded CIGARs (sequencealigning_amd.nw.CigarBatch)."""


def test_cigar_batch_sequence_semantics():
    """nw_align_batch's CIGARs (CigarBatch) read like the list of
    [(length, op), ...] they stand for: index, negative index, slice,
    iteration, equality with lists and with another batch, pickling (the
    multi-GPU gather sends them through a queue)."""
    import pickle

    import numpy as np

    from sequencealigning_amd.nw import CigarBatch
    words = np.array([(3 << 4) | 7, (1 << 4) | 8, 0xdead, (2 << 4) | 1, (5 << 4) | 2], np.uint32)
    cb = CigarBatch(words, np.array([0, 3, 3], np.uint64), np.array([2, 0, 2], np.uint32))
    want = [[(3, "="), (1, "X")], [], [(2, "I"), (5, "D")]]
    assert len(cb) == 3 and cb[0] == want[0] and cb[-1] == want[2] and cb[1] == []
    assert cb[1:] == want[1:] and list(cb) == want
    assert cb == want and want == cb and not (cb != want)
    assert cb != want[:2] and cb != [want[0], want[2], want[1]]
    assert pickle.loads(pickle.dumps(cb)) == cb
    assert list(cb.words(2)) == [(2 << 4) | 1, (5 << 4) | 2]


def test_cigar_batch_list_operations():
    """list-only operations on a CigarBatch (concatenation,
    json.dumps through tolist(), isinstance(list)) have a real-list path."""
    import json

    import numpy as np

    from sequencealigning_amd.nw import CigarBatch
    words = np.array([(3 << 4) | 7, (2 << 4) | 1], np.uint32)
    cb = CigarBatch(words, np.array([0, 1], np.uint64), np.array([1, 1], np.uint32))
    lst = cb.tolist()
    assert isinstance(lst, list) and lst == [[(3, "=")], [(2, "I")]]
    assert cb + [[(1, "X")]] == lst + [[(1, "X")]]
    assert [[(1, "X")]] + cb == [[(1, "X")]] + lst
    assert json.loads(json.dumps(cb.tolist())) == [[[3, "="]], [[2, "I"]]]
