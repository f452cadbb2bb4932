"""CPU: the column-span driver of one long pair (SURVEY.md §8(f) #3,
sequencealigning_amd/span.py) on gloo at world sizes 2 and 3.

The per-rank compute is a CPU span engine (below, test-only) that restates
the span contract of include/saln.h: it fills query columns col_lo+1 ..
col_hi of every db row from the boundary rows its left neighbour sent
(needleman_wunsch_affine.rs:217-236 on V' = 2V + p, nw_common.hpp) and walks
its part of the first printed path (walk_greedy / the span walker's crossing
rules, nw_kernels.hip).  The driver's band relay, the right-to-left walk over
the ranks, the dead-end retry and the CIGAR assembly are the product's; the
assembled result must equal the oracle's (refcpu: score, end states, panic,
first printed alignment)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

SENT = -32768
SCHEME = (5, -4, -8, -6)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _CpuSpanEngine:
    """Span of columns lo+1 .. hi (test engine; V' = 2V + p, flags ORed by max)."""

    def __init__(self, q, d, lo, hi, scoring=SCHEME):
        self.q = np.frombuffer(q, np.uint8).astype(np.int64)
        self.d = np.frombuffer(d, np.uint8).astype(np.int64)
        self.lq, self.ld, self.lo, self.hi = len(q), len(d), lo, hi
        self.m, self.x, self.go, self.ge = scoring
        self.out = None
        self.inbox = None
        self.have = 0  # inbox rows delivered (band relay)

    # band relay: the fill "runs" row by row as far as its inbox allows; a
    # request for outbox rows past the delivered inbox is a protocol error
    def start_fill(self):
        self.inbox = np.zeros(self.ld, np.int64)
        self.have = 0 if self.lo > 0 else self.ld
        self.out = None

    def put_inbox(self, a, b, rows):
        assert a == self.have + 1, ("bands out of order", a, self.have)
        self.inbox[a - 1:b] = rows
        self.have = b

    def outbox_rows(self, a, b):
        assert self.have >= b, ("outbox rows requested before their inbox rows", b, self.have)
        if self.out is None and self.have == self.ld:
            self.fill(self.inbox if self.lo > 0 else None)
        if self.out is None:  # partial: rows 1 .. b from the rows delivered so far
            part = _CpuSpanEngine(bytes(self.q.astype(np.uint8)), bytes(self.d[:b].astype(np.uint8)),
                                  self.lo, self.hi, (self.m, self.x, self.go, self.ge))
            part.fill(self.inbox[:b] if self.lo > 0 else None)
            return part.out[a - 1:b]
        return self.out[a - 1:b]

    def d_row0(self, j):
        return (j + 1) * self.ge + self.go

    def i_col0(self, i):
        return self.go + (i + 1) * self.ge

    def fill(self, inbox):
        lo, hi, ld = self.lo, self.hi, self.ld
        W = hi - lo
        js = np.arange(lo + 1, hi + 1)
        go2, ge2 = 2 * self.go, 2 * self.ge
        M = np.empty((ld + 1, W), np.int64)
        I = np.empty_like(M)
        D = np.empty_like(M)
        M[0] = I[0] = 2 * SENT
        D[0] = 2 * self.d_row0(js) + 1  # row-0 D: panic nodes
        H = np.maximum(np.maximum(M[0], I[0]), D[0])
        if lo == 0:
            hleft = lambda r: 0 if r == 0 else max(2 * SENT, 2 * self.i_col0(r) + 1)
            icand = lambda r: max(2 * SENT + go2, 2 * self.i_col0(r) + 1) + ge2
        else:
            h0 = max(2 * SENT, 2 * self.d_row0(lo) + 1)
            hl = np.concatenate([[h0], (inbox << 32) >> 32])  # low words, sign-extended
            ic = inbox >> 32
            hleft = lambda r: int(hl[r])
            icand = lambda r: int(ic[r - 1])
        sub = np.where(self.q[js - 1][None, :] == self.d[:, None], 2 * self.m, 2 * self.x)
        k = np.arange(W)
        for r in range(1, ld + 1):
            diag = np.concatenate([[hleft(r - 1)], H[:-1]])
            Mr = diag + sub[r - 1]
            Dr = np.maximum(M[r - 1] + go2, D[r - 1]) + ge2
            # I[c] = max(M[c-1] + go2, I[c-1]) + ge2, I[0] = icand: a prefix max of I - ge2*c
            A = np.maximum.accumulate(np.concatenate([[icand(r)], Mr[:-1] + go2 + ge2 - ge2 * k[1:]]))
            Ir = A + ge2 * k
            M[r], I[r], D[r] = Mr, Ir, Dr
            H = np.maximum(np.maximum(Mr, Ir), Dr)
        self.M, self.I, self.D = M, I, D
        hr = np.maximum(np.maximum(M[1:, -1], I[1:, -1]), D[1:, -1])
        ir = np.maximum(M[1:, -1] + go2, I[1:, -1]) + ge2
        self.out = (hr & 0xFFFFFFFF) | (ir << 32)

    def finish(self):
        if self.out is None:
            assert self.have == self.ld
            self.fill(self.inbox if self.lo > 0 else None)

    def close(self):
        pass

    def _c(self, j):
        return j - self.lo - 1

    def _v(self, X, i, j):
        return int(X[i, self._c(j)]) >> 1

    def _h(self, i, j):
        return max(self._v(self.M, i, j), self._v(self.I, i, j), self._v(self.D, i, j))

    def _argmax(self, i, j):  # walk codes (nw_common.hpp argmax_row0_walk; interior ties)
        if i == 0:
            return 1 if j == 0 else (4 if self.d_row0(j) >= SENT else 3)
        h = self._h(i, j)
        return ((self._v(self.M, i, j) == h) * 1 | (self._v(self.I, i, j) == h) * 2 |
                (self._v(self.D, i, j) == h) * 4)

    def score(self):
        h = max(int(self.M[-1, -1]), int(self.I[-1, -1]), int(self.D[-1, -1]))
        return h >> 1, 2 if h & 1 else 0

    def walk(self, entry):
        from sequencealigning_amd import span as S
        i, j, kind, _ = entry
        if kind >= S.SPAN_EXIT:
            return tuple(entry), np.zeros(0, np.uint32)
        es = 0
        st = lambda a: S.SPAN_D if a & 4 else (S.SPAN_I if a & 2 else S.SPAN_M)
        if kind == S.SPAN_END:
            es = self._argmax(i, j)
            cur = S.first_end_state(es)
        elif kind == S.SPAN_VIA_M:
            cur = st(self._argmax(i, j))
        elif kind == S.SPAN_VIA_I:
            cur = S.SPAN_M if self._v(self.M, i, j) + self.go >= self._v(self.I, i, j) else S.SPAN_I
        else:
            cur = kind
        runs = []

        def push(op):
            if runs and runs[-1][1] == op:
                runs[-1][0] += 1
            else:
                runs.append([1, op])

        def words():
            return np.array([(n << 4) | op for n, op in runs], np.uint32)
        lo = self.lo
        while True:
            if cur == S.SPAN_M:
                if i == 0 or j == 0:
                    ev = S.EV_ORIGIN if i == 0 and j == 0 else S.EV_DEAD
                    break
                push(7 if self.q[j - 1] == self.d[i - 1] else 8)
                if lo > 0 and j - 1 == lo:
                    return (i - 1, j - 1, S.SPAN_VIA_M, es), words()
                cur = st(self._argmax(i - 1, j - 1))
                i, j = i - 1, j - 1
            elif cur == S.SPAN_I:
                if i == 0 or j == 0:
                    ev = S.EV_PANIC if j == 0 and i >= 1 else S.EV_DEAD
                    break
                push(1)
                if lo > 0 and j - 1 == lo:
                    return (i, j - 1, S.SPAN_VIA_I, es), words()
                if j == 1:
                    op_ = SENT + self.go > self.i_col0(i)
                else:
                    op_ = self._v(self.M, i, j - 1) + self.go >= self._v(self.I, i, j - 1)
                cur = S.SPAN_M if op_ else S.SPAN_I
                j -= 1
            else:
                if i == 0 or j == 0:
                    ev = S.EV_PANIC if i == 0 and j >= 1 else S.EV_DEAD
                    break
                push(2)
                if i == 1:
                    op_ = SENT + self.go > self.d_row0(j)
                else:
                    op_ = self._v(self.M, i - 1, j) + self.go >= self._v(self.D, i - 1, j)
                cur = S.SPAN_M if op_ else S.SPAN_D
                i -= 1
        return (i, j, S.SPAN_EXIT + ev, es), words()


def _pairs():
    from nw_check import rand_seq
    rng = np.random.default_rng(31)
    out = []
    for lq, ld in [(700, 300), (600, 650), (1030, 120)]:
        q = rand_seq(rng, lq)
        d = bytearray(q[:ld]) if ld <= lq else bytearray(q)
        for k in range(0, len(d), 17):  # a few substitutions
            d[k] = ord("ACGT"[(d[k] + 1) % 4])
        out.append((q, bytes(d)))
    out.append((rand_seq(rng, 520), rand_seq(rng, 90)))   # iid: gaps at the ends, panics
    out.append((rand_seq(rng, 777), rand_seq(rng, 333)))
    return out


def _worker(rank, world, port, pairs, out):
    import torch.distributed as dist

    from sequencealigning_amd.span import ShardedLongPair
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = []
    for q, d in pairs:
        sp = ShardedLongPair(q, d, band_rows=64, engine=_CpuSpanEngine)
        r = sp.align()
        sp.close()
        if rank == 0:
            got.append((r.score, r.status, r.end_states, r.printed, r.cigar))
    if rank == 0:
        out.put(got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_long_pair_gloo(world):
    """ShardedLongPair at world 2 / 3 (gloo relay, CPU span engines): score,
    panic status, end states and the first printed alignment assembled on
    rank 0 equal the oracle's for mutated and iid pairs."""
    from oracle import refcpu

    from sequencealigning_amd.nw import cigar_ops_string
    pairs = _pairs()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pairs, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for (qs, ds), (score, status, es, printed, cig) in zip(pairs, got):
        o = refcpu.nw(qs, ds, literal_dfs=False)
        assert score == o.score
        assert (status == 2) == o.panics
        assert es == o.end_states
        assert printed == (o.first_ops is not None)
        if printed:
            assert cigar_ops_string(cig) == o.first_ops


def test_single_engine_matches_oracle():
    """The test engine itself, one span over the whole pair (no driver)."""
    from oracle import refcpu

    from sequencealigning_amd import span as S
    from sequencealigning_amd.nw import cigar_ops_string
    for qs, ds in _pairs():
        e = _CpuSpanEngine(qs, ds, 0, len(qs))
        e.fill(None)
        sc, st = e.score()
        ev, es, segs = S.walk_spans([e.walk], len(qs), len(ds))
        o = refcpu.nw(qs, ds, literal_dfs=False)
        assert sc == o.score and (st == 2) == o.panics and es == o.end_states
        assert (ev == S.EV_ORIGIN) == (o.first_ops is not None)
        if ev == S.EV_ORIGIN:
            assert cigar_ops_string(S.merge_walk_ops(segs)) == o.first_ops


def test_span_boundary_geometry(saln):
    """Host-only span geometry (no device): boundary columns = stripes + 1,
    64-column stripes (K = 1) while a span has at most 1,024 of them, else
    128-column ones; a caller-owned boundary buffer's size."""
    from sequencealigning_amd import _lib
    L = _lib.lib()
    assert L.saln_nw_span_boundary_cols(0, 12288, 0) == 12288 // 64 + 1
    # the same span sharing its GPU with the rest of a 100 kbp pair: 128-column stripes
    assert L.saln_nw_span_boundary_cols(0, 12288, 100_000) == 12288 // 128 + 1
    assert L.saln_nw_span_boundary_cols(0, 100_000, 0) == (100_000 + 127) // 128 + 1
    assert L.saln_nw_span_boundary_cols(256, 300, 0) == 2
    assert L.saln_nw_span_boundary_cols(512, 512, 0) == 0
    assert L.saln_nw_span_boundary_elems(100_001) % 4 == 0
    assert L.saln_nw_span_boundary_elems(100_001) >= 100_001 + 9  # rows 1..ld + the pad slots


def test_span_columns_and_merge():
    from sequencealigning_amd import span as S
    assert S.span_columns(100_000, 8)[0] == (0, 12288)
    cols = S.span_columns(100_000, 8)
    assert cols[-1][1] == 100_000 and all(a % 256 == 0 for a, _ in cols)
    assert all(cols[k][1] == cols[k + 1][0] for k in range(7))
    assert S.span_columns(257, 2) == [(0, 256), (256, 257)]
    with pytest.raises(ValueError):
        S.span_columns(256, 2)
    # walk order (back to front), runs merged at the seam, then reversed
    segs = [np.array([(3 << 4) | 7, (2 << 4) | 1], np.uint32),
            np.array([(1 << 4) | 1, (4 << 4) | 8], np.uint32)]
    assert S.merge_walk_ops(segs) == [(4, "X"), (3, "I"), (3, "=")]
    # dead-end order of the end states: D, M, I
    assert S.first_end_state(7) == S.SPAN_D and S.end_states_after(7, S.SPAN_D) == 3
    assert S.end_states_after(3, S.SPAN_M) == 2 and S.end_states_after(2, S.SPAN_I) == 0


class _Recorder:
    """Recording fake of the RCCL path: engine calls and dist.irecv / isend
    go into one log, in the order ShardedLongPair._fill_nccl issues them."""

    def __init__(self, log):
        self.log = log

    def reset(self):
        self.log.append(("reset",))

    def inbox_view(self, a, b):
        return ("inbox", a, b)

    def launch_fill(self):
        self.log.append(("fill",))

    def watch_outbox(self, a, b):
        self.log.append(("watch", a, b))
        return ("outbox", a, b)

    def side_stream(self):
        log = self.log

        class _Ctx:
            def __enter__(self):
                log.append(("side+",))

            def __exit__(self, *e):
                log.append(("side-",))
        return _Ctx()

    def finish(self):
        self.log.append(("finish",))


def test_nccl_band_pipeline_enqueue_order(monkeypatch):
    """ShardedLongPair's RCCL path at world 3 (each rank driven in turn with a
    recording engine and recording irecv / isend): every band's receive is
    posted before the fill, the fill before any watch, each send right after
    the watch of its band and inside the side stream, and the end rank posts
    no sends / the first no receives."""
    import torch.distributed as dist

    from sequencealigning_amd import span as S

    class _Work:
        def wait(self):
            pass
    world, ld, band = 3, 1000, 256
    bands = S._bands(ld, band)
    assert bands[0] == (1, 256) and bands[-1] == (769, 1000)
    for rank in range(world):
        log = []
        monkeypatch.setattr(dist, "irecv", lambda t, src, group: log.append(("irecv", t, src)) or _Work())
        monkeypatch.setattr(dist, "isend", lambda t, dst, group: log.append(("isend", t, dst)) or _Work())
        sp = object.__new__(S.ShardedLongPair)
        sp.world, sp.rank, sp.bands, sp.nccl = world, rank, bands, True
        sp.left = "L" if rank > 0 else None
        sp.right = "R" if rank + 1 < world else None
        sp.engine = _Recorder(log)
        sp._fill_nccl()
        kinds = [e[0] for e in log]
        assert kinds[0] == "reset" and kinds[-1] == "finish"
        fill = kinds.index("fill")
        recvs = [i for i, k in enumerate(kinds) if k == "irecv"]
        assert len(recvs) == (len(bands) if rank > 0 else 0)
        assert all(i < fill for i in recvs)
        assert [log[i][1] for i in recvs] == ([("inbox", a, b) for a, b in bands] if rank else [])
        assert all(log[i][2] == rank - 1 for i in recvs)
        sends = [i for i, k in enumerate(kinds) if k == "isend"]
        assert len(sends) == (len(bands) if rank + 1 < world else 0)
        for (a, b), i in zip(bands, sends):
            assert log[i - 1] == ("watch", a, b) and log[i][1] == ("outbox", a, b) and i > fill
            assert log[i][2] == rank + 1
        if sends:
            side_on, side_off = kinds.index("side+"), kinds.index("side-")
            assert side_on < sends[0] and sends[-1] < side_off and fill < side_on
