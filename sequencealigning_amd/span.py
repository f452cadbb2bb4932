"""One long pair split by query columns over GPUs.

The reference fills one pair row by row, query inner
(src/needleman_wunsch_affine.rs:217-236), and walks it back from the end cell
(:242-334).  Here span r of R owns the query columns ``span_columns(len_q,
R)[r]`` and runs the row fill's column stripes over every db row on its own
GPU (``saln_nw_span_*``, include/saln.h), keeping only its part of the
1 B/cell parent mask: a pair whose mask exceeds one GPU's HBM spreads over the
GPUs of a node.  The boundary leaving span r's last column (one 8-byte
element per db row) travels to span r+1 in row bands while both fill:

* ``nccl`` (one process per GPU, RCCL over xGMI): span r+1 posts every band's
  ``irecv`` into its inbox, then launches its fill, which polls the inbox row
  by row; span r queues, per band, a watch kernel (returns once the band's
  outbox rows are published) and an ``isend`` behind it on a side stream.
  Every kernel is queued after the work it waits for (receives before the
  fill, the fill before its watches), so a stream sharing a hardware queue
  can only serialise the pipeline, never deadlock it.
* ``relay`` (gloo, host tensors): bands go through host memory and a span's
  fill starts once its whole inbox has arrived (a sequential chain; tests and
  gloo-only setups).
* ``SpanChain`` (one process, one GPU): the spans of a pair on one device,
  chained by device copies behind watch kernels (tests; pairs of any width).

The traceback runs right to left: the span holding the end cell walks from it
until the walk leaves its first column, its exit is the next span's entry;
the span where the walk ends reports the event (origin / panic / dead end;
a dead end restarts from the next tied end state, like the reference's DFS,
:251-280).  Run words are concatenated in walk order, runs of one op merged
at the seams, and reversed into the CIGAR.

Critical path: the row chain of every column is unchanged, so
R spans take about one span's fill time (the rows x row step) plus R - 1 band
hand-offs; what scales with R is the mask memory per GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .nw import NwAlignment, _decode_cigar

SPAN_M, SPAN_I, SPAN_D, SPAN_VIA_M, SPAN_VIA_I, SPAN_END, SPAN_EXIT = 0, 1, 2, 3, 4, 5, 8
EV_ORIGIN, EV_PANIC, EV_DEAD = 0, 1, 2
ARG_M, ARG_I, ARG_D = 1, 2, 4
COL_EMPTY = 0x80000000  # an unpublished boundary row (low word)


def span_columns(len_q: int, n: int) -> list[tuple[int, int]]:
    """[(col_lo, col_hi)] of n spans: 256-column tiles split as evenly as
    possible, every span at least one tile (col_lo a multiple of 256)."""
    tiles = (len_q + 255) // 256
    if n < 1 or tiles < n:
        raise ValueError(f"{len_q} query columns give {tiles} 256-column tiles: at most that "
                         f"many spans")
    cuts = [256 * ((tiles * r) // n) for r in range(n)] + [len_q]
    return [(cuts[r], cuts[r + 1]) for r in range(n)]


def first_end_state(es: int) -> int:
    """End states in the reference DFS's pop order D, M, I (:251-280)."""
    return SPAN_D if es & ARG_D else (SPAN_M if es & ARG_M else SPAN_I)


def end_states_after(es: int, st: int) -> int:
    return es & (ARG_M | ARG_I) if st == SPAN_D else (es & ARG_I if st == SPAN_M else 0)


def merge_walk_ops(segments) -> list[tuple[int, str]]:
    """CIGAR (forward) from the spans' run words in walk order (each segment
    back to front, segments from the end cell's span leftwards): runs of one
    op continuing across a seam are merged, then the order is reversed."""
    w = np.concatenate([np.asarray(x, np.uint32).ravel() for x in segments] or
                       [np.zeros(0, np.uint32)])
    n, op = (w >> 4).astype(np.int64), w & 15
    keep = n > 0
    n, op = n[keep], op[keep]
    if not len(n):
        return []
    starts = np.flatnonzero(np.r_[True, op[1:] != op[:-1]])
    lens = np.add.reduceat(n, starts)[::-1]
    ops = op[starts][::-1]
    return [(int(a), _lib.CIGAR_OPS[int(b)]) for a, b in zip(lens.tolist(), ops.tolist())]


def walk_spans(walkers, len_q: int, len_db: int):
    """The right-to-left walk over spans (walkers[r](entry) -> (exit, ops)
    for span r, cursors as (i, j, kind, end_states) tuples).  Returns
    (event, end_states, per-span op segments of the printed walk)."""
    R = len(walkers)
    entry = (len_db, len_q, SPAN_END, 0)
    es_all, es_left, first = 0, 0, True
    while True:
        segs = [None] * R
        cur = entry
        for r in range(R - 1, -1, -1):
            cur, ops = walkers[r](cur)
            segs[r] = ops
            if r == R - 1 and first:
                es_all = cur[3]
                es_left = end_states_after(es_all, first_end_state(es_all))
        first = False
        ev = cur[2] - SPAN_EXIT
        if cur[2] < SPAN_EXIT or ev not in (EV_ORIGIN, EV_PANIC, EV_DEAD):
            raise RuntimeError(f"span walk did not end at column 0: exit {cur}")
        if ev != EV_DEAD or not es_left:
            return ev, es_all, segs[::-1]
        st = first_end_state(es_left)
        es_left = end_states_after(es_left, st)
        entry = (len_db, len_q, st, 0)


class CigarWords:
    """A CIGAR as the library's words ((len << 4) | op, forward order), read as
    the list of (len, op) tuples NwAlignment.cigar holds, decoded on first
    use: a 100 kbp pair has ~10^4 runs, and building their tuples costs more
    than the device walk."""

    def __init__(self, words):
        self.words = np.asarray(words, np.uint32)
        self._list = None

    def _decoded(self):
        if self._list is None:
            self._list = [(int(w) >> 4, _lib.CIGAR_OPS[int(w) & 15]) for w in self.words.tolist()]
        return self._list

    def __iter__(self):
        return iter(self._decoded())

    def __len__(self):
        return len(self.words)

    def __getitem__(self, k):
        return self._decoded()[k]

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self):
        return f"CigarWords({len(self.words)} runs)"


def result_from_walk(score: int, status: int, ev: int, es: int, segs) -> NwAlignment:
    """NwAlignment like saln_nw_align's (make_result, nw_kernels.hip): the
    CIGAR only when the walk printed (ended at the origin)."""
    cig = merge_walk_ops(segs) if ev == EV_ORIGIN else []
    return NwAlignment(int(score), int(status), int(es), ev == EV_ORIGIN, cig)


class NwSpan:
    """One span on one device (saln_nw_span_*).  The boundary columns are a
    torch int64 tensor (``boundary``; ``inbox`` / ``outbox`` are views of
    it, element r = db row r), so torch.distributed can send and receive
    rows of them."""

    def __init__(self, len_q: int, len_db: int, col_lo: int, col_hi: int, *, scoring=None,
                 device: int = 0, device_cols: int = 0):
        import torch
        L = _lib.lib()
        self.len_q, self.len_db, self.col_lo, self.col_hi = len_q, len_db, col_lo, col_hi
        self.device = device
        self.dev = torch.device("cuda", device)
        self.ctx = _lib.context(device)
        self.scol = int(L.saln_nw_span_boundary_elems(len_db))
        # device_cols: the columns of every span filling on this device at
        # once (SpanChain: the whole pair), which sets the stripe width
        self.ncol = int(L.saln_nw_span_boundary_cols(col_lo, col_hi, device_cols))
        self.boundary = torch.empty(self.ncol * self.scol, dtype=torch.int64, device=self.dev)
        self._h = C.c_void_p()
        _lib.check(L.saln_nw_span_create(self.ctx, len_q, len_db, col_lo, col_hi, device_cols,
                                         _lib.scoring_arg(scoring),
                                         C.c_void_p(self.boundary.data_ptr()), C.byref(self._h)),
                   "saln_nw_span_create")
        mb, cap = C.c_uint64(), C.c_uint64()
        L.saln_nw_span_info(self._h, C.byref(mb), None, C.byref(cap))
        self.mask_bytes, self.ops_cap = mb.value, cap.value
        self.inbox = self.boundary[:self.scol]
        self.outbox = self.boundary[(self.ncol - 1) * self.scol:]
        self._ops = (C.c_uint32 * max(1, self.ops_cap))()

    def _s(self, stream):
        import torch
        if stream is None:
            return _lib.torch_stream(self.device)
        if isinstance(stream, torch.cuda.Stream):
            # torch's null stream is handle 0, which the C ABI reads as "the
            # context's own stream": pass it as hipStreamLegacy (_lib.torch_stream)
            return stream.cuda_stream or _lib.HIP_STREAM_LEGACY
        return stream

    def reset(self, stream=None) -> None:
        _lib.check(_lib.lib().saln_nw_span_reset(self._h, self._s(stream)), "saln_nw_span_reset")

    def fill(self, q, d, stream=None) -> None:
        _lib.check(_lib.lib().saln_nw_span_fill(self._h, C.c_void_p(q.data_ptr()),
                                                C.c_void_p(d.data_ptr()), self._s(stream)),
                   "saln_nw_span_fill")

    def watch(self, row_lo: int, row_hi: int, stream=None) -> None:
        _lib.check(_lib.lib().saln_nw_span_watch(self._h, row_lo, row_hi, self._s(stream)),
                   "saln_nw_span_watch")

    def walk(self, q, d, entry, stream=None):
        """(exit cursor tuple, run words in walk order) from entry (i, j, kind, es)."""
        e_in = _lib.SpanCursor(*[int(x) for x in entry])
        e_out = _lib.SpanCursor()
        n = C.c_uint64()
        _lib.check(_lib.lib().saln_nw_span_walk(self._h, C.c_void_p(q.data_ptr()),
                                                C.c_void_p(d.data_ptr()), C.byref(e_in),
                                                C.byref(e_out), self._ops, self.ops_cap,
                                                C.byref(n), self._s(stream)),
                   "saln_nw_span_walk")
        ops = np.ctypeslib.as_array(self._ops)[:n.value].copy()
        return (e_out.i, e_out.j, e_out.kind, e_out.end_states), ops

    def score(self, stream=None) -> tuple[int, int]:
        sc, st = C.c_int32(), C.c_int32()
        _lib.check(_lib.lib().saln_nw_span_score(self._h, C.byref(sc), C.byref(st),
                                                 self._s(stream)), "saln_nw_span_score")
        return sc.value, st.value

    def status(self) -> int:
        """Device flags since the last call (waits for the device); read and clear."""
        f = C.c_uint32()
        rc = _lib.lib().saln_nw_span_status(self._h, C.byref(f))
        if rc not in (_lib.OK, _lib.E_DEVICE_WAIT):
            _lib.check(rc, "saln_nw_span_status")
        return f.value

    def check(self) -> None:
        if self.status():
            raise _lib.SalnError(_lib.E_DEVICE_WAIT, "span fill: a boundary wait timed out")

    def set_wait_limit(self, polls: int) -> None:
        _lib.check(_lib.lib().saln_nw_span_set_wait_limit(self._h, polls),
                   "saln_nw_span_set_wait_limit")

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().saln_nw_span_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _bands(len_db: int, band_rows: int) -> list[tuple[int, int]]:
    return [(r, min(len_db, r + band_rows - 1)) for r in range(1, len_db + 1, band_rows)]


class SpanChain:
    """All spans of one pair on one device in one process: the spans' fills
    run concurrently, each on its own stream, the outbox -> inbox hand-off of
    every band a device copy behind a watch kernel on the edge's stream
    (queued fill 0, hand-offs 0 -> 1, fill 1, ...: each kernel after the work
    it waits for).  ``cu_split`` (default) gives span r its own slice of the
    device's CUs (a CU-masked stream: its own hardware queue, its stripes on
    its own SIMDs), the single-GPU emulation of one span per GPU; otherwise
    the spans' kernels share the device's queues and CUs.
    ``pipelined=False`` runs the spans one after another on one stream (every
    inbox complete before its fill starts)."""

    def __init__(self, q: bytes, d: bytes, n_spans: int, *, scoring=None, device: int = 0,
                 band_rows: int = 2048, cu_split: bool = True, edge_masks: str = "shared",
                 cu_ranges=None):
        import torch
        self.q_bytes, self.d_bytes = bytes(q), bytes(d)
        self.len_q, self.len_db = len(q), len(d)
        self.device = device
        dev = torch.device("cuda", device)
        self.q = torch.frombuffer(bytearray(self.q_bytes), dtype=torch.uint8).to(dev)
        self.d = torch.frombuffer(bytearray(self.d_bytes), dtype=torch.uint8).to(dev)
        self.cols = span_columns(self.len_q, n_spans)
        # all spans fill on this one device at once: stripe widths for the
        # whole pair's columns
        self.spans = [NwSpan(self.len_q, self.len_db, lo, hi, scoring=scoring, device=device,
                             device_cols=self.len_q) for lo, hi in self.cols]
        self.bands = _bands(self.len_db, band_rows)
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(2 * n_spans)]
        self.cu_streams, self.edge_streams = [], []
        if cu_split:
            # span r's fills on CUs [r n / R, (r+1) n / R); the hand-offs of each
            # edge on a stream of its own (all CUs).  CU-masked streams are not
            # shared with other streams' hardware queues: no edge's forwards
            # queue behind another edge's, or behind a fill
            L, ctx = _lib.lib(), _lib.context(device)
            n = C.c_uint32()
            _lib.check(L.saln_device_cu_count(ctx, C.byref(n)), "saln_device_cu_count")
            if n.value >= n_spans:
                # cu_ranges (experiments): span r's mask bits, default an equal
                # contiguous share (bit c is a CU of XCD c mod 8: balanced)
                for lo, hi in cu_ranges or [(n.value * r // n_spans, n.value * (r + 1) // n_spans)
                                            for r in range(n_spans)]:
                    h = C.c_void_p()
                    _lib.check(L.saln_stream_create_cu_range(ctx, lo, hi, C.byref(h)),
                               "saln_stream_create_cu_range")
                    self.cu_streams.append(h)
                # edge r: every CU ("shared": one mask for all edges), every CU
                # but bit n-1-r ("unique": no two edge streams with equal
                # masks), or the last 8 bits ("reserved", experiments: give the
                # spans cu_ranges below them)
                nw = (n.value + 31) // 32
                for r in range(n_spans - 1):
                    words = [0xFFFFFFFF] * nw
                    if n.value % 32:
                        words[-1] = (1 << (n.value % 32)) - 1
                    if edge_masks == "unique":
                        b = n.value - 1 - r
                        words[b // 32] &= ~(1 << (b % 32)) & 0xFFFFFFFF
                    elif edge_masks == "reserved":  # the last octet (one CU per XCD)
                        words = [0] * nw
                        for b in range(n.value - 8, n.value):
                            words[b // 32] |= 1 << (b % 32)
                    arr = (C.c_uint32 * nw)(*words)
                    h = C.c_void_p()
                    _lib.check(L.saln_stream_create_cu_mask(ctx, arr, nw, C.byref(h)),
                               "saln_stream_create_cu_mask")
                    self.edge_streams.append(h)

    def fill(self, pipelined: bool = True) -> None:
        import torch
        main = torch.cuda.current_stream(self.device)
        for s in self.spans:
            s.reset(main)
        if pipelined and self.cu_streams:
            L = _lib.lib()
            torch.cuda.synchronize(self.device)  # the resets precede every watch
            for r, s in enumerate(self.spans):
                s.fill(self.q, self.d, self.cu_streams[r].value)
                if r + 1 < len(self.spans):  # one relay of every row per edge
                    _lib.check(L.saln_nw_span_forward(s._h, self.spans[r + 1]._h, 1, self.len_db,
                                                      self.edge_streams[r].value),
                               "saln_nw_span_forward")
            torch.cuda.synchronize(self.device)
            return
        if not pipelined:
            for r, s in enumerate(self.spans):
                if r:
                    s.inbox.copy_(self.spans[r - 1].outbox)
                s.fill(self.q, self.d, main)
            return
        ev = torch.cuda.Event()
        ev.record(main)
        fs, xs = self.streams[0::2], self.streams[1::2]
        for r, s in enumerate(self.spans):
            fs[r].wait_event(ev)
            s.fill(self.q, self.d, fs[r])
            if r + 1 < len(self.spans):
                nxt = self.spans[r + 1]
                xs[r].wait_event(ev)
                with torch.cuda.stream(xs[r]):
                    for a, b in self.bands:
                        s.watch(a, b, xs[r])
                        nxt.inbox[a:b + 1].copy_(s.outbox[a:b + 1])
        for st in self.streams:
            main.wait_stream(st)

    def check(self) -> None:
        for s in self.spans:
            s.check()

    def walk(self) -> NwAlignment:
        import torch
        torch.cuda.synchronize(self.device)
        self.check()
        score, status = self.spans[-1].score()
        # every span's speculative passes at once over one record table
        # (saln_nw_spans_walk); span by span when they do not link
        L = _lib.lib()
        hs = (C.c_void_p * len(self.spans))(*[s._h.value for s in self.spans])
        cap = self.len_q + self.len_db + 16
        buf = (C.c_uint32 * cap)()
        ex, n = _lib.SpanCursor(), C.c_uint64()
        rc = L.saln_nw_spans_walk(hs, len(self.spans), C.c_void_p(self.q.data_ptr()),
                                  C.c_void_p(self.d.data_ptr()), C.byref(ex), buf, cap,
                                  C.byref(n), _lib.torch_stream(self.device))
        if rc == _lib.OK:  # the CIGAR, merged at the seams in the library
            ev = ex.kind - SPAN_EXIT
            words = np.ctypeslib.as_array(buf)[:n.value].copy()
            return NwAlignment(int(score), int(status), int(ex.end_states), ev == EV_ORIGIN,
                               CigarWords(words if ev == EV_ORIGIN else words[:0]))
        if rc != _lib.SPAN_UNLINKED:
            _lib.check(rc, "saln_nw_spans_walk")
        walkers = [lambda e, s=s: s.walk(self.q, self.d, e) for s in self.spans]
        ev, es, segs = walk_spans(walkers, self.len_q, self.len_db)
        return result_from_walk(score, status, ev, es, segs)

    def align(self, pipelined: bool = True) -> NwAlignment:
        self.fill(pipelined)
        return self.walk()

    def close(self) -> None:
        for s in self.spans:
            s.close()
        if self.cu_streams:
            import torch
            torch.cuda.synchronize(self.device)
            L, ctx = _lib.lib(), _lib.context(self.device)
            for h in self.cu_streams + self.edge_streams:
                L.saln_stream_destroy(ctx, h)
            self.cu_streams, self.edge_streams = [], []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def nw_align_long_spans(q: bytes, d: bytes, n_spans: int, *, scoring=None, device: int = 0,
                        band_rows: int = 2048, pipelined: bool = True,
                        cu_split: bool = True) -> NwAlignment:
    """n_w_align of one pair (needleman_wunsch_affine.rs:424) through n_spans
    column spans on one device (SpanChain)."""
    ch = SpanChain(q, d, n_spans, scoring=scoring, device=device, band_rows=band_rows,
                   cu_split=cu_split)
    try:
        return ch.align(pipelined)
    finally:
        ch.close()


class _DeviceSpanEngine:
    """ShardedLongPair's per-rank engine on this rank's GPU.  Three streams of
    its own: the fill, the inbox copies of the band relay, and the watches
    with what reads the outbox behind them (sends, D2H copies)."""

    def __init__(self, q: bytes, d: bytes, col_lo: int, col_hi: int, scoring, device: int):
        import torch
        dev = torch.device("cuda", device)
        self.device = device
        self.q = torch.frombuffer(bytearray(q), dtype=torch.uint8).to(dev)
        self.d = torch.frombuffer(bytearray(d), dtype=torch.uint8).to(dev)
        self.span = NwSpan(len(q), len(d), col_lo, col_hi, scoring=scoring, device=device)
        self.side = torch.cuda.Stream(device=dev)
        self.fill_s = torch.cuda.Stream(device=dev)
        self.in_s = torch.cuda.Stream(device=dev)

    def reset(self) -> None:
        """Presets the boundary columns; every later stream of the pair
        (fill, inbox copies, watches) is ordered after it."""
        import torch
        self.span.reset(self.fill_s)
        ev = torch.cuda.Event()
        ev.record(self.fill_s)
        self.side.wait_event(ev)
        self.in_s.wait_event(ev)
        # RCCL receives into the inbox are ordered after the current stream
        torch.cuda.current_stream(self.device).wait_event(ev)

    def launch_fill(self) -> None:
        self.span.fill(self.q, self.d, self.fill_s)

    # band relay (gloo): the fill starts first and polls its inbox row by row
    def start_fill(self) -> None:
        self.reset()
        self.launch_fill()

    def put_inbox(self, a: int, b: int, rows: np.ndarray) -> None:
        """Inbox rows a .. b from host memory (H2D on the inbox stream, beside
        the running fill).  The fill was queued first and polls these rows, so
        the copy must not wait behind it: a pinned-host H2D copy runs on a DMA
        engine (SDMA), not on a compute queue, so it cannot queue behind the
        running kernel whatever hardware queue the two streams share.  Should
        it ever be served by a blit kernel stuck behind the fill, the fill's
        bounded polls end it with the span's wait-timeout flag, which finish()
        turns into an error (span.check) - never a hang or a silent result."""
        import torch
        src = torch.from_numpy(np.ascontiguousarray(rows, np.int64)).pin_memory()
        with torch.cuda.stream(self.in_s):
            self.span.inbox[a:b + 1].copy_(src, non_blocking=True)
        self.in_s.synchronize()  # `src` lives until the copy is done

    def outbox_rows(self, a: int, b: int) -> np.ndarray:
        """Outbox rows a .. b once the fill has published them (watch, then D2H)."""
        import torch
        with torch.cuda.stream(self.side):
            self.span.watch(a, b, self.side)
            out = self.span.outbox[a:b + 1].to("cpu", non_blocking=False)
        return out.numpy()

    # RCCL transport: views and the side stream the sends are queued on
    def inbox_view(self, a: int, b: int):
        return self.span.inbox[a:b + 1]

    def watch_outbox(self, a: int, b: int):
        """Queues the watch of rows a .. b on the side stream; returns their
        outbox view (for a send queued after it, inside side_stream())."""
        self.span.watch(a, b, self.side)
        return self.span.outbox[a:b + 1]

    def side_stream(self):
        import torch
        return torch.cuda.stream(self.side)

    def finish(self) -> None:
        import torch
        torch.cuda.synchronize(self.device)
        self.span.check()

    def walk(self, entry):
        return self.span.walk(self.q, self.d, entry)

    def score(self) -> tuple[int, int]:
        return self.span.score()

    def close(self) -> None:
        self.span.close()


_EDGES: dict = {}


def _edge_groups(world: int):
    import torch.distributed as dist
    key = (id(dist.group.WORLD), world)
    if key not in _EDGES:
        _EDGES[key] = [dist.new_group([e, e + 1]) for e in range(world - 1)]
    return _EDGES[key]


class ShardedLongPair:
    """One pair split by query columns over the ranks of the default process
    group (one process per GPU).  Rank r fills span r;
    boundary rows move rank r -> r+1 in bands of ``band_rows`` rows (nccl:
    RCCL send/recv on per-edge two-rank groups, pipelined with the fills;
    gloo: the host relay), then the walk crosses the ranks right to left (a
    16-byte cursor per hop) and rank 0 gathers the run words.  ``align()``
    returns the NwAlignment on rank 0 (score, status, end states, printed,
    CIGAR: saln_nw_align's for the same pair) and None elsewhere.

    ``engine`` (tests) replaces the device span: engine(q, d, col_lo, col_hi)
    with ``start_fill()``, ``put_inbox(a, b, rows)``, ``outbox_rows(a, b)``
    (int64 rows a..b), ``finish()``, ``walk(entry) -> (exit, ops)``,
    ``score()`` and ``close()``; it runs on the band relay (gloo).  The RCCL
    path drives the engine through ``reset()``, ``inbox_view(a, b)``,
    ``launch_fill()``, ``watch_outbox(a, b)``, ``side_stream()`` and
    ``finish()`` (``nccl=True`` with an engine: tests of its enqueue order).

    Both transports move the boundary in bands of ``band_rows`` rows while the
    fills run: rank r receives band k, then sends its own band k, so a band
    only waits for the bands before it (no cycle between the ranks)."""

    def __init__(self, q: bytes, d: bytes, *, scoring=None, device: int | None = None,
                 band_rows: int = 4096, engine=None, nccl: bool | None = None):
        import torch
        import torch.distributed as dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.len_q, self.len_db = len(q), len(d)
        self.cols = span_columns(self.len_q, self.world)
        self.bands = _bands(self.len_db, band_rows)
        lo, hi = self.cols[self.rank]
        backend = dist.get_backend()
        self.nccl = (engine is None and backend == "nccl") if nccl is None else nccl
        if engine is None:
            dev = torch.cuda.current_device() if device is None else device
            self.engine = _DeviceSpanEngine(q, d, lo, hi, scoring, dev)
            self.tdev = torch.device("cuda", dev) if self.nccl else torch.device("cpu")
        else:
            self.engine = engine(q, d, lo, hi)
            self.tdev = torch.device("cpu")
        # one two-rank group per edge (r, r+1): sends to the right and
        # receives from the left run on different communicators / streams
        # (created once per process group: every rank builds them in the same
        # order, and later pairs reuse them)
        self.edges = _edge_groups(self.world)
        self.left = self.edges[self.rank - 1] if self.rank > 0 else None
        self.right = self.edges[self.rank] if self.rank + 1 < self.world else None

    def _fill_nccl(self) -> None:
        """RCCL: every band's receive is posted first (queued behind the reset
        only), then the fill that polls them, then per band a watch and the
        send queued behind it on the side stream.  Each kernel is queued after
        the work it waits for, so streams sharing a hardware queue can only
        serialise the pipeline, never deadlock it."""
        import torch.distributed as dist
        eng = self.engine
        eng.reset()
        works = []
        if self.left is not None:
            for a, b in self.bands:
                works.append(dist.irecv(eng.inbox_view(a, b), src=self.rank - 1, group=self.left))
        eng.launch_fill()
        if self.right is not None:
            with eng.side_stream():
                for a, b in self.bands:
                    buf = eng.watch_outbox(a, b)
                    works.append(dist.isend(buf, dst=self.rank + 1, group=self.right))
        for w in works:
            w.wait()
        eng.finish()

    def _fill_relay(self) -> None:
        """gloo: the same band pipeline through host memory.  The fill starts
        at once and polls its inbox; per band, receive it from the left and
        copy it in (H2D), then wait for the own outbox band (watch), copy it
        out (D2H) and send it to the right."""
        import torch
        import torch.distributed as dist
        eng = self.engine
        eng.start_fill()
        for a, b in self.bands:
            if self.left is not None:
                t = torch.empty(b - a + 1, dtype=torch.int64)
                dist.recv(t, src=self.rank - 1, group=self.left)
                eng.put_inbox(a, b, t.numpy())
            if self.right is not None:
                t = torch.from_numpy(np.ascontiguousarray(eng.outbox_rows(a, b), np.int64))
                dist.send(t, dst=self.rank + 1, group=self.right)
        eng.finish()  # raises if a boundary wait timed out (SALN_FLAG_WAIT_TIMEOUT)

    def fill(self) -> None:
        if self.nccl:
            self._fill_nccl()
        else:
            self._fill_relay()

    def walk(self) -> NwAlignment | None:
        """The right-to-left walk over the ranks; the result on rank 0."""
        import torch
        import torch.distributed as dist

        from .dist import gather_records
        R, r = self.world, self.rank
        cur = torch.zeros(4, dtype=torch.int64, device=self.tdev)
        score = torch.zeros(2, dtype=torch.int64, device=self.tdev)
        if r == R - 1:
            sc, st = self.engine.score()
            score[0], score[1] = sc, st
        dist.broadcast(score, src=R - 1)
        entry = (self.len_db, self.len_q, SPAN_END, 0)
        es_all = es_left = 0
        first = True
        while True:
            if r < R - 1:
                dist.recv(cur, src=r + 1, group=self.right)
                entry = tuple(int(x) for x in cur.tolist())
            ex, ops = self.engine.walk(entry)
            if r == R - 1 and first:
                es_all = ex[3]
                es_left = end_states_after(es_all, first_end_state(es_all))
            if r > 0:
                cur = torch.tensor(list(ex), dtype=torch.int64, device=self.tdev)
                dist.send(cur, dst=r - 1, group=self.left)
            # rank 0 knows the event, the end cell's rank the next end state
            ctl = torch.tensor([ex[2] - SPAN_EXIT if r == 0 else 0, es_left, es_all],
                               dtype=torch.int64, device=self.tdev)
            ev_t = ctl.clone()
            dist.broadcast(ev_t, src=0)
            es_t = ctl.clone()
            dist.broadcast(es_t, src=R - 1)
            ev = int(ev_t[0])
            es_left, es_all = int(es_t[1]), int(es_t[2])
            first = False
            if ev != EV_DEAD or not es_left:
                break
            st = first_end_state(es_left)
            es_left = end_states_after(es_left, st)
            entry = (self.len_db, self.len_q, st, 0)
        words = gather_records(torch.from_numpy(np.asarray(ops, np.int64)).to(self.tdev))
        lens = gather_records(torch.tensor([len(ops)], dtype=torch.int64, device=self.tdev))
        if r != 0:
            return None
        w = words.cpu().numpy()
        n = lens.cpu().numpy()
        segs, pos = [], 0
        for k in range(R):
            segs.append(w[pos:pos + int(n[k])].astype(np.uint32))
            pos += int(n[k])
        return result_from_walk(int(score[0]), int(score[1]), ev, es_all, segs[::-1])

    def align(self) -> NwAlignment | None:
        self.fill()
        return self.walk()

    def close(self) -> None:
        self.engine.close()
