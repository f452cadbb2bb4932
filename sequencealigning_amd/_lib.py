"""ctypes binding of ``libsaln.so`` (the C ABI declared in ``include/saln.h``).

The library is built in-tree by ``__graft_entry__.build()``.  There is no
CPU fallback: if the shared object is missing, importing the compute entry
points raises, and creating a context without a gfx950 device fails with
``SALN_E_NO_DEVICE``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# SALN_LIB: an instrumented in-tree build (tools/) instead of libsaln.so;
# bench.py refuses to run with it set
LIB_PATH = os.environ.get("SALN_LIB") or os.path.join(_HERE, "libsaln.so")

# saln_status (include/saln.h)
OK = 0
NOT_IMPLEMENTED = 1
REF_PANIC_BOUNDARY = 2
REF_PANIC_TRIM = 3
REF_PANIC_SLICE = 4
NONCONVERGED = 5
ENUM_CAP = 6
SPAN_UNLINKED = 7
E_INVALID = -1
E_HIP = -2
E_NO_DEVICE = -3
E_CAPACITY = -4
E_IO = -5
E_FASTA = -6
E_FASTA_CHARS = -7
E_DEVICE_WAIT = -8
FLAG_WAIT_TIMEOUT = 1   # SALN_FLAG_WAIT_TIMEOUT
FLAG_SPEC_UNLINKED = 2  # SALN_FLAG_SPEC_UNLINKED

STATUS_NAMES = {
    OK: "OK", NOT_IMPLEMENTED: "NOT_IMPLEMENTED", REF_PANIC_BOUNDARY: "REF_PANIC_BOUNDARY",
    REF_PANIC_TRIM: "REF_PANIC_TRIM", REF_PANIC_SLICE: "REF_PANIC_SLICE",
    NONCONVERGED: "NONCONVERGED", ENUM_CAP: "ENUM_CAP", SPAN_UNLINKED: "SPAN_UNLINKED", E_INVALID: "E_INVALID", E_HIP: "E_HIP",
    E_NO_DEVICE: "E_NO_DEVICE", E_CAPACITY: "E_CAPACITY", E_IO: "E_IO", E_FASTA: "E_FASTA",
    E_FASTA_CHARS: "E_FASTA_CHARS", E_DEVICE_WAIT: "E_DEVICE_WAIT",
}

CIGAR_OPS = {7: "=", 8: "X", 1: "I", 2: "D"}


class NwScoring(C.Structure):
    _fields_ = [("match", C.c_int32), ("mismatch", C.c_int32), ("gap_open", C.c_int32),
                ("gap_extend", C.c_int32)]


class NwResult(C.Structure):
    _fields_ = [("score", C.c_int32), ("status", C.c_int32), ("cigar_len", C.c_uint32),
                ("end_states", C.c_uint8), ("printed", C.c_uint8), ("flags", C.c_uint8),
                ("reserved", C.c_uint8)]


class SpanCursor(C.Structure):
    """saln_nw_span_cursor: a span walk's entry / exit."""
    _fields_ = [("i", C.c_int32), ("j", C.c_int32), ("kind", C.c_int32),
                ("end_states", C.c_uint32)]


# numpy view of saln_nw_result
RESULT_DTYPE = [("score", "<i4"), ("status", "<i4"), ("cigar_len", "<u4"), ("end_states", "u1"),
                ("printed", "u1"), ("flags", "u1"), ("reserved", "u1")]

class WfaResult(C.Structure):
    _fields_ = [("score", C.c_int32), ("status", C.c_int32), ("steps", C.c_uint32),
                ("aln_len1", C.c_uint32), ("aln_len2", C.c_uint32), ("conv_offset", C.c_int32),
                ("conv_state", C.c_uint8), ("conv_np", C.c_uint8),
                ("conv_parents", C.c_uint8 * 3), ("reserved", C.c_uint8 * 3)]


WFA_RESULT_DTYPE = [("score", "<i4"), ("status", "<i4"), ("steps", "<u4"), ("aln_len1", "<u4"),
                    ("aln_len2", "<u4"), ("conv_offset", "<i4"), ("conv_state", "u1"),
                    ("conv_np", "u1"), ("conv_parents", "u1", (3,)), ("reserved", "u1", (3,))]

# symbols every build must export (tests check this list against include/saln.h)
EXPORTS = [
    "saln_context_create", "saln_context_destroy", "saln_last_error", "saln_abi_version",
    "saln_nw_align", "saln_nw_render", "saln_nw_dense_mask", "saln_nw_align_batch",
    "saln_nw_plan_create", "saln_nw_plan_create_full", "saln_nw_plan_dense_mask",
    "saln_nw_plan_walk_codes",
    "saln_nw_plan_info", "saln_nw_cigar_offsets", "saln_nw_execute",
    "saln_nw_plan_set_timing", "saln_nw_plan_kernel_time", "saln_nw_plan_set_async",
    "saln_nw_plan_set_score_only", "saln_nw_plan_sync", "saln_nw_plan_destroy",
    "saln_nw_plan_status", "saln_nw_plan_set_wait_limit",
    "saln_nw_avsa_create", "saln_nw_avsa_execute", "saln_nw_avsa_info", "saln_nw_avsa_destroy",
    "saln_nw_avsa_status", "saln_nw_avsa_launch_geometry",
    "saln_nw_span_boundary_elems", "saln_nw_span_boundary_cols", "saln_nw_span_create", "saln_nw_span_info",
    "saln_nw_span_boundary", "saln_nw_span_reset", "saln_nw_span_fill", "saln_nw_span_watch",
    "saln_nw_span_walk", "saln_nw_span_score", "saln_nw_span_status",
    "saln_nw_span_set_wait_limit", "saln_nw_span_destroy", "saln_nw_span_forward", "saln_nw_spans_walk",
    "saln_device_cu_count", "saln_stream_create_cu_range", "saln_stream_destroy",
    "saln_device_cu_probe", "saln_nw_plan_set_tb_stream", "saln_stream_create_cu_mask",
    "saln_wfa_align_batch", "saln_wfa_render", "saln_wfa_plan_create", "saln_wfa_execute",
    "saln_wfa_plan_destroy",
    "saln_wfa_affine_batch", "saln_wfa_affine_plan_create", "saln_wfa_affine_execute",
    "saln_wfa_affine_plan_destroy",
    "saln_parse_fasta", "saln_parse_fasta_buffer", "saln_records_count", "saln_records_get",
    "saln_records_free",
    "saln_option_set", "saln_option_get", "saln_option_name", "saln_options_reset",
    "saln_context_option_set", "saln_context_option_get", "saln_context_option_clear",
    "saln_nw_render_batch", "saln_nw_render_text", "saln_nw_text_count", "saln_nw_text_get",
    "saln_nw_text_gpu_decided",
    "saln_nw_text_free",
    "saln_wfa_render_batch", "saln_wfa_text_count", "saln_wfa_text_get", "saln_wfa_text_free",
]

_lib = None
_lock = threading.Lock()


class SalnError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        msg = last_error() if _lib is not None else ""
        super().__init__(f"{what}: {STATUS_NAMES.get(code, code)} {msg}".strip())


class WfaPenalties(C.Structure):
    """saln_wfa_penalties: corrected gap-affine WFA (x, o, e); wfa.rs:14-21 defaults."""
    _fields_ = [("mismatch", C.c_int32), ("gap_open", C.c_int32), ("gap_extend", C.c_int32)]


def lib() -> C.CDLL:
    """Load libsaln.so (raises if the in-tree build is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        # torch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7).  If
        # torch is importable, load it first so libsaln binds to that same
        # HIP runtime by soname; loading /opt/rocm's copy first would leave
        # two HIP runtimes in the process and torch would see no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (there is no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        u8p, u32p, u64p, i32p = (C.POINTER(C.c_uint8), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint64), C.POINTER(C.c_int32))
        vp = C.c_void_p
        L.saln_last_error.restype = C.c_char_p
        L.saln_context_create.argtypes = [C.c_int, C.POINTER(vp)]
        L.saln_context_destroy.argtypes = [vp]
        L.saln_nw_align.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_int, C.c_int32,
                                    C.POINTER(NwScoring), C.POINTER(NwResult), u32p, C.c_uint64]
        L.saln_nw_render.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_int32, C.c_uint64,
                                     C.c_char_p, C.c_uint64, u64p, u64p, i32p]
        L.saln_nw_dense_mask.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64,
                                         C.POINTER(NwScoring), vp]
        L.saln_nw_align_batch.argtypes = [vp, vp, vp, C.c_uint64, vp, vp, C.c_uint64, vp, vp,
                                          C.c_uint64, C.c_int32, C.POINTER(NwScoring), vp, vp,
                                          vp]
        L.saln_nw_plan_create.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp,
                                          C.c_uint64, C.c_int32, C.POINTER(NwScoring),
                                          C.POINTER(vp)]
        L.saln_nw_plan_create_full.argtypes = L.saln_nw_plan_create.argtypes
        L.saln_nw_plan_dense_mask.argtypes = [vp, C.c_uint64, vp]
        L.saln_nw_plan_walk_codes.argtypes = [vp, C.c_uint64, vp]
        L.saln_nw_plan_info.argtypes = [vp, u64p, u64p, u64p]
        L.saln_nw_cigar_offsets.argtypes = [vp, vp]
        L.saln_nw_execute.argtypes = [vp, vp, vp, vp, vp, vp]
        L.saln_nw_plan_set_timing.argtypes = [vp, C.c_int]
        L.saln_nw_plan_kernel_time.argtypes = [vp, C.c_char_p, C.POINTER(C.c_double), u64p]
        L.saln_nw_plan_set_async.argtypes = [vp, C.c_int]
        L.saln_nw_plan_sync.argtypes = [vp, vp, C.c_int]
        L.saln_nw_plan_set_score_only.argtypes = [vp, C.c_int]
        L.saln_nw_plan_destroy.argtypes = [vp]
        L.saln_nw_plan_status.argtypes = [vp, u32p]
        L.saln_nw_plan_set_wait_limit.argtypes = [vp, C.c_uint32]
        L.saln_nw_avsa_status.argtypes = [vp, u32p]
        L.saln_nw_avsa_launch_geometry.argtypes = [C.c_int, u64p, u64p]
        L.saln_nw_avsa_create.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_int32,
                                          C.POINTER(NwScoring), C.POINTER(vp)]
        L.saln_nw_avsa_execute.argtypes = [vp, vp, vp, vp, vp]
        L.saln_nw_avsa_info.argtypes = [vp, u64p, u64p]
        L.saln_nw_avsa_destroy.argtypes = [vp]
        L.saln_nw_span_boundary_elems.argtypes = [C.c_uint64]
        L.saln_nw_span_boundary_elems.restype = C.c_uint64
        L.saln_nw_span_boundary_cols.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.saln_nw_span_boundary_cols.restype = C.c_uint64
        L.saln_nw_span_create.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                          C.c_uint64, C.POINTER(NwScoring), vp, C.POINTER(vp)]
        L.saln_nw_span_info.argtypes = [vp, u64p, u64p, u64p]
        L.saln_nw_span_boundary.argtypes = [vp, C.POINTER(vp), C.POINTER(vp)]
        L.saln_nw_span_reset.argtypes = [vp, vp]
        L.saln_nw_span_fill.argtypes = [vp, vp, vp, vp]
        L.saln_nw_span_watch.argtypes = [vp, C.c_uint64, C.c_uint64, vp]
        L.saln_nw_span_walk.argtypes = [vp, vp, vp, C.POINTER(SpanCursor), C.POINTER(SpanCursor),
                                        u32p, C.c_uint64, u64p, vp]
        L.saln_nw_span_score.argtypes = [vp, i32p, i32p, vp]
        L.saln_nw_span_status.argtypes = [vp, u32p]
        L.saln_nw_span_set_wait_limit.argtypes = [vp, C.c_uint32]
        L.saln_nw_span_destroy.argtypes = [vp]
        L.saln_nw_span_forward.argtypes = [vp, vp, C.c_uint64, C.c_uint64, vp]
        L.saln_nw_spans_walk.argtypes = [C.POINTER(vp), C.c_uint32, vp, vp, C.POINTER(SpanCursor),
                                         u32p, C.c_uint64, u64p, vp]
        L.saln_device_cu_count.argtypes = [vp, u32p]
        L.saln_stream_create_cu_range.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(vp)]
        L.saln_stream_destroy.argtypes = [vp, vp]
        L.saln_device_cu_probe.argtypes = [vp, vp, C.c_uint32, u32p, u32p]
        L.saln_stream_create_cu_mask.argtypes = [vp, u32p, C.c_uint32, C.POINTER(vp)]
        L.saln_nw_plan_set_tb_stream.argtypes = [vp, vp]
        L.saln_wfa_plan_create.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp,
                                           C.c_uint64, C.c_int32, C.c_uint32, C.c_uint32,
                                           C.POINTER(vp)]
        L.saln_wfa_execute.argtypes = [vp, vp, vp, vp, vp]
        L.saln_wfa_plan_destroy.argtypes = [vp]
        L.saln_wfa_align_batch.argtypes = [vp, vp, vp, C.c_uint64, vp, vp, C.c_uint64, vp, vp,
                                           C.c_uint64, C.c_int32, C.c_uint32, C.c_uint32, vp,
                                           vp, vp, C.c_uint32]
        L.saln_wfa_render.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_int32, C.c_uint32,
                                      C.c_uint32, C.c_char_p, C.c_uint64, u64p,
                                      C.POINTER(WfaResult)]
        L.saln_wfa_affine_batch.argtypes = [vp, vp, vp, C.c_uint64, vp, vp, C.c_uint64, vp, vp,
                                            C.c_uint64, C.POINTER(WfaPenalties), C.c_int32, vp]
        L.saln_wfa_affine_plan_create.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp,
                                                  C.c_uint64, C.POINTER(WfaPenalties),
                                                  C.c_int32, C.POINTER(vp)]
        L.saln_wfa_affine_execute.argtypes = [vp, vp, vp, vp, vp]
        L.saln_wfa_affine_plan_destroy.argtypes = [vp]
        L.saln_parse_fasta.argtypes = [C.c_char_p, C.POINTER(vp), u8p, C.c_uint64, u64p]
        L.saln_parse_fasta_buffer.argtypes = [vp, C.c_uint64, C.POINTER(vp), u8p, C.c_uint64,
                                              u64p]
        L.saln_records_count.argtypes = [vp]
        L.saln_records_count.restype = C.c_uint64
        L.saln_records_get.argtypes = [vp, C.c_uint64, C.POINTER(vp), u64p, C.POINTER(vp), u64p]
        L.saln_records_free.argtypes = [vp]
        L.saln_records_free.restype = None
        L.saln_nw_render_batch.argtypes = [vp, vp, vp, C.c_uint64, vp, vp, C.c_uint64, vp, vp,
                                           C.c_uint64, C.c_int32, C.c_uint64, C.c_int,
                                           C.POINTER(vp)]
        L.saln_nw_render_text.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_int32,
                                          C.c_uint64, C.POINTER(vp)]
        L.saln_nw_text_count.argtypes = [vp]
        L.saln_nw_text_count.restype = C.c_uint64
        L.saln_nw_text_gpu_decided.argtypes = [vp]
        L.saln_nw_text_gpu_decided.restype = C.c_uint64
        L.saln_nw_text_get.argtypes = [vp, C.c_uint64, C.POINTER(vp), u64p, u64p, i32p,
                                       C.POINTER(NwResult), u64p]
        L.saln_nw_text_free.argtypes = [vp]
        L.saln_nw_text_free.restype = None
        L.saln_wfa_render_batch.argtypes = [vp, vp, vp, C.c_uint64, vp, vp, C.c_uint64, vp, vp,
                                            C.c_uint64, C.c_int32, C.c_uint32, C.c_uint32,
                                            C.POINTER(vp)]
        L.saln_wfa_text_count.argtypes = [vp]
        L.saln_wfa_text_count.restype = C.c_uint64
        L.saln_wfa_text_get.argtypes = [vp, C.c_uint64, C.POINTER(vp), u64p,
                                        C.POINTER(WfaResult)]
        L.saln_wfa_text_free.argtypes = [vp]
        L.saln_wfa_text_free.restype = None
        L.saln_option_set.argtypes = [C.c_char_p, C.c_int64]
        L.saln_option_get.argtypes = [C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.saln_option_name.argtypes = [C.c_uint32, C.POINTER(C.c_char_p)]
        L.saln_context_option_set.argtypes = [vp, C.c_char_p, C.c_int64]
        L.saln_context_option_get.argtypes = [vp, C.c_char_p, C.POINTER(C.c_int64)]
        L.saln_context_option_clear.argtypes = [vp, C.c_char_p]
        _lib = L
        return L


def last_error() -> str:
    msg = lib().saln_last_error()
    return msg.decode(errors="replace") if msg else ""


def check(rc: int, what: str, ok=(OK,)) -> int:
    if rc not in ok:
        raise SalnError(rc, what)
    return rc


_contexts: dict[int, C.c_void_p] = {}


def context(device: int = 0) -> C.c_void_p:
    """Per-process context for `device` (created on first use)."""
    with _lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = C.c_void_p()
            check(lib().saln_context_create(device, C.byref(ctx)), "saln_context_create")
            _contexts[device] = ctx
        return ctx


HIP_STREAM_LEGACY = 1  # hipStreamLegacy (hip_runtime_api.h): the legacy null stream


def torch_stream(device) -> int:
    """torch's current stream on `device` as a libsaln stream argument.  The
    C ABI reads NULL as "the context's own stream" (non-blocking, unordered
    with torch's default stream), so torch's null stream is passed as
    hipStreamLegacy: the kernels then run in order with torch's work."""
    import torch
    h = torch.cuda.current_stream(device).cuda_stream
    return h if h else HIP_STREAM_LEGACY


def scoring_arg(scoring) -> C.POINTER(NwScoring) | None:
    if scoring is None:
        return None
    if isinstance(scoring, NwScoring):
        return C.pointer(scoring)
    m, x, o, e = scoring
    return C.pointer(NwScoring(m, x, o, e))


# ------------------------------------------------------------------ options
def set_option(name: str, value: int) -> None:
    """saln_option_set: one of the engine's tuning knobs (include/saln.h)."""
    check(lib().saln_option_set(name.encode(), int(value)), f"saln_option_set({name})")


def get_option(name: str) -> tuple[int, int]:
    """(current value, default) of an option."""
    v, d = C.c_int64(), C.c_int64()
    check(lib().saln_option_get(name.encode(), C.byref(v), C.byref(d)), f"saln_option_get({name})")
    return v.value, d.value


def option_names() -> list[str]:
    out, i = [], 0
    while True:
        nm = C.c_char_p()
        if lib().saln_option_name(i, C.byref(nm)) != OK:
            return out
        out.append(nm.value.decode())
        i += 1


def non_default_options() -> dict[str, int]:
    """The options whose value differs from the default (bench.py records them)."""
    out = {}
    for nm in option_names():
        v, d = get_option(nm)
        if v != d:
            out[nm] = v
    return out


def set_context_option(ctx, name: str, value: int) -> None:
    """saln_context_option_set: an override of one context (include/saln.h)."""
    check(lib().saln_context_option_set(ctx, name.encode(), int(value)),
          f"saln_context_option_set({name})")


def get_context_option(ctx, name: str) -> int:
    """A context's effective value of an option."""
    v = C.c_int64()
    check(lib().saln_context_option_get(ctx, name.encode(), C.byref(v)),
          f"saln_context_option_get({name})")
    return v.value


def clear_context_option(ctx, name: str | None = None) -> None:
    """Drop one override of a context (name) or all of them (None)."""
    check(lib().saln_context_option_clear(ctx, name.encode() if name else None),
          "saln_context_option_clear")


def new_context(device: int = 0) -> C.c_void_p:
    """A context of its own (not the per-process one of context()); the
    caller destroys it with lib().saln_context_destroy."""
    ctx = C.c_void_p()
    check(lib().saln_context_create(device, C.byref(ctx)), "saln_context_create")
    return ctx


class options:
    """Context manager: set options for a block, restore the previous values.

        with options(**{"nw.pk_tab": 0}): ...
    """

    def __init__(self, **kw):
        self.kw = kw
        self.prev = {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.prev[k] = get_option(k)[0]
            set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.prev.items():
            set_option(k, v)
        return False
