"""sequencealigning_amd — MI355X-native drop-in engine for the NW-affine hot
and WFA paths of Qw11111111111/SequenceAligning (src/needleman_wunsch_affine.rs,
src/wfa.rs).

Compute lives in ``libsaln.so`` (HIP kernels for gfx950 behind the C ABI in
``include/saln.h``); this package is the host-side mirror of the reference's
interface: ``parse_fasta``/``Record``/``Mode`` (src/parse.rs), the
``AlignerError`` family (src/errors.rs), ``n_w_align`` and ``wfa_align``.
"""
from .records import (AlignerError, AlignmentError, Algo, CharError, FastaError, Mode, Record,
                      Records, parse_fasta, parse_fasta_bytes)
from .nw import (NwAlignment, NwAllVsAll, NwPlan, alignment_rows, cigar_ops_string, dense_mask, n_w_align,
                 nw_align_batch, nw_score_all_vs_all, pack_csr, render, render_batch)
from . import wfa
from .wfa import WfaAlignment, WfaPlan, wfa_align, wfa_align_batch
from . import wfa_affine
from ._lib import get_option, option_names, options, set_option

__all__ = [
    "AlignerError", "AlignmentError", "Algo", "CharError", "FastaError", "Mode", "Record",
    "Records", "parse_fasta", "parse_fasta_bytes", "NwAlignment", "NwPlan", "alignment_rows",
    "cigar_ops_string", "dense_mask", "n_w_align", "NwAllVsAll", "nw_score_all_vs_all", "nw_align_batch", "pack_csr", "render", "render_batch",
    "wfa", "WfaAlignment", "WfaPlan", "wfa_align", "wfa_align_batch", "wfa_affine",
    "get_option", "option_names", "options", "set_option",
]
