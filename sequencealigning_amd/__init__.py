"""sequencealigning_amd — MI355X-native drop-in engine for the NW-affine hot
path of Qw11111111111/SequenceAligning (src/needleman_wunsch_affine.rs).

Compute lives in ``libsaln.so`` (HIP kernels for gfx950 behind the C ABI in
``include/saln.h``); this package is the host-side mirror of the reference's
interface: ``parse_fasta``/``Record``/``Mode`` (src/parse.rs), the
``AlignerError`` family (src/errors.rs) and ``n_w_align``.
"""
from .records import (AlignerError, AlignmentError, Algo, CharError, FastaError, Mode, Record,
                      Records, parse_fasta, parse_fasta_bytes)
from .nw import (NwAlignment, NwPlan, alignment_rows, cigar_ops_string, dense_mask, n_w_align,
                 nw_align_batch, pack_csr, render)

__all__ = [
    "AlignerError", "AlignmentError", "Algo", "CharError", "FastaError", "Mode", "Record",
    "Records", "parse_fasta", "parse_fasta_bytes", "NwAlignment", "NwPlan", "alignment_rows",
    "cigar_ops_string", "dense_mask", "n_w_align", "nw_align_batch", "pack_csr", "render",
]
