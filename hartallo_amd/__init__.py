"""hartallo_amd -- MI355X (gfx950) native H.264 Baseline encode path of
allweax/hartallo: the per-macroblock RDO loop (diamond ME, quarter-pel
interpolation, 4x4 transform/quant, CAVLC rate, intra RDO, deblocking) as
hand-written HIP kernels, and its spatial-SVC enhancement layers, bit-exact
with the reference encoder, behind a
C ABI (include/hartallo_amd.h) that a hartallo plugin forwards to.
"""
from ._lib import (EXPORTED_SYMBOLS, HL_AMD_RESULT_TYPE_DATA, HL_AMD_RESULT_TYPE_HDR, LIB_PATH, EncodeResult, Encoder,
                   HlAmdError, SvcEncoder, load_library)

__all__ = [
    "Encoder",
    "SvcEncoder",
    "EncodeResult",
    "HlAmdError",
    "load_library",
    "LIB_PATH",
    "EXPORTED_SYMBOLS",
    "HL_AMD_RESULT_TYPE_DATA",
    "HL_AMD_RESULT_TYPE_HDR",
]
