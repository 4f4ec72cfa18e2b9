"""norm_amd -- MI355X-native Reed-Solomon FEC for NORM (RS8 / RS16 / MDP).

The hot path (parity generation and erasure repair over batches of FEC blocks) runs
as hand-written gfx950 HIP kernels in libnfec.so behind the C ABI of include/nfec.h.
This package is the Python mirror of the reference's NormEncoder/NormDecoder plugin
surface (include/normEncoder.h:38-54) plus batch entry points for device-resident data.
"""
from ._native import (NFEC_RS8, NFEC_RS16, NFEC_MDP, NFEC_ACCUMULATE, NFEC_FEATURE_RS16_TOEPLITZ,  # noqa: F401
                      NfecError, lib)
from .codec import (  # noqa: F401
    NormEncoderRS8, NormDecoderRS8, NormEncoderRS16, NormDecoderRS16, NormEncoderMDP, NormDecoderMDP,
    BlockLayout, build_generator, device_count, fill_blocks, make_erasures, stream_copy, zero_erasures,
)

__version__ = "0.1.0"
