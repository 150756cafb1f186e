"""srcdsp_amd -- MI355X (gfx950) implementation of SrcDsp's sample-buffer hot path.

The operators (FilterDnsamplingFir, FilterFir, FilterUpsamplingFir, Mixer,
FixedPatternCorrelator, FifoWithTimeTrack; files.read/saveBinarySamples) mirror the reference classes and run in the HIP
kernels of libsrcdsp_hip.so through its C ABI (include/srcdsp_hip.h).
"""
from ._capi import SrcdspError, lib  # noqa: F401
from . import files  # noqa: F401
from .operators import (  # noqa: F401
    FifoWithTimeTrack,
    FilterDnsamplingFir,
    FilterFir,
    FilterUpsamplingFir,
    FixedPatternCorrelator,
    Mixer,
    MixerDecimatorChain,
    decim_step_batched,
    fill_synthetic,
)

__all__ = ["FifoWithTimeTrack", "files", "FilterDnsamplingFir", "FilterFir", "FilterUpsamplingFir", "Mixer", "MixerDecimatorChain",
           "FixedPatternCorrelator", "decim_step_batched", "fill_synthetic", "SrcdspError", "lib"]
