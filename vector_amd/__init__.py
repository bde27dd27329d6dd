"""vector_amd — MI355X-native DSP hot path of ramiyako/vector.

FIR -> decimate -> block FFT / PSD -> sliding cross-correlation, as hand-written
CDNA4 HIP kernels in libvsig.so (C ABI, include/vsig.h), behind the reference's
own Python call signatures (utils.py).  No CPU fallback: without the library or
a HIP device every call raises ``VsigUnavailable``.
"""
from ._lib import RefineFault, VsigError, VsigUnavailable, get_context, load_library  # noqa: F401
from . import dsp  # noqa: F401
from .dsp import (Correlator, FirFilter, correlate, correlate_peak,  # noqa: F401
                  cross_correlate_signals, filter, find_correlation_peak,
                  find_packet_location_in_vector, fir_filter, peak_stats, spectrum)
from .spectrogram import create_spectrogram, spectrogram_params  # noqa: F401
from .channelizer import Channelizer, filter_channel, pfb_channelize  # noqa: F401
from .vectors import (apply_frequency_shift, resample_signal, load_packet, load_packet_info, mat2wv,  # noqa: F401
                      save_vector, save_vector_wv, transplant_packet_in_vector)
from .analysis import (boxcar_energy, detect_packet_bounds, find_packet_start,  # noqa: F401
                       normalize_spectrogram, order_statistics, threshold_stats)

__version__ = "0.1.0"
