"""Periodic (DFT-even) analysis windows, as ``scipy.signal.get_window(name, n,
fftbins=True)`` builds them for ``scipy.signal.spectrogram``
(scipy/signal/windows/_windows.py: general_cosine & friends; the reference uses
'hann', 'blackmanharris' and 'boxcar', utils.py:273-276,337).

Host-side setup of O(nperseg) coefficients (like a filter design), cached per
(name, n); the samples themselves never touch the host.
"""
from __future__ import annotations

import functools

import numpy as np

_COSINE = {
    "hann": (0.5, 0.5), "hanning": (0.5, 0.5), "han": (0.5, 0.5),
    "hamming": (0.54, 0.46), "hamm": (0.54, 0.46), "ham": (0.54, 0.46),
    "blackman": (0.42, 0.50, 0.08), "black": (0.42, 0.50, 0.08), "blk": (0.42, 0.50, 0.08),
    "blackmanharris": (0.35875, 0.48829, 0.14128, 0.01168),
    "blackharr": (0.35875, 0.48829, 0.14128, 0.01168),
    "bkh": (0.35875, 0.48829, 0.14128, 0.01168),
    "nuttall": (0.3635819, 0.4891775, 0.1365995, 0.0106411),
    "nutl": (0.3635819, 0.4891775, 0.1365995, 0.0106411),
    "nut": (0.3635819, 0.4891775, 0.1365995, 0.0106411),
    "flattop": (0.21557895, 0.41663158, 0.277263158, 0.083578947, 0.006947368),
    "flat": (0.21557895, 0.41663158, 0.277263158, 0.083578947, 0.006947368),
    "flt": (0.21557895, 0.41663158, 0.277263158, 0.083578947, 0.006947368),
}
_ONES = {"boxcar", "box", "ones", "rect", "rectangular"}


def _general_cosine_sym(m: int, a) -> np.ndarray:
    fac = np.linspace(-np.pi, np.pi, m)
    w = np.zeros(m)
    for k, ak in enumerate(a):
        w += ak * np.cos(k * fac)
    return w


def _periodic(sym_fn, n: int) -> np.ndarray:
    if n <= 1:
        return np.ones(n)
    return sym_fn(n + 1)[:-1]


@functools.lru_cache(maxsize=64)
def _named(name: str, param, n: int) -> np.ndarray:
    key = name.lower()
    if key in _COSINE:
        return _periodic(lambda m: _general_cosine_sym(m, _COSINE[key]), n)
    if key in _ONES:
        return np.ones(n)
    if key in ("bartlett", "bart", "brt"):
        return _periodic(lambda m: np.bartlett(m), n)
    if key in ("triang", "triangle", "tri"):
        def tri(m):
            k = np.arange(1, (m + 1) // 2 + 1)
            if m % 2 == 0:
                w = (2 * k - 1.0) / m
                return np.concatenate([w, w[::-1]])
            w = 2 * k / (m + 1.0)
            return np.concatenate([w, w[-2::-1]])
        return _periodic(tri, n)
    if key in ("kaiser", "ksr"):
        if param is None:
            raise ValueError("The 'kaiser' window needs a parameter -- pass a tuple.")
        return _periodic(lambda m: np.kaiser(m, float(param)), n)
    raise ValueError(f"Unknown window type: {name!r} (vector_amd supports {sorted(_COSINE) + sorted(_ONES)}"
                     " + bartlett, triang, kaiser)")


def get_window(window, n: int) -> np.ndarray:
    """float64 periodic window of length n (scipy.signal.get_window semantics
    for the supported names; tuples ('kaiser', beta))."""
    if isinstance(window, tuple):
        name, param = window[0], (window[1] if len(window) > 1 else None)
    else:
        name, param = window, None
    if not isinstance(name, str):
        raise ValueError(f"window must be a string, a tuple or an array, got {type(window)}")
    return _named(name, param, int(n)).copy()
