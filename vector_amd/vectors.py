"""The data formats and element-wise steps either side of the chain
(SURVEY.md §8(f) f2-f4), with the bulk work on the GPU:

  apply_frequency_shift        utils.py:120-127            mix_c64 kernel
  transplant_packet_in_vector  utils.py:1437-1501          |x|^2 sums + scale_c64
  mat2wv / save_vector_wv      mat_to_wv_converter.py:7-64, utils.py:672-677
                                                           wv_quantize kernel
  load_packet / load_packet_info / save_vector
                               utils.py:48-105, 659-670    MAT v5 planes <-> complex64
                                                           (planar_to_c64 / c64_to_planar)

The MAT v5 container (128-byte header, tagged data elements) and the SMU-WV
text header are parsed / written on the host (O(1) work); sample planes move
as raw bytes and are converted on the device.  Reference semantics are kept:
the same dtypes, the same printed messages, the same error conditions.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import time
import zlib
from datetime import datetime

import numpy as np
import torch

from . import _lib
from .dsp import _device_c64, _is_dev, _ptr, peak_stats

__all__ = ["apply_frequency_shift", "resample_signal", "transplant_packet_in_vector", "mat2wv",
           "save_vector_wv",
           "load_packet", "load_packet_info", "save_vector", "read_mat", "write_mat_vector"]


def _as_out(t: torch.Tensor, like_dev: bool):
    return t if like_dev else t.cpu().numpy()


# ---------------------------------------------------------------------------
# apply_frequency_shift — utils.py:120-127
# ---------------------------------------------------------------------------
def apply_frequency_shift(signal, freq_shift, sample_rate, start_index: int = 0):
    """signal * exp(2j*pi*freq_shift*t), t = arange(n)/sample_rate, as complex64.
    The phase is formed in double precision exactly as numpy forms it
    (w = (2*pi)*f, theta = w * (i / sr)), reduced modulo 2*pi in double, and the
    rotation applied in fp32 (agrees with the reference to ~1e-7 relative).
    ``start_index`` offsets t (for time-chunk shards of one capture)."""
    if freq_shift == 0:
        return signal
    ctx = _lib.get_context()
    x = _device_c64(signal, ctx)
    n = int(x.shape[0])
    y = torch.empty_like(x)
    w = (2j * np.pi * freq_shift).imag          # the imaginary part numpy multiplies t by
    ctx.bind_stream()
    ctx.check(ctx.lib.vsig_mix_c64_dev(ctx.h, _ptr(x), n, float(w), float(sample_rate),
                                       int(start_index), _ptr(y)), "mix")
    return _as_out(y, _is_dev(signal))


# ---------------------------------------------------------------------------
# transplant_packet_in_vector — utils.py:1437-1501
# ---------------------------------------------------------------------------
def resample_signal(signal, orig_sr, target_sr):
    """utils.py:107-118: ``scipy.signal.resample(signal, int(len * ratio))`` as
    complex64 -- the spectrum of any length (Bluestein on the FFT engine,
    bigfft.hip), its bins copied into the new length with scipy's Nyquist
    rule, the inverse transform of any length.  Returns ``signal`` itself when
    the rates are equal, like the reference."""
    if orig_sr == target_sr:
        return signal
    dev = _is_dev(signal)
    n = int(signal.shape[0]) if dev else len(signal)
    num = int(n * (target_sr / orig_sr))
    if num < 1:
        raise ValueError(f"invalid number of data points ({num}) specified")
    ctx = _lib.get_context()
    if dev:
        real = not signal.is_complex()
        t = signal.to(torch.complex128 if signal.dtype in (torch.complex128, torch.float64)
                      else torch.complex64).contiguous()
    else:
        a = np.asarray(signal)
        real = not np.iscomplexobj(a)
        wide = a.dtype in (np.complex128, np.float64, np.longdouble, np.clongdouble) or \
            np.issubdtype(a.dtype, np.integer)
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.complex128 if wide else np.complex64)
                             ).to(f"cuda:{ctx.device}")
    code = "c128" if t.dtype == torch.complex128 else "c64"
    y = torch.empty(num, dtype=torch.complex64, device=t.device)
    ctx.check(ctx.lib.vsig_resample_dev(ctx.h, _lib.DTYPES[code], _ptr(t), n, num, 1 if real else 0,
                                        _ptr(y)), "resample")
    return y if dev else y.cpu().numpy()


def _mean_power(t: torch.Tensor) -> np.float32:
    """np.mean(np.abs(seg) ** 2) of a complex64 segment: sum in double on the
    GPU, rounded to the float32 numpy returns."""
    if t.numel() == 0:
        return np.float32(np.nan)
    _, _, _, s2, n = peak_stats(t)
    return np.float32(s2 / n)


def transplant_packet_in_vector(vector, packet_signal, vector_location, packet_location=0,
                                replace_length=None, normalize_power=True):
    """utils.py:1437-1501: a copy of ``vector`` with
    packet_signal[packet_location : +L] (power-normalised to the region it
    replaces when normalize_power) written at vector_location.  complex64
    vectors (the reference's load_packet dtype); numpy in -> numpy out."""
    ctx = _lib.get_context()
    dev_in = _is_dev(vector)
    if dev_in:
        if vector.dtype != torch.complex64:
            raise NotImplementedError("transplant_packet_in_vector: complex64 vectors only")
        v = vector.contiguous()
    else:
        va = np.asarray(vector)
        if va.dtype != np.complex64:
            raise NotImplementedError("transplant_packet_in_vector: complex64 vectors only")
        v = torch.from_numpy(np.ascontiguousarray(va)).to(f"cuda:{ctx.device}")
    p = _device_c64(packet_signal, ctx)
    new = v.clone()
    nv, npk = int(v.shape[0]), int(p.shape[0])
    if replace_length is None:
        replace_length = npk - packet_location
    vector_end = min(vector_location + replace_length, nv)
    actual_replace_length = vector_end - vector_location
    packet_end = min(packet_location + actual_replace_length, npk)
    actual_packet_length = packet_end - packet_location
    if 0 <= vector_location < nv and actual_packet_length > 0:
        seg = p[packet_location:packet_location + actual_packet_length]
        scale = None
        if normalize_power and actual_packet_length > 0:
            orig = v[vector_location:vector_location + actual_packet_length]
            original_power = _mean_power(orig)
            packet_power = _mean_power(seg)
            if packet_power > 0 and original_power > 0:
                scale = np.sqrt(original_power / packet_power)
                print(f"Power normalization applied: scale factor = {scale:.3f}")
            elif packet_power == 0:
                print("Warning: Packet has zero power - normalization skipped")
            elif original_power == 0:
                print("Warning: Original region has zero power - normalization skipped")
        dst = new[vector_location:vector_location + actual_packet_length]
        if not dst.is_contiguous() or not seg.is_contiguous():
            raise RuntimeError("internal: non-contiguous transplant views")
        ctx.bind_stream()
        ctx.check(ctx.lib.vsig_scale_c64_dev(ctx.h, _ptr(seg), int(actual_packet_length),
                                             float(scale) if scale is not None else 1.0, _ptr(dst)),
                  "scale")
    return _as_out(new, dev_in)


# ---------------------------------------------------------------------------
# SMU-WV writer — vector_analyzer/mat_to_wv_converter.py:7-64
# ---------------------------------------------------------------------------
def _max_abs_f32(x: torch.Tensor) -> np.float32:
    """np.max(np.abs(x)) of complex64 x, with numpy's complex-abs formula."""
    ctx = _lib.get_context()
    n = int(x.shape[0])
    a = torch.empty(n, dtype=torch.complex64, device=x.device)
    ctx.check(ctx.lib.vsig_abs_c64_dev(ctx.h, _lib.DTYPES["c64"], _ptr(x), n, _ptr(a)), "abs")
    from .analysis import _thresh_dev
    f = torch.view_as_real(a).reshape(-1)
    _, _, _, mx = _thresh_dev(ctx, f, "f32", np.inf)
    return np.float32(mx)


def mat2wv(path_signal, sFilename, fSampleRate, bNormalize=True, var_name=None):
    """mat2wv (mat_to_wv_converter.py:7-64): quantise to interleaved int16 I/Q on
    the GPU and write the SMU-WV file (same header fields and order)."""
    ctx = _lib.get_context()
    if isinstance(path_signal, str):
        if var_name is None:
            raise ValueError("When path_signal is a filename, var_name must be specified")
        data = read_mat(path_signal)
        if var_name not in data:
            raise KeyError(var_name)
        x = _load_complex64_dev(data, var_name, ctx)
    elif _is_dev(path_signal):
        x = _device_c64(path_signal.reshape(-1), ctx)
    else:
        x = _device_c64(np.asarray(path_signal).flatten(), ctx)
    N = int(x.shape[0])
    norm = 0.0
    if bNormalize:
        print("Normalize signal")
        m = _max_abs_f32(x)
        norm = float(m)
        # peak / mean power of the normalised signal (metadata of the header)
        xs = torch.empty_like(x)
        ctx.check(ctx.lib.vsig_scale_c64_dev(ctx.h, _ptr(x), N, float(np.float32(1) / m)
                                             if m else 0.0, _ptr(xs)), "scale")
        _, peak, _, s2, _ = peak_stats(xs)
        fPeakPower = np.float32(np.float32(peak) ** 2)
        fPeakPowerdBfs = -10 * np.log10(fPeakPower)
        fMeanPower = np.float32(s2 / N)
        fRMSdBfs = -10 * np.log10(fMeanPower)
    else:
        fPeakPowerdBfs = 0.0
        fRMSdBfs = 0.0
    q = torch.empty(2 * N, dtype=torch.int16, device=x.device)
    ctx.bind_stream()
    ctx.check(ctx.lib.vsig_wv_quantize_dev(ctx.h, _ptr(x), N, float(norm), _ptr(q)), "wv")
    interleaved = q.cpu().numpy()
    total_bytes = 4 * N + 1
    with open(sFilename, "wb") as fid:
        fid.write("{TYPE: SMU-WV,0}".encode())
        fid.write("{COMMENT: Generated by mat2wv.py}".encode())
        fid.write(f"{{DATE: {datetime.now().strftime('%Y-%m-%d;%H:%M:%S')}}}".encode())
        fid.write(f"{{LEVEL OFFS: {fRMSdBfs}, {fPeakPowerdBfs}}}".encode())
        fid.write(f"{{CLOCK: {fSampleRate}}}".encode())
        fid.write(f"{{SAMPLES: {N}}}".encode())
        fid.write(f"{{WAVEFORM-{total_bytes}:#".encode())
        fid.write(interleaved.tobytes())
        fid.write(b"}")


def save_vector_wv(vector, output_path, sample_rate, normalize=False):
    """utils.py:672-677."""
    mat2wv(vector, output_path, sample_rate, bNormalize=normalize)


# ---------------------------------------------------------------------------
# MAT v5 (uncompressed and miCOMPRESSED elements) — the subset scipy.io
# loadmat / savemat produce for the reference's packets and vectors
# ---------------------------------------------------------------------------
_MI_NP = {1: np.int8, 2: np.uint8, 3: np.int16, 4: np.uint16, 5: np.int32, 6: np.uint32,
          7: np.float32, 9: np.float64, 12: np.int64, 13: np.uint64}
_MX_NP = {6: np.float64, 7: np.float32, 8: np.int8, 9: np.uint8, 10: np.int16, 11: np.uint16,
          12: np.int32, 13: np.uint32, 14: np.int64, 15: np.uint64}


def _tag(buf, off, endian):
    t, n = struct.unpack(endian + "II", buf[off:off + 8])
    if t >> 16:                                   # small data element
        return t & 0xFFFF, t >> 16, off + 4, off + 8
    return t, n, off + 8, off + 8 + ((n + 7) // 8) * 8


def _parse_matrix(buf, endian):
    """-> (name, mx_class, dims, complex, (re_type, re_bytes), (im_type, im_bytes))."""
    off = 0
    t, n, d, off = _tag(buf, off, endian)         # array flags
    flags = struct.unpack(endian + "I", buf[d:d + 4])[0]
    mx_class, is_complex = flags & 0xFF, bool(flags & 0x800)
    t, n, d, off = _tag(buf, off, endian)         # dimensions
    dims = struct.unpack(endian + f"{n // 4}i", buf[d:d + n])
    t, n, d, off = _tag(buf, off, endian)         # name
    name = bytes(buf[d:d + n]).decode("latin1")
    if mx_class not in _MX_NP:
        return name, mx_class, dims, is_complex, None, None
    t, n, d, off = _tag(buf, off, endian)
    re = (t, buf[d:d + n])
    im = None
    if is_complex:
        t, n, d, off = _tag(buf, off, endian)
        im = (t, buf[d:d + n])
    return name, mx_class, dims, is_complex, re, im


def _mat_elements(path):
    raw = np.memmap(path, dtype=np.uint8, mode="r")
    if len(raw) < 128:
        raise ValueError(f"{path}: not a MAT-file")
    endian = "<" if bytes(raw[126:128]) == b"IM" else ">"
    if struct.unpack(endian + "H", bytes(raw[124:126]))[0] != 0x0100:
        raise NotImplementedError(f"{path}: only MAT v5 files are supported (v7.3 is HDF5)")
    header = bytes(raw[:116]).rstrip(b"\x00 ")
    off = 128
    elems = []
    mv = memoryview(raw)
    while off + 8 <= len(raw):
        t, n = struct.unpack(endian + "II", bytes(raw[off:off + 8]))
        body = mv[off + 8:off + 8 + n]
        off += 8 + ((n + 7) // 8) * 8
        if t == 15:                               # miCOMPRESSED: one zlib stream
            inner = zlib.decompress(bytes(body))
            t2, n2 = struct.unpack(endian + "II", inner[:8])
            if t2 == 14:
                elems.append(_parse_matrix(memoryview(inner)[8:8 + n2], endian))
        elif t == 14:
            elems.append(_parse_matrix(body, endian))
    return header, endian, elems


def _plane_to_np(plane, endian):
    t, b = plane
    dt = np.dtype(_MI_NP[t]).newbyteorder(endian)
    return np.frombuffer(b, dtype=dt)


def read_mat(path):
    """{name: value} for the numeric arrays of a MAT v5 file, on the host
    (scalars as Python numbers, arrays squeezed) — loadmat(squeeze_me=True)'s
    view of the reference's files.  Sample planes of complex arrays are kept as
    raw planes under key (name, 'planes') for the GPU loader."""
    header, endian, elems = _mat_elements(path)
    out = {"__header__": header, "__version__": "1.0", "__globals__": []}
    for name, mx_class, dims, is_complex, re, im in elems:
        if re is None:
            continue
        r = _plane_to_np(re, endian)
        if len(r) > 4:                            # sample planes: converted on the GPU
            out[(name, "planes")] = (re, im, endian, dims)
            arr = None
        elif is_complex:
            arr = r.astype(np.float64) + 1j * _plane_to_np(im, endian).astype(np.float64)
        else:
            arr = r.astype(_MX_NP[mx_class])
        if arr is not None:
            arr = arr.reshape(dims, order="F").squeeze()
            out[name] = arr.item() if arr.ndim == 0 else arr
        else:
            out[name] = None                      # materialised by the GPU loader
    return out


def _packet_var(data, file_path):
    if "Y" in data:
        return "Y"
    candidates = [k for k in data.keys() if isinstance(k, str) and not k.startswith("__")]
    if len(candidates) == 1:
        return candidates[0]
    keys = [k for k in data.keys() if isinstance(k, str)]
    raise ValueError(f"Ambiguous packet data in {file_path}. Available keys: {keys}")


def _load_complex64_dev(data, name, ctx):
    """GPU conversion of a variable's planes to a flat complex64 tensor."""
    planes = data.get((name, "planes"))
    dev = f"cuda:{ctx.device}"
    if planes is None:                            # real array (or scalar)
        val = np.asarray(data[name]).ravel(order="F")
        return torch.from_numpy(np.ascontiguousarray(val.astype(np.complex64))).to(dev)
    (rt, rb), im, endian, dims = planes
    n = int(np.prod(dims))
    if rt not in _MI_NP:
        raise NotImplementedError(f"MAT storage type {rt}")
    if endian != "<":
        raise NotImplementedError("big-endian MAT files")
    re_d = torch.frombuffer(bytearray(rb), dtype=torch.uint8).to(dev)
    im_d = torch.frombuffer(bytearray(im[1]), dtype=torch.uint8).to(dev) if im else None
    if im is not None and im[0] != rt:            # mixed storage types: bring imag to re's
        imv = _plane_to_np(im, endian).astype(_MI_NP[rt])
        im_d = torch.from_numpy(imv.view(np.uint8).copy()).to(dev)
    y = torch.empty(n, dtype=torch.complex64, device=dev)
    ctx.bind_stream()
    ctx.check(ctx.lib.vsig_planar_to_c64_dev(ctx.h, int(rt), _ptr(re_d),
                                             _ptr(im_d) if im_d is not None else None, n, _ptr(y)),
              "planar_to_c64")
    # MATLAB is column-major: a 1-D capture (1 x n or n x 1) is already in order;
    # a 2-D matrix is flattened in C order like packet.flatten() after loadmat
    if len(dims) == 2 and dims[0] > 1 and dims[1] > 1:
        y = y.view(dims[1], dims[0]).t().contiguous().view(-1)
    return y


def load_packet(file_path, device: bool = False):
    """utils.py:48-86: the 'Y' variable (or the only variable) as a flat
    complex64 array; device=True keeps it in HBM (torch tensor)."""
    try:
        file_size_mb = os.path.getsize(file_path) / (1024 * 1024)
        is_large_file = file_size_mb > 50
        if is_large_file:
            print(f"📁 Loading large file: {file_size_mb:.1f}MB")
        ctx = _lib.get_context()
        data = read_mat(file_path)
        name = _packet_var(data, file_path)
        packet = _load_complex64_dev(data, name, ctx)
        if packet.numel() > 20_000_000:
            duration_sec = packet.numel() / 56e6
            memory_mb = packet.numel() * 8 / (1024 * 1024)
            print(f"⚠️ Heavy packet loaded: {packet.numel():,} samples ({duration_sec:.2f}s, "
                  f"{memory_mb:.1f}MB)")
        return packet if device else packet.cpu().numpy()
    except Exception as e:
        print(f"Error loading packet from {file_path}: {e}")
        raise


def load_packet_info(file_path, device: bool = False):
    """utils.py:88-105: (packet complex64, pre_samples)."""
    ctx = _lib.get_context()
    data = read_mat(file_path)
    name = _packet_var(data, file_path)
    packet = _load_complex64_dev(data, name, ctx)
    pre = int(data.get("pre_samples", 0))
    return (packet if device else packet.cpu().numpy()), pre


def write_mat_vector(output_path, y_re: np.ndarray, y_im: np.ndarray, pre_samples: int = 0):
    """scipy.io.savemat(path, {'Y': complex64 row vector, 'pre_samples': int})
    byte layout (format 5, oned_as='row'); the header carries the write time."""
    n = len(y_re)
    if 4 * n >= 2 ** 32:
        raise ValueError("Matrix too large to save with Matlab 5 format")

    def pad8(b):
        return b + b"\x00" * ((8 - len(b) % 8) % 8)

    def el(t, payload):
        return struct.pack("<II", t, len(payload)) + pad8(payload)

    hdr = (f"MATLAB 5.0 MAT-file Platform: {os.name}, Created on: {time.asctime()}"
           ).encode().ljust(116, b"\x00")
    hdr += b"\x00" * 8 + struct.pack("<H", 0x0100) + b"IM"
    y = (el(6, struct.pack("<II", 0x0800 | 7, 0)) + el(5, struct.pack("<ii", 1, n))
         + struct.pack("<HH", 1, 1) + b"Y\x00\x00\x00"
         + el(7, y_re.astype("<f4").tobytes()) + el(7, y_im.astype("<f4").tobytes()))
    pre = (el(6, struct.pack("<II", 14, 0)) + el(5, struct.pack("<ii", 1, 1))
           + el(1, b"pre_samples") + el(12, struct.pack("<q", int(pre_samples))))
    with open(output_path, "wb") as f:
        f.write(hdr + el(14, y) + el(14, pre))


def save_vector(vector, output_path):
    """utils.py:659-670: flat complex64 'Y' + pre_samples=0, planes split on the GPU."""
    ctx = _lib.get_context()
    if _is_dev(vector):
        x = _device_c64(vector.reshape(-1), ctx)
    else:
        x = _device_c64(np.asarray(vector).flatten(), ctx)
    n = int(x.shape[0])
    re = torch.empty(n, dtype=torch.float32, device=x.device)
    im = torch.empty(n, dtype=torch.float32, device=x.device)
    ctx.bind_stream()
    ctx.check(ctx.lib.vsig_c64_to_planar_dev(ctx.h, _ptr(x), n, _ptr(re), _ptr(im)), "planes")
    write_mat_vector(output_path, re.cpu().numpy(), im.cpu().numpy(), 0)
