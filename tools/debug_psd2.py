import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import vector_amd as va
N = 8192
n = np.arange(N)
for k0 in [0, 1, 5, 300, 4096]:
    x = np.exp(2j*np.pi*k0*n/N).astype(np.complex64)
    x = np.concatenate([x, x, x])
    _, _, S = va.spectrum(x, 1.0, "boxcar", N, 0, N)
    for f in range(3):
        s = S[:, f]
        big = np.nonzero(s > 1e-3)[0]
        print(k0, f, "argmax", s.argmax(), "max", s.max(), "nbig", len(big), big[:8], "sum", s.sum())
# impulse
for m in [0, 1, 17, 256, 511, 8191]:
    x = np.zeros(N, np.complex64); x[m] = 1
    _, _, S = va.spectrum(x, 1.0, "boxcar", N, 0, N)
    s = S[:, 0] * N * N
    print("delta", m, s.min(), s.max(), np.nonzero(np.abs(s-1) > 1e-3)[0][:10], len(np.nonzero(np.abs(s-1) > 1e-3)[0]))
