import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import vector_amd as va
from oracle import ref
for nfft in [4096, 8192, 16384]:
    for nframes in [1, 2, 5, 16]:
        x = ref.synth_iq(nfft * nframes, seed=3)
        _, _, S = va.spectrum(x, 1.0, "hann", nfft, 0, nfft)
        _, _, R = ref.spectrum(x, 1.0, "hann", nfft, 0, nfft)
        err = np.abs(S - R).max(axis=0) / R.max(axis=0)
        print(nfft, nframes, np.array2string(err, precision=2))
        sys.stdout.flush()
