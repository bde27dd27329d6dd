"""Debug: GPU refined correlation vs numpy bits near the max (tone golden)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import vector_amd as va
from oracle import npdot
g = np.load("tests/golden/tone_transplant.npz")
for i in (1, 3):
    vec, seg = g["vector"], g[f"seg{i}"]
    r = np.correlate(vec.astype(np.complex128), seg, "full")
    ar = np.abs(r)
    c, lags = va.cross_correlate_signals(seg, vec)
    ac = np.abs(c)
    st = va.dsp.refine_status()
    top = np.argsort(-ar)[:8]
    print("case", i, "status", st, "numpy argmax", int(np.argmax(ar)), "gpu argmax", int(np.argmax(ac)),
          "golden", int(g[f"vec{i}_argmax"]))
    for k in top:
        print(f"  k={k} np={ar[k]!r} gpu={ac[k]!r} c_eq={c[k] == r[k]} dre={c[k].real - r[k].real:.3e} dim={c[k].imag - r[k].imag:.3e}")
    lag, val, conf = va.correlate_peak(seg, vec)
    print("  fused", lag, repr(val), "want", g[f"vec{i}_peak"][:2])
    pk = g[f"packet{i}"]
    lag, val, conf = va.correlate_peak(seg, pk)
    print("  self", lag, repr(val), "want", g[f"pkt{i}_peak"][:2], va.dsp.refine_status())
