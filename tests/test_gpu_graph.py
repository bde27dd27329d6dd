"""The chain step as a captured HIP graph (torch.cuda.CUDAGraph on ROCm).

Every size of the step is decided on the device -- the FIR / PSD / correlator
launches take their geometry from the host-known chunk shape, and the one-launch
refine (refine.hip refine_fused) sizes its candidate pass from the partials it
reduces and resets its own counters -- so StreamChain.step() (bench.py's step)
captures into a graph and replays with new input: the replayed results equal
the eager step's, bit for bit, and the planted preamble's lag is exact.
"""
import numpy as np
import pytest
import scipy.signal
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("decim", [4, 1])
def test_stream_chain_step_graph_replay(gpu, decim):
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    n, L, nfft = 1 << 20, 4096 // decim, 8192 // decim
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L * decim, seed=41)
    tmpl = np.convolve(pre, taps)[: L * decim][::decim].astype(np.complex64)
    base = ref.synth_iq(n, seed=42)
    k0s = [1000 * decim, (n // decim // 2) * decim, (n // decim - L - 50) * decim]
    xs = []
    for k in k0s:
        x = base.copy()
        x[k: k + L * decim] += 3 * pre
        xs.append(torch.from_numpy(x).cuda())
    cfg = ChainConfig(n_local=n, taps=taps, decim=decim, nfft=nfft, template=tmpl)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        ch = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
        want = []
        for x in xs:                                  # eager steps (also the warm-up)
            ch.x.copy_(x)
            ch.step()
            want.append((ch.y.clone(), ch.sxx.clone(), ch.rec.clone()))
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            ch.step()
        for s, x in enumerate(xs):
            ch.x.copy_(x)
            g.replay()
            st.synchronize()
            y, sxx, rec = want[s]
            assert torch.equal(ch.y, y)
            assert torch.equal(ch.sxx, sxx)
            assert torch.equal(ch.rec, rec)
            assert ch.global_peak()[1] == k0s[s] // decim      # exact lag
