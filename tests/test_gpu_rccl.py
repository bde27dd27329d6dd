"""The production transport on the GPU at world 2: StreamChain + HipBackend over
TorchTransport = torch.distributed "nccl" (RCCL) -- batch_isend_irecv halos
and the asynchronous all_gather_into_tensor of the peak records, ordered
against torch's current stream exactly as bench.py --gpus N runs them.

The pool's boxes have one GPU, so both ranks run on cuda:0 as two processes;
RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"),
so each rank gets its own NCCL_HOSTID and the ranks talk through RCCL's
socket transport on the loopback interface (P2P / SHM off).  The wire is not
xGMI (that is for the 8-GPU run), but every RCCL call, stream dependency and
buffer of the product path is the real one.  Against the single-rank chain
over the whole capture: exact lag on both ranks for three steps with the
preamble moved each step (across the rank boundary: the right halo;
just after it: the left halo), filtered stream / spectra to 1e-5, and the
per-rank diagnostics bench.py gathers over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

N_LOCAL, DECIM, NFFT, L = 1 << 20, 4, 2048, 1024


def _case():
    import scipy.signal
    from oracle import ref
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L * DECIM, seed=71)
    tmpl = np.convolve(pre, taps)[: L * DECIM][::DECIM].astype(np.complex64)
    n = N_LOCAL
    ny = n // DECIM
    # preamble straddling the rank boundary, early in rank 1, late in rank 0
    k0s = [(ny - L // 2) * DECIM, (ny + 300) * DECIM, (ny - 3 * L) * DECIM]
    return taps, pre, tmpl, k0s


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", NCCL_HOSTID=f"vsig-rank{rank}",
                      NCCL_SOCKET_IFNAME="lo", NCCL_NET="Socket", NCCL_P2P_DISABLE="1",
                      NCCL_SHM_DISABLE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
    taps, pre, tmpl, k0s = _case()
    cfg = ChainConfig(n_local=N_LOCAL, taps=taps, decim=DECIM, nfft=NFFT, template=tmpl)
    be = HipBackend(cfg, 0)
    ch = StreamChain(cfg, be, rank, world)
    out = {}
    for s, k0 in enumerate(k0s):
        bench.generate_chunk(ch.x, rank * N_LOCAL, 900 + rank, pre, k0)
        if s == 2:
            ch.enable_wait_timing(True)
        ch.step()
        m, lag, s1, s2, nout = ch.global_peak()
        out[f"lag{s}"] = lag
        out[f"peak{s}"] = m
        out[f"y{s}"] = ch.y.cpu().numpy()
        out[f"sxx{s}"] = ch.sxx.cpu().numpy()
    waits = ch.wait_ms(1)
    rows = bench.gather_rank_rows(bench.rank_row(1e-3, 1, {"fir": 1.0}, waits), world, dev)
    out["ranks_world"] = bench.summarize_ranks(rows)["world"]
    out["right_halo_wait"] = waits["right_halo"]
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


def test_stream_chain_over_rccl_two_ranks(gpu, tmp_path):
    import torch.multiprocessing as mp
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    import sys
    sys.path.insert(0, ROOT)
    import bench
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=150)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "an RCCL rank did not finish"
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    # the single-rank chain over the whole capture (same generator, same seeds per chunk)
    taps, pre, tmpl, k0s = _case()
    N = world * N_LOCAL
    cfg = ChainConfig(n_local=N, taps=taps, decim=DECIM, nfft=NFFT, template=tmpl)
    whole = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
    for s, k0 in enumerate(k0s):
        for r in range(world):
            bench.generate_chunk(whole.x[r * N_LOCAL:(r + 1) * N_LOCAL], r * N_LOCAL, 900 + r, pre, k0)
        whole.step()
        m, lag, _, _, _ = whole.global_peak()
        assert lag == k0 // DECIM
        yw, sw = whole.y.cpu().numpy(), whole.sxx.cpu().numpy()
        y = np.concatenate([res[r][f"y{s}"] for r in range(world)])
        sx = np.concatenate([res[r][f"sxx{s}"] for r in range(world)])
        assert np.abs(y - yw).max() <= 1e-5 * np.abs(yw).max()
        assert np.abs(sx - sw).max() <= 1e-5 * sw.max()
        for r in range(world):
            assert int(res[r][f"lag{s}"]) == lag              # exact, on both ranks
            assert float(res[r][f"peak{s}"]) == pytest.approx(m, rel=1e-6)
    for r in range(world):
        assert int(res[r]["ranks_world"]) == world
        assert float(res[r]["right_halo_wait"]) >= 0.0
