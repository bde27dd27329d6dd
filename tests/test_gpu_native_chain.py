"""The C-ABI shard (vsig_chain_*, chain.hip) on the GPU.

* world 1: the native chain equals the Python StreamChain (same kernels, same
  order: bit-identical y / spectra / peak).
* world 2 and 3 through the in-process loopback transport (one host thread and
  context per rank, all on cuda:0): halos, frame alignment and the global
  argmax reproduce the single-rank chain over the whole capture (fp32 arrays to
  1e-5 of their maximum -- the overlap-save blocks fall differently -- exact
  lag).
* the RCCL transport at world 1 (an ncclComm_t of one rank made through
  vsig_rccl_comm_init): same result as without a transport.
"""
import ctypes as C
import threading

import numpy as np
import pytest
import scipy.signal
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _case(N, decim, L, seed):
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L * decim, seed=seed)
    tmpl = np.convolve(pre, taps)[: L * decim][::decim].astype(np.complex64)
    x = ref.synth_iq(N, seed=seed)
    k0 = (N // decim // 2 + 333) * decim
    x[k0: k0 + L * decim] += 3 * pre
    return taps, tmpl, x, k0


def _cfg(n, taps, decim, tmpl, nfft=1024):
    from vector_amd.shard import ChainConfig
    return ChainConfig(n_local=n, taps=taps, decim=decim, nfft=nfft, template=tmpl)


@pytest.mark.parametrize("decim", [1, 4])
def test_native_chain_world1_equals_python(gpu, decim):
    from vector_amd.shard import HipBackend, NativeChain, StreamChain
    N, L = 1 << 20, 512
    taps, tmpl, x, k0 = _case(N, decim, L, 3)
    cfg = _cfg(N, taps, decim, tmpl)
    xt = torch.from_numpy(x).cuda()
    py = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
    py.x.copy_(xt)
    py.step()
    nat = NativeChain(cfg, 0)
    nat.load(xt)
    nat.step()
    y, s = nat.outputs()
    torch.cuda.synchronize()
    assert torch.equal(y, py.y)
    assert torch.equal(s, py.sxx)
    a, b = nat.global_peak(), py.global_peak()
    assert a[1] == b[1] == k0 // decim
    assert a[0] == b[0] and a[4] == b[4]


@pytest.mark.parametrize("world,decim", [(2, 1), (3, 4), (2, 4)])
def test_native_chain_loopback_ranks(gpu, world, decim):
    from vector_amd.shard import Loopback, NativeChain
    n, L = 1 << 18, 700
    N = world * n
    taps, tmpl, x, k0 = _case(N, decim, L, 5 + world)
    whole = NativeChain(_cfg(N, taps, decim, tmpl), 0)
    whole.load(torch.from_numpy(x).cuda())
    whole.step()
    y1, s1 = whole.outputs()
    p1 = whole.global_peak()
    torch.cuda.synchronize()
    lb = Loopback(world)
    res, errs = [None] * world, []

    def rank_main(r):
        try:
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                ch = NativeChain(_cfg(n, taps, decim, tmpl), 0, r, world, lb.transport(r))
                ch.load(torch.from_numpy(x[r * n:(r + 1) * n]).cuda())
                ch.step()
                y, s = ch.outputs()
                pk = ch.global_peak()
                st.synchronize()
                res[r] = (y.cpu().numpy(), s.cpu().numpy(), pk)
                del ch
        except Exception as e:      # surfaced below
            errs.append(repr(e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    y = np.concatenate([res[r][0] for r in range(world)])
    s = np.concatenate([res[r][1] for r in range(world)])
    yw, sw = y1.cpu().numpy(), s1.cpu().numpy()
    assert np.abs(y - yw).max() <= 1e-5 * np.abs(yw).max()
    assert np.abs(s - sw).max() <= 1e-5 * sw.max()
    for r in range(world):
        pk = res[r][2]
        assert pk[1] == p1[1] == k0 // decim              # exact, on every rank
        assert pk[0] == pytest.approx(p1[0], rel=1e-6)
        assert pk[4] == p1[4]
        assert pk[2] == pytest.approx(p1[2], rel=1e-5)


@pytest.mark.parametrize("world", [2, 3])
def test_native_chain_loopback_multi_step(gpu, world):
    """Three steps per rank with the preamble at a different global offset each
    time (re-loaded inputs): the loopback's halo boxes and peak gather rounds
    are reused across steps, and every step reports its own lag on every rank."""
    from vector_amd.shard import Loopback, NativeChain
    n, L, decim = 1 << 17, 700, 4
    N = world * n
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L * decim, seed=21)
    tmpl = np.convolve(pre, taps)[: L * decim][::decim].astype(np.complex64)
    base = ref.synth_iq(N, seed=22)
    k0s = [(n // decim - L // 2) * decim, 1000 * decim, (N // decim - L - 50) * decim]
    xs = []
    for k in k0s:
        x = base.copy()
        x[k: k + L * decim] += 3 * pre
        xs.append(x)
    lb = Loopback(world)
    res, errs = [None] * world, []

    def rank_main(r):
        try:
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                ch = NativeChain(_cfg(n, taps, decim, tmpl), 0, r, world, lb.transport(r))
                got = []
                for x in xs:
                    ch.load(torch.from_numpy(x[r * n:(r + 1) * n]).cuda())
                    ch.step()
                    got.append(ch.global_peak())
                st.synchronize()
                res[r] = got
                del ch
        except Exception as e:      # surfaced below
            errs.append(repr(e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    for r in range(world):
        assert [g[1] for g in res[r]] == [k // decim for k in k0s]
        assert res[r] == res[0]


def test_native_chain_rccl_world1(gpu):
    from vector_amd._lib import Transport
    from vector_amd.shard import NativeChain
    ctx = gpu.get_context()
    lib = ctx.lib
    if not lib.vsig_rccl_available():
        pytest.skip("librccl not found")
    uid = C.create_string_buffer(128)
    ctx.check(lib.vsig_rccl_unique_id(uid), "unique id")
    comm = C.c_void_p()
    ctx.check(lib.vsig_rccl_comm_init(1, 0, uid, 0, C.byref(comm)), "comm init")
    try:
        tr = Transport()
        ctx.check(lib.vsig_rccl_transport(comm, C.byref(tr)), "transport")
        N, L = 1 << 19, 300
        taps, tmpl, x, k0 = _case(N, 2, L, 9)
        xt = torch.from_numpy(x).cuda()
        a = NativeChain(_cfg(N, taps, 2, tmpl), 0, 0, 1, tr)
        a.load(xt)
        a.step()
        b = NativeChain(_cfg(N, taps, 2, tmpl), 0)
        b.load(xt)
        b.step()
        assert a.global_peak() == b.global_peak()
        assert a.global_peak()[1] == k0 // 2
        del a, b
    finally:
        lib.vsig_rccl_comm_destroy(comm)


def test_c_shard_example_loopback(gpu, tmp_path):
    """examples/shard_c.c from plain C: 3 ranks as threads on cuda:0 through the
    loopback transport; exit 0 = every rank reports the preamble's lag."""
    import subprocess
    from test_host_cpu import _build_c_example
    exe = _build_c_example(str(tmp_path / "shard_c"), "shard_c")
    r = subprocess.run([exe, "loopback", "3"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("global peak") == 3


def test_c_shard_example_rccl_world1(gpu, tmp_path):
    """examples/shard_c.c over RCCL (one rank): the unique id, comm init and the
    peak all-gather through librccl from C."""
    import subprocess
    from test_host_cpu import _build_c_example
    exe = _build_c_example(str(tmp_path / "shard_c"), "shard_c")
    r = subprocess.run([exe, "rccl", "0", "1", str(tmp_path / "uid")], capture_output=True,
                       text=True, timeout=120)
    if r.returncode == 2 and "no RCCL" in r.stderr:
        pytest.skip("librccl not found")
    assert r.returncode == 0, r.stdout + r.stderr


def test_c_shard_example_rccl_world2_one_gpu(gpu, tmp_path):
    """examples/shard_c.c over RCCL at world 2 from plain C (ncclSend / ncclRecv
    halos and ncclAllGather peaks through vsig_rccl_transport), both ranks on
    this box's one GPU: each process names its own NCCL_HOSTID, so RCCL runs its
    socket transport on loopback (bench.rehearsal_env).  Exit 0 on both = every
    rank found the preamble at its global lag."""
    import os
    import subprocess
    import sys
    from test_host_cpu import _build_c_example
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    exe = _build_c_example(str(tmp_path / "shard_c"), "shard_c")
    uid = str(tmp_path / "uid2")
    procs = []
    for r in range(2):
        env = dict(os.environ, **bench.rehearsal_env(r))
        procs.append(subprocess.Popen([exe, "rccl", str(r), "2", uid, "0"], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    if any(rc == 2 and "no RCCL" in e for rc, _, e in outs):
        pytest.skip("librccl not found")
    assert all(rc == 0 for rc, _, _ in outs), outs
    assert sum(o.count("global peak") for _, o, _ in outs) == 2
