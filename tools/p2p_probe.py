"""Which RCCL transport two ranks on the one GPU of a pool box get (verdict r05
item 7: a rehearsal with RCCL's P2P transport left enabled).

  python tools/p2p_probe.py OUTDIR

Runs two 2-rank all-reduces on cuda:0 (children of this script, 60 s bound
each, NCCL_DEBUG=INFO): (a) one host id for both ranks and P2P / SHM enabled
-- the only setting in which RCCL could pick its P2P transport; (b) a host id
per rank, P2P / SHM still enabled (bench.rehearsal_env minus its
NCCL_P2P_DISABLE / NCCL_SHM_DISABLE).  Writes each case's exit status and the
RCCL lines that name a transport or refuse the setup to OUTDIR/p2p_probe.txt.
"""
import os
import re
import subprocess
import sys


def child():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    t = torch.ones(1 << 20, device="cuda") * (dist.get_rank() + 1)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    ok = float(t[0].item()) == 3.0
    print(f"rank {dist.get_rank()} allreduce {'ok' if ok else 'WRONG'}", flush=True)
    dist.destroy_process_group()


def run_case(name, per_rank_host, outdir):
    from torch.distributed import TCPStore
    store = TCPStore("127.0.0.1", 0, world_size=None, is_master=True, wait_for_workers=False)
    procs, logs = [], []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(store.port), TORCHELASTIC_USE_AGENT_STORE="True",
                   NCCL_DEBUG="INFO", NCCL_SOCKET_IFNAME="lo")
        for k in ("NCCL_P2P_DISABLE", "NCCL_SHM_DISABLE", "NCCL_NET"):
            env.pop(k, None)
        env["NCCL_HOSTID"] = f"vsig-rank{r}" if per_rank_host else "vsig-host"
        log = open(os.path.join(outdir, f"p2p_{name}_rank{r}.log"), "w")
        logs.append(log)
        procs.append(subprocess.Popen(["timeout", "-k", "10", "60", sys.executable,
                                       os.path.abspath(__file__), "--child"],
                                      env=env, stdout=log, stderr=subprocess.STDOUT))
    codes = [p.wait() for p in procs]
    for log in logs:
        log.close()
    del store
    keep = re.compile(r"via |Duplicate|P2P|SHM|NET/|error|Error|allreduce")
    lines = []
    for r in range(2):
        for line in open(os.path.join(outdir, f"p2p_{name}_rank{r}.log")):
            if keep.search(line):
                lines.append(f"  rank{r}: {line.rstrip()[:200]}")
    return codes, lines


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    out = []
    for name, per in (("one_host", False), ("host_per_rank", True)):
        codes, lines = run_case(name, per, outdir)
        out.append(f"case {name}: exit codes {codes}")
        out.extend(lines[:40])
    open(os.path.join(outdir, "p2p_probe.txt"), "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    if "--child" in sys.argv:
        child()
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/p2p")
