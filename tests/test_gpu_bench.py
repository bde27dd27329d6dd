"""bench.py end to end on the GPU at small sizes, every workload with its CPU
baseline leg: the JSON contract the driver reads (metric / value / roofline /
cpu_baseline / check) and the planted-preamble check."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("workload", ["c5", "c2", "sync", "pfb"])
def test_bench_workload_small(gpu, workload):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload,
           "--samples", str(1 << 22), "--steps", "2", "--warmup", "1",
           "--cpu-samples", str(1 << 16), "--cpu-workers", "2", "--c2-samples", str(1 << 21),
           "--c2-steps", "2"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline", "check"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    assert d["check"]["ok"], d["check"]
    roof = d["roofline"]
    assert roof["bound"] == "hbm" and 0 < roof["frac"] < 1 and roof["avg_launch_ms"] > 0
    cpu = d["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] == "port"
    if workload == "c5":      # north_star's config-2 FIR+PSD leg rides along
        c2 = d["stages_roofline_c2"]
        assert c2["check"]["ok"], c2["check"]
        assert 0 < c2["fir+psd"]["hbm_frac"] < 1 and c2["samples"] == 1 << 21


@pytest.mark.parametrize("world,workload", [(2, "c5"), (4, "c5"), (8, "c5"), (2, "c2"), (2, "pfb")])
def test_bench_n_ranks_rehearsal_over_rccl(gpu, world, workload):
    """bench.py --gpus N end to end as the driver's N-GPU run executes it (its own
    launcher, one process per rank, torch.distributed over RCCL: halos by
    batch_isend_irecv, the peak all-gather, the per-rank line), with every rank
    on this box's one GPU over RCCL's socket transport (bench.rehearsal_env).
    The line carries the gathered per-rank diagnostics and the exact lag."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--workload",
           workload, "--samples", str(1 << 21), "--steps", "3", "--warmup", "1",
           "--rehearse-one-gpu"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                       # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["rccl_world"] == world and "rehearsal" in d
    assert d["check"]["ok"], d["check"]
    if workload == "pfb":
        return
    rk = d["ranks"]
    assert rk["world"] == world and 0 <= rk["pace_rank"] < world
    assert len(rk["per_rank"]) == world
    for k in ("fir", "psd", "xcorr", "refine"):
        assert rk[k]["min"] > 0
    for k in ("left_halo_wait", "right_halo_wait", "gather_wait"):
        assert rk[k]["max"] >= 0
    assert rk["ms_per_step"]["max"] == pytest.approx(d["ms_per_step"], rel=1e-3)
