"""The refine's cross-block hand-offs as compiled: every
signalling atomic add (counters, the keys' flag) is issued behind a drained
vmcnt with no store in flight, and every read of a guarded word is an sc1
load (tools/isa_handoffs.py on refine.hip's product object; no GPU)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_refine_handoffs_in_isa(capsys):
    if not (shutil.which("objcopy") and os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump")):
        pytest.skip("binutils / ROCm llvm tools not present")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_handoffs
    rc = isa_handoffs.main()
    out = capsys.readouterr().out
    assert rc == 0, out
    assert "0 violations" in out
    n = int(out.split(" signalling atomics")[0].split()[-1])
    assert n >= 8, out        # the fused launch's tickets, counters, seen and flag are all there
