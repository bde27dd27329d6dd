"""Pin the refine's cross-block hand-off protocol in the generated ISA
(the hand-offs rely on gfx950 code generation, not on C++
release / acquire).  refine.hip hands data between workgroups as
  agent-scope atomic stores of the payload (global_store ... sc1)
  -> s_waitcnt vmcnt(0) (stores_done: acknowledged)
  -> the signal: an atomic add on a counter or on the keys' flag
     (global_atomic_add_x2; refine_fused publishes its flag that way too)
and reads it back with agent-scope atomic loads (global_load ... sc1).
This tool disassembles the device code object of refine.hip's compiled
object and checks, per kernel, that every global_atomic_add_x2 has no
global store or atomic issued after the last s_waitcnt vmcnt(0) before it
(nothing the signal covers can still be in flight), and that refine_fused
polls and reads the published words with sc1 loads (past the CU's L1).
MI355X_MICROARCH.md, 'Valid forms' (sc1 payload + drained vmcnt + signal).

  python tools/isa_handoffs.py [object.o]     (default: the product object)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(obj: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "co.o")
        subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x.o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                        f"--output={co}", "--unbundle"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                              capture_output=True, text=True).stdout


def kernels(dis: str):
    """{symbol: [instruction text]} for each function in the disassembly."""
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur and line.startswith("\t"):
            out[cur].append(line.strip().split("//")[0].strip())
    return out


def _is_vmcnt0(ins: str) -> bool:
    return ins.startswith("s_waitcnt") and ("vmcnt(0)" in ins or ins == "s_waitcnt 0")


def check(instrs):
    """Violations in one kernel: signals with a memory write still in flight."""
    bad = []
    for i, ins in enumerate(instrs):
        if not ins.startswith("global_atomic_add_x2"):
            continue
        for j in range(i - 1, -1, -1):
            p = instrs[j]
            if _is_vmcnt0(p):
                break
            if p.startswith(("global_store", "global_atomic", "buffer_store", "flat_store")):
                bad.append((i, ins, j, p))
                break
    return bad


def main(obj: str | None = None) -> int:
    if obj is None:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from vector_amd import _build
        obj = _build.compile_object("refine.hip")
    ks = {k: v for k, v in kernels(disassemble(obj)).items() if "refine" in k}
    nsig = nbad = 0
    for name, ins in sorted(ks.items()):
        nsig += sum(1 for x in ins if x.startswith("global_atomic_add_x2"))
        # every load of a word the signals guard (same base registers as a
        # signalling atomic: the counters, the flag, the keys) bypasses L1
        bases = {m.group(1) for x in ins if x.startswith("global_atomic_add_x2")
                 for m in [re.search(r"(s\[\d+:\d+\])", x)] if m}
        for x in ins:
            m = re.search(r"(s\[\d+:\d+\])", x)
            if x.startswith("global_load") and m and m.group(1) in bases and "sc1" not in x:
                nbad += 1
                print(f"VIOLATION {name[:60]}: '{x}' reads a hand-off word without sc1")
        for i, s, j, p in check(ins):
            nbad += 1
            print(f"VIOLATION {name[:60]}: '{s}' at {i} with '{p}' at {j} still in flight")
    print(f"{len(ks)} refine kernels, {nsig} signalling atomics, {nbad} violations")
    return 1 if nbad else 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:2]))
