"""Instruction mix of one kernel in a device assembly file (tuning aid):
  python tools/isa_mix.py k.s SUBSTRING [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
for m in re.finditer(r"^(\S*" + re.escape(pat) + r"\S*):", s, re.M):
    nm = m.group(1)
    j = s.find(".Lfunc_end", m.end())
    body = s[m.end():j].splitlines()
    ops = collections.Counter()
    for l in body:
        l = l.strip()
        if not l or l.startswith((".", ";")) or l.endswith(":"):
            continue
        ops[l.split()[0]] += 1
    print(nm[:90], "total", sum(ops.values()))
    for k, v in ops.most_common(top):
        print(f"  {k:30s} {v}")
