"""Build the A/B libraries next to libvsig.so (same sources, extra defines)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vector_amd import _build  # noqa: E402

# name -> defines of a current A/B (the define lives in the kernel sources only
# while its measurement is open; measured alternatives are deleted with it and
# recorded in DESIGN.md, see round 3's list)
VARIANTS = {
    "libvsig_rtrace": ("VSIG_REFINE_TRACE=1",),
}
# name -> {source: extra compiler flags} (code-generation A/Bs)
FLAG_VARIANTS = {
}
for name in (sys.argv[1:] or list(VARIANTS) + list(FLAG_VARIANTS)):
    _build.build(defines=VARIANTS.get(name, ()), src_flags=FLAG_VARIANTS.get(name),
                 out=os.path.join(_build.HERE, name + ".so"), verbose=False)
    print("built", name)
