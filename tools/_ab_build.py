"""Build the A/B libraries next to libvsig.so (same sources, extra defines)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vector_amd import _build  # noqa: E402

VARIANTS = {
    "libvsig_x32": ("VSIG_XCORR_BIG_FROM=2049",),
    "libvsig_noswz": ("VSIG_NO_SWZ",),
    "libvsig_fold": ("VSIG_FIR_DEC_FOLD",),
    "libvsig_firko": ("VSIG_FIR_KO",),
    "libvsig_nox4": ("VSIG_NO_X4",),
    "libvsig_nokeyed": ("VSIG_NO_KEYED",),
    "libvsig_xilv": ("VSIG_XCORR_ILV",),
    "libvsig_pfb128": ("VSIG_PFB_FPG=128",),
    "libvsig_pfb256": ("VSIG_PFB_FPG=256",),
    "libvsig_pfb512": ("VSIG_PFB_FPG=512",),
    "libvsig_ilv50": ("VSIG_ILV_S=5", "VSIG_ILV_U=0"),
    "libvsig_ilv61": ("VSIG_ILV_S=6", "VSIG_ILV_U=1"),
    "libvsig_pfbfwd": ("VSIG_PFB_FWD_ONLY",),
    "libvsig_pfbv3": ("VSIG_PFB_VAR64=3",),
    "libvsig_nobufld": ("VSIG_NO_BUFLD",),
    "libvsig_unphased": ("VSIG_FFT_UNPHASED",),
    "libvsig_rg1024": ("VSIG_REFINE_G1=1024", "VSIG_REFINE_G2=256"),
    "libvsig_nol1tw": ("VSIG_NO_L1TW",),
    "libvsig_rko1": ("VSIG_REFINE_KO=1",),
    "libvsig_rko2": ("VSIG_REFINE_KO=2",),
    "libvsig_rko3": ("VSIG_REFINE_KO=3",),
    "libvsig_rko4": ("VSIG_REFINE_KO=4",),
    "libvsig_rko5": ("VSIG_REFINE_KO=5",),
    "libvsig_noxpad": ("VSIG_NO_XPAD",),
    "libvsig_nodv": ("VSIG_NO_DVSPLIT",),
    "libvsig_nosegpf": ("VSIG_NO_SEGPF",),
    "libvsig_segpf32": ("VSIG_SEGPF_DIST=32",),
    "libvsig_segpf128": ("VSIG_SEGPF_DIST=128",),
    "libvsig_segpf0": ("VSIG_SEGPF_POS=0",),
    "libvsig_segpf1": ("VSIG_SEGPF_POS=1",),
    "libvsig_segpf96": ("VSIG_SEGPF_DIST=96",),
    "libvsig_segpf192": ("VSIG_SEGPF_DIST=192",),
    "libvsig_segpf256": ("VSIG_SEGPF_DIST=256",),
    "libvsig_koseg": ("VSIG_KO_SEGLD",),
    "libvsig_kotmp": ("VSIG_KO_TMPLD",),
    "libvsig_koboth": ("VSIG_KO_SEGLD", "VSIG_KO_TMPLD"),
    "libvsig_kolkey": ("VSIG_KO_LKEY",),
    "libvsig_kopart": ("VSIG_KO_PART",),
    "libvsig_kosums": ("VSIG_KO_SUMS",),
    "libvsig_koxepi": ("VSIG_KO_XEPI",),
    "libvsig_rg64": ("VSIG_REFINE_GRID=64",),
    "libvsig_rg128": ("VSIG_REFINE_GRID=128",),
    "libvsig_konobar": ("VSIG_KO_NOBAR",),
    "libvsig_konolds": ("VSIG_KO_NOLDS",),
    "libvsig_koxepi": ("VSIG_KO_XEPI",),
    "libvsig_koxsqrt": ("VSIG_KO_XSQRT",),
    "libvsig_xw": ("VSIG_XCORR_W",),
    "libvsig_nodskip": ("VSIG_NO_DSKIP",),
    "libvsig_fin256": ("VSIG_FIN_CHUNK=256",),
    "libvsig_fin512": ("VSIG_FIN_CHUNK=512",),
    "libvsig_fin1024": ("VSIG_FIN_CHUNK=1024",),
}
for name in (sys.argv[1:] or VARIANTS):
    _build.build(defines=VARIANTS[name], out=os.path.join(_build.HERE, name + ".so"), verbose=False)
    print("built", name)
