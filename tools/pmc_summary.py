"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per vsig kernel.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so reads are doubled (x2 correction); WRITE_SIZE is
taken as is.  Usage:
  python tools/pmc_summary.py gpurun_out/pmc1 profiles/pmc_r01.json KEYSPEC
where KEYSPEC is the bench config suffix, e.g.
  n=268435456:ntaps=255:decim=1:nfft=8192:L=4096
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

FAMILY = {"fir_os_kernel": "fir", "fir_dec_kernel": "fir", "fir_poly_kernel": "fir", "psd_pair_kernel": "psd",
          "psd_split_kernel": "psd", "xcorr_os_kernel": "xcorr", "xcorr_half_kernel": "xcorr",
          "pfb_kernel": "pfb", "peak_reduce": "peak", "partial_finalize": "finalize",
          "refine_finalize_select": "finalize", "refine_fused": "refine", "refine_numpy": "refine",
          "refine_stage1": "refine1", "refine_stage2": "refine2", "bf_col_kernel": "bigfft_col",
          "bf_row_kernel": "bigfft_row"}


def family(name):
    for k, v in FAMILY.items():
        if k in name:
            return v
    return None


def main(src, dst, keyspec):
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(src, "p*", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            fam = family(row["Kernel_Name"])
            if fam is None:
                continue
            acc[fam][row["Counter_Name"]].append(float(row["Counter_Value"]))
            # rocprofv3's VGPR_Count scales the descriptor's VGPR granule field by 4 on
            # gfx950, whose granule is 8: it reads half the allocation (123 VGPRs ->
            # 16 granules -> 64); vgpr = the allocation, vgpr_rocprof = as reported
            meta[fam] = dict(kernel=row["Kernel_Name"].split("(")[0], vgpr=2 * int(row["VGPR_Count"]),
                             vgpr_rocprof=int(row["VGPR_Count"]),
                             lds=int(row["LDS_Block_Size"]), scratch=int(row["Scratch_Size"]),
                             wg=int(row["Workgroup_Size"]), grid=int(row["Grid_Size"]))
    out = {"config_key_suffix": keyspec, "kernels": {}}
    for fam, ctrs in acc.items():
        med = {k: sorted(v)[len(v) // 2] for k, v in ctrs.items()}
        d = dict(meta[fam])
        d["counters"] = med
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            rd = med["FETCH_SIZE"] * 1024 * 2      # gfx950 x2 read correction
            wr = med["WRITE_SIZE"] * 1024
            d["hbm_read_bytes"] = rd
            d["hbm_write_bytes"] = wr
            d["hbm_bytes_per_launch"] = rd + wr
        if "TCC_HIT_sum" in med:
            d["l2_hit_rate"] = med["TCC_HIT_sum"] / max(1.0, med["TCC_HIT_sum"] + med["TCC_MISS_sum"])
        if "SQ_WAVE_CYCLES" in med and med["SQ_WAVE_CYCLES"]:
            wc = med["SQ_WAVE_CYCLES"]
            d["frac_wait_any"] = med.get("SQ_WAIT_ANY", 0) / wc
            d["frac_wait_inst"] = med.get("SQ_WAIT_INST_ANY", 0) / wc
            d["frac_active"] = med.get("SQ_ACTIVE_INST_ANY", 0) / wc
        if "SQ_INSTS_VALU" in med and med.get("GRBM_GUI_ACTIVE"):
            # VALU issue utilisation: wave64 VALU instructions x 4 issue cycles
            # (MI355X_MICROARCH.md issue-cost table) over 256 CUs x 4 SIMDs x the
            # launch's busy cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs)
            d["valu_issue_frac"] = med["SQ_INSTS_VALU"] * 4 / (1024 * med["GRBM_GUI_ACTIVE"] / 8)
        out["kernels"][fam] = d
    json.dump(out, open(dst, "w"), indent=1)
    # per-kernel files bench.py looks up (config_key match)
    for fam, d in out["kernels"].items():
        if "hbm_bytes_per_launch" in d:
            rec = {"config_key": f"{fam}:{keyspec}", "hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
                   "source": f"{os.path.basename(dst)} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE)"}
            if "valu_issue_frac" in d:
                rec["valu_issue_frac"] = round(d["valu_issue_frac"], 4)
            out["kernels"][fam]["bench_record"] = rec
            tag = os.path.basename(dst)[len("pmc_"):] if os.path.basename(dst).startswith("pmc_") \
                else os.path.basename(dst)
            json.dump(rec, open(os.path.join(os.path.dirname(dst), f"pmc_{fam}_{tag}"), "w"), indent=1)
    json.dump(out, open(dst, "w"), indent=1)
    for fam, d in out["kernels"].items():
        print(fam, {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items() if k != "counters"})


if __name__ == "__main__":
    main(*sys.argv[1:4])
