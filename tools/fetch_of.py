"""Mean HBM read bytes per dispatch (FETCH_SIZE x 2 x 1024, the gfx950
correction of MI355X_MICROARCH.md) of the kernels whose name contains a
substring, from a rocprofv3 --pmc FETCH_SIZE csv directory.
  python tools/fetch_of.py DIR SUBSTRING"""
import csv
import glob
import os
import sys

d, sub = sys.argv[1], sys.argv[2]
vals = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if sub in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
                vals.setdefault(r["Dispatch_Id"], 0.0)
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
v = list(vals.values())
print(f"{sub}: {len(v)} dispatches, mean {sum(v) / max(len(v), 1) * 2 * 1024 / 1e9:.3f} GB read per dispatch")
