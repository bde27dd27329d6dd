"""Per-call durations (us) and start gaps of the kernels matching a substring,
in dispatch order, from a rocprofv3 results .db (tuning aid):
  python tools/db_seq.py run_results.db SUBSTRING [SUBSTRING ...]"""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                   "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
pats = sys.argv[2:]
prev_end = None
for name, st, en in rows:
    tag = next((p for p in pats if p in name), None)
    gap = (st - prev_end) / 1e3 if prev_end is not None else 0.0
    prev_end = en
    if tag:
        print(f"{tag:10s} {(en - st) / 1e3:9.1f} us  (gap before {gap:7.1f} us)")
