#!/usr/bin/env python
"""Kernels around each optimizer launch of a rocprofv3 kernel trace: what runs (and what idles) between one step's
optimizer and the next step's first kernels.
    python tools/diag/step_gaps.py prof_kernel_trace.csv [n_boundaries=3]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ad = [i for i, r in enumerate(rows) if "adam_step" in r["Kernel_Name"]]
for i in ad[-nb - 2:-2]:
    t0 = int(rows[i]["End_Timestamp"])
    print(f"--- optimizer launch ending at {t0}")
    for r in rows[max(0, i - 3):i + 8]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f'{s/1e3:9.1f} {e/1e3:9.1f} q{r["Queue_Id"]} {r["Kernel_Name"][:70]}')
