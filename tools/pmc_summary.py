#!/usr/bin/env python
"""Average PMC counters per kernel over the rocprofv3 csv passes under a directory.

    python tools/pmc_summary.py gpurun_out/<tag>
"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("kernel_name")
                name = r.get("Counter_Name") or r.get("Counter-Name")
                v = r.get("Counter_Value") or r.get("Counter-Value")
                disp = r.get("Dispatch_Id") or r.get("Dispatch-Id") or "0"
                if k is None or name is None or v is None:
                    continue
                vals[k[:90]][name].append((disp, float(v)))
    for k, cs in sorted(vals.items()):
        print(k)
        for name, lst in sorted(cs.items()):
            # counters are reported per dimension instance: sum within a dispatch, average over dispatches
            per = collections.defaultdict(float)
            for d, v in lst:
                per[d] += v
            avg = sum(per.values()) / max(1, len(per))
            print(f"    {name:32s} {avg:16.1f}")


if __name__ == "__main__":
    main()
