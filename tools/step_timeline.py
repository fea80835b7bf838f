"""Print one training step's kernel timeline from a rocprofv3 kernel trace (the Nth-from-last step,
delimited by the optimizer kernel), with gaps between consecutive kernels.
usage: python tools/step_timeline.py prof_kernel_trace.csv [n_from_last=3]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nth = int(sys.argv[2]) if len(sys.argv) > 2 else 3
def is_opt(r):
    return "adam_step" in r["Kernel_Name"] or "adam_fused" in r["Kernel_Name"]


# a step ends with its optimizer group (one launch, or several when ranges are updated separately -- e.g. the
# unzeroed out.weight range at a large vocabulary): the LAST launch of each consecutive group delimits steps.  A step
# whose optimizer updates some ranges early on a side stream (BERT at 1M items: out.weight beside the encoder
# backward) ends with rs_seed_advance instead: when that kernel is in the trace it delimits the steps.
if any("seed_advance" in r["Kernel_Name"] for r in rows):
    ad = [i for i, r in enumerate(rows) if "seed_advance" in r["Kernel_Name"]]
else:
    ad = [i for i, r in enumerate(rows) if is_opt(r) and (i + 1 == len(rows) or not is_opt(rows[i + 1]))]
# steps of the timed graph replays only: bench.py's event-timed leg runs eager steps with timing events and a
# torch spin kernel around the dominant launch after the timed ones -- skip every step holding a non-HIP-graph kernel
# of that kind (torch's spin / elementwise kernels)
clean = [k for k in range(1, len(ad)) if not any(
    "spin_kernel" in r["Kernel_Name"] or "at::" in r["Kernel_Name"] for r in rows[ad[k - 1] + 1:ad[k] + 1])]
k = clean[-nth] if len(clean) >= nth else clean[-1]
hi, lo = ad[k], ad[k - 1]
sel = rows[lo + 1:hi + 1]
t0 = int(sel[0]["Start_Timestamp"])
prev = None
busy = 0
for r in sel:
    s = int(r["Start_Timestamp"]) - t0
    e = int(r["End_Timestamp"]) - t0
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f'{s/1e3:8.1f} {e/1e3:8.1f} dur {(e-s)/1e3:6.1f} gap {gap:6.1f} q{r["Queue_Id"]} wg {int(r["Grid_Size_X"])*int(r["Grid_Size_Y"])//int(r["Workgroup_Size_X"]):6d} {r["Kernel_Name"][:60]}')
    prev = max(prev or 0, e)
    busy += e - s
print(f"step span {(int(sel[-1]['End_Timestamp'])-t0)/1e3:.1f} us, kernel time {busy/1e3:.1f} us")
# the true step period: optimizer end to optimizer end over consecutive clean steps (includes the gap before each
# step's first kernel, which the span above does not)
per = sorted((int(rows[ad[k]]["End_Timestamp"]) - int(rows[ad[k - 1]]["End_Timestamp"])) / 1e3
             for k in clean if k - 1 in clean or k - 1 >= 1)
if per:
    print(f"optimizer-to-optimizer period over {len(per)} steps: median {per[len(per) // 2]:.1f} us, "
          f"min {per[0]:.1f}, max {per[-1]:.1f}")
