#!/usr/bin/env python
"""profiles/traffic.json from rocprofv3 PMC passes (tools/gpu.sh pmc / traffic output directory).

    python tools/make_traffic.py gpurun_out/<tag> CONFIG [profiles/traffic.json]

HBM traffic per launch = FETCH_SIZE x 2 + WRITE_SIZE (KiB -> bytes), the MI355X_MICROARCH.md
correction for gfx950 (FETCH_SIZE counts half of the bytes of wide coalesced reads; WRITE_SIZE
is exact for 16-B-per-lane stores).  The bench's dominant "kernel" for SAS is rs_attn_bwd, two
launches (dQ+delta, dK/dV): its entry is the sum of the two.
"""
import collections
import csv
import glob
import json
import os
import sys

KEYS = {"rs_attn_bwd (attn_bwd_lds: dQ + dK/dV workgroups)": ["attn_bwd_lds_kernel"],
        "rs_wgrad_grouped (wgrad_group_kernel + reduce_cols_kernel)": ["wgrad_group_kernel", "reduce_cols_kernel"],
        "rs_wgrad_grouped (wgrad_group256_kernel + reduce_cols_kernel)": ["wgrad_group256_kernel",
                                                                         "reduce_cols_kernel"],
        "rs_vocab_head_fwd (E-tile-stationary logits + online-softmax partials)": ["pp_kernel<256, false>",
                                                                                  "ce_tiles_kernel"]}


def per_dispatch(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(dict))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k, name, v = r.get("Kernel_Name"), r.get("Counter_Name"), r.get("Counter_Value")
                disp = r.get("Dispatch_Id", "0")
                if k and name in ("FETCH_SIZE", "WRITE_SIZE"):
                    d = vals[k][name]
                    d[disp] = d.get(disp, 0.0) + float(v)
    out = {}
    for k, cs in vals.items():
        f = cs.get("FETCH_SIZE", {})
        w = cs.get("WRITE_SIZE", {})
        if not f or not w:
            continue
        fb = 2 * 1024 * sum(f.values()) / len(f)
        wb = 1024 * sum(w.values()) / len(w)
        out[k] = {"fetch_bytes": fb, "write_bytes": wb, "bytes": fb + wb}
    return out


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                              "traffic.json")
    k = per_dispatch(root)
    res = {}
    for key, parts in KEYS.items():
        hits = [v for name, v in k.items() for p in parts if p in name]
        if len(hits) == len(parts):
            res[key] = int(sum(h["bytes"] for h in hits))
    res["_per_kernel"] = {n[:80]: {a: int(b) for a, b in v.items()} for n, v in k.items()}
    res["_method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over tools/kbench.py at the "
                      "bench shapes; bytes/launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 correction)")
    allres = json.load(open(dst)) if os.path.exists(dst) else {}
    allres[cfg] = res
    json.dump(allres, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
