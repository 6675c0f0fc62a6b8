#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs per kernel dispatch group.

   python tools/pmc_summary.py <prof dir> [labels]

Dispatches of the decode kernels are listed in launch order; `labels`
(comma-separated, e.g. c3,c2,c4) names consecutive groups of equal size
(bench.py runs its configs in that order with the same step count)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    rows = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    meta = {}
    for f in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
        tag = f.split(os.sep)[-2]
        for row in csv.DictReader(open(f)):
            key = (tag, int(row["Dispatch_Id"]))
            rows[key][row["Counter_Name"]] += float(row["Counter_Value"])
            meta[key] = (row["Kernel_Name"], int(row["Grid_Size"]))
    return rows, meta


def summarise(d, labels):
    rows, meta = load(d)
    by_tag = defaultdict(list)
    for key in sorted(rows):
        if "decode_kernel" in meta[key][0] or "decode_sb_kernel" in meta[key][0]:
            by_tag[key[0]].append(key)
    out = defaultdict(lambda: defaultdict(list))
    for tag, keys in by_tag.items():
        per = max(1, len(keys) // max(1, len(labels)))
        for i, key in enumerate(keys):
            lab = labels[min(i // per, len(labels) - 1)] if labels else meta[key][0]
            for c, v in rows[key].items():
                out[lab][c].append(v)
            out[lab]["kernel"] = meta[key][0]
            out[lab]["grid"] = meta[key][1]
    res = {}
    for lab, m in out.items():
        res[lab] = {c: (sum(v) / len(v) if isinstance(v, list) else v) for c, v in m.items()}
        g = res[lab]
        waves = g.get("SQ_WAVES", 0) or 1
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
            if c in g:
                g[c + "_per_wave"] = g[c] / waves
    return res


if __name__ == "__main__":
    labels = sys.argv[2].split(",") if len(sys.argv) > 2 else []
    print(json.dumps(summarise(sys.argv[1], labels), indent=1))
