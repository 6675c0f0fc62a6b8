#!/usr/bin/env python3
"""Per-wave SQ counters of tools/pmc_ab.sh output directories:
    python tools/pmc_table.py gpurun_out/<dir> [...]
One line per <variant>_<config> subdirectory (sums over its dispatches)."""
import csv
import glob
import os
import sys
from collections import defaultdict

print("%-14s %6s %6s %5s %6s %8s %6s %8s %7s" % ("variant_cfg", "VALU", "SALU", "LDS", "LDSact", "conflict",
                                                  "ratio", "wavecyc", "B/pkt"))
for top in sys.argv[1:]:
    for d in sorted(glob.glob(os.path.join(top, "*"))):
        acc = defaultdict(float)
        for f in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
            for row in csv.DictReader(open(f)):
                acc[row["Counter_Name"]] += float(row["Counter_Value"])
        w = acc.get("SQ_WAVES", 0)
        if not w:
            continue
        act = acc.get("SQ_ACTIVE_INST_LDS", 0)
        print("%-14s %6.0f %6.0f %5.0f %6.0f %8.0f %6.3f %8.0f %7.1f" % (
            os.path.basename(d), acc["SQ_INSTS_VALU"] / w, acc["SQ_INSTS_SALU"] / w, acc["SQ_INSTS_LDS"] / w,
            act / w, acc.get("SQ_LDS_BANK_CONFLICT", 0) / w,
            acc.get("SQ_LDS_BANK_CONFLICT", 0) / act if act else 0, acc["SQ_WAVE_CYCLES"] / w,
            acc.get("FETCH_SIZE", 0) * 2048 / (w * 64)))
