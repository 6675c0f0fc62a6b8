#!/usr/bin/env python3
"""Copy the judged summaries of a tools/profile.sh run into profiles/.

    python tools/make_profiles.py <tag> [configs] [packets]

profiles/<tag>_c3_kernel_stats.csv   rocprofv3 --kernel-trace --stats, headline bench command
profiles/<tag>_all_kernel_stats.csv  same, all configs
profiles/<tag>_bench.json            the bench.py lines of those two runs
profiles/<tag>_pmc.json              per-config counters (per decode dispatch)
profiles/hbm_traffic.json            HBM bytes per packet per config (bench.py roofline.traffic)

HBM bytes: FETCH_SIZE and WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE counts
half the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM
section), so fetch bytes = 2 * 1024 * FETCH_SIZE; write bytes = 1024 *
WRITE_SIZE. The x2 was checked on this kernel's own pattern: for C2 (every
byte read once) it gives exactly the algorithmic bytes.
"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_summary  # noqa: E402


def main():
    tag = sys.argv[1]
    labels = (sys.argv[2] if len(sys.argv) > 2 else "c3,c2,c4").split(",")
    packets = int(sys.argv[3]) if len(sys.argv) > 3 else 16777216
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt_c3", "kt_kernel_stats.csv"), os.path.join(dst, tag + "_c3_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, tag + "_all_kernel_stats.csv"))
    bench = {}
    for name in ("kt_c3_bench.json", "kt_bench.json"):
        lines = open(os.path.join(src, name)).read().strip().splitlines()
        bench[name] = json.loads(lines[-1])
    json.dump(bench, open(os.path.join(dst, tag + "_bench.json"), "w"), indent=1)
    pmc = pmc_summary.summarise(src, labels)
    json.dump(pmc, open(os.path.join(dst, tag + "_pmc.json"), "w"), indent=1, sort_keys=True)
    traffic = {"_note": "HBM bytes per packet from rocprofv3 PMC (profile %s, %d packets per dispatch): "
                        "fetch = 2*1024*FETCH_SIZE (gfx950 half-count), write = 1024*WRITE_SIZE" % (tag, packets)}
    for lab, g in pmc.items():
        f = 2 * 1024 * g["FETCH_SIZE"] / packets
        w = 1024 * g["WRITE_SIZE"] / packets
        traffic[lab] = {"fetch_bytes_per_packet": round(f, 2), "write_bytes_per_packet": round(w, 2),
                        "profile": tag}
    json.dump(traffic, open(os.path.join(dst, "hbm_traffic.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
