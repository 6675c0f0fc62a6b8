#!/usr/bin/env python3
"""Copy the judged summaries of a tools/profile.sh run into profiles/.

    python tools/make_profiles.py <tag> [configs]

profiles/<tag>_c3_kernel_stats.csv   rocprofv3 --kernel-trace --stats, headline bench command
profiles/<tag>_all_kernel_stats.csv  same, all configs
profiles/<tag>_bench.json            the bench.py lines of those two runs
profiles/<tag>_pmc.json              per config: counters per decode dispatch (mean of 4),
                                     per wave and per packet
profiles/hbm_traffic.json            HBM bytes per packet per config (bench.py roofline.traffic)

HBM bytes: FETCH_SIZE and WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE counts
half the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM
section), so fetch bytes = 2 * 1024 * FETCH_SIZE; write bytes = 1024 *
WRITE_SIZE. The x2 was checked on this kernel's own pattern: for C2 (every
byte read once) it gives exactly the algorithmic bytes. FETCH_SIZE also
counts Infinity Cache hits (same section): re-reads of lines still on die
show up as fetch bytes above the algorithmic ones.
"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
import pmc_summary  # noqa: E402


def packets_of(cfg):
    import bench
    # c4f: C4's batch with the fused fields; c2n etc.: the config's batch through the narrow record
    c = bench.CONFIGS[cfg[:-1] if cfg.endswith("f") or cfg.endswith("n") else cfg]
    return c.get("packets", 64 * 2**20)


def main():
    tag = sys.argv[1]
    labels = (sys.argv[2] if len(sys.argv) > 2 else "c3,c2,c4,c1").split(",")
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
    pmc, traffic = {}, {"_note": "HBM bytes per packet from rocprofv3 PMC (profile %s, full-size batches, mean of "
                                 "4 dispatches): fetch = 2*1024*FETCH_SIZE (gfx950 half-count), write = "
                                 "1024*WRITE_SIZE" % tag}
    for lab in labels:
        g = pmc_summary.summarise(os.path.join(src, lab), [lab])[lab]
        n = packets_of(lab)
        waves = g.get("SQ_WAVES", 0) or 1
        for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT"):
            if c in g:
                g[c + "_per_wave"] = g[c] / waves
        if g.get("SQ_ACTIVE_INST_LDS"):
            g["lds_conflict_ratio"] = g["SQ_LDS_BANK_CONFLICT"] / g["SQ_ACTIVE_INST_LDS"]
        f = 2 * 1024 * g["FETCH_SIZE"] / n
        w = 1024 * g["WRITE_SIZE"] / n
        g["packets_per_dispatch"] = n
        g["fetch_bytes_per_packet"] = f
        g["write_bytes_per_packet"] = w
        pmc[lab] = g
        traffic[lab] = {"fetch_bytes_per_packet": round(f, 2), "write_bytes_per_packet": round(w, 2), "profile": tag,
                        "kernel": g.get("kernel", "")}
    json.dump(pmc, open(os.path.join(dst, tag + "_pmc.json"), "w"), indent=1, sort_keys=True)
    json.dump(traffic, open(os.path.join(dst, "hbm_traffic.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
