"""Summary of tools/c3_mode_pmc.sh: per allocation (6 decode dispatches each,
the last 4 used), the kernel time from the counter records' timestamps and the
mean of each counter per dispatch, with derived ratios: EA read latency
(TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ, cycles), credit stalls per read request,
UTCL1 translation misses per request, TCP->TCC read latency per ... and the
L2 hit rate.

    python tools/c3_mode_summary.py gpurun_out/c3mode
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(path):
    disp = defaultdict(dict)
    for row in csv.DictReader(open(path)):
        d = disp[int(row["Dispatch_Id"])]
        d[row["Counter_Name"]] = float(row["Counter_Value"])
        d["ms"] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
    ids = sorted(disp)
    return [disp[i] for i in ids]


def main():
    root = sys.argv[1]
    out = []
    for sub in ("ea", "tlb", "tcc"):
        f = glob.glob(os.path.join(root, sub, "*counter_collection.csv"))
        if not f:
            continue
        rows = load(f[0])
        per = [rows[k:k + 6][2:] for k in range(0, len(rows), 6)]
        out.append("# pass %s (%d dispatches, %d allocations)" % (sub, len(rows), len(per)))
        base = None
        for a, ds in enumerate(per):
            if not ds:
                continue
            mean = {k: sum(d.get(k, 0) for d in ds) / len(ds) for k in ds[0]}
            s = "alloc %d: %.3f ms" % (a, mean["ms"])
            if "TCC_EA0_RDREQ_sum" in mean:
                # Little's law: requests in flight at the memory side ~ LEVEL_sum / kernel time
                inflight = mean["TCC_EA0_RDREQ_LEVEL_sum"] / mean["ms"]
                base = base or inflight
                s += "  EA read latency %.1f cycles  reads in flight (rel. alloc 0) %.3f  credit stall/req %.4f" \
                     "  rdreq %.4g" % (mean["TCC_EA0_RDREQ_LEVEL_sum"] / mean["TCC_EA0_RDREQ_sum"], inflight / base,
                                       mean["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / mean["TCC_EA0_RDREQ_sum"],
                                       mean["TCC_EA0_RDREQ_sum"])
            if "TCP_UTCL1_TRANSLATION_MISS_sum" in mean:
                m, h = mean["TCP_UTCL1_TRANSLATION_MISS_sum"], mean["TCP_UTCL1_TRANSLATION_HIT_sum"]
                s += "  UTCL1 miss %.4g hit %.4g (miss rate %.5f)  TCP->TCC read latency sum %.4g" % (
                    m, h, m / max(1.0, m + h), mean.get("TCP_TCC_READ_REQ_LATENCY_sum", 0))
            if "TCC_HIT_sum" in mean:
                hh, mm = mean["TCC_HIT_sum"], mean["TCC_MISS_sum"]
                s += "  L2 hit %.4f  tag stall %.4g  EA write level %.4g" % (
                    hh / max(1.0, hh + mm), mean["TCC_TAG_STALL_sum"], mean.get("TCC_EA0_WRREQ_LEVEL_sum", 0))
            out.append(s)
    print("\n".join(out))


if __name__ == "__main__":
    main()
