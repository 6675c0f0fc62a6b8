#!/usr/bin/env python3
"""How busy the host->device copy path is during C5's replays: from a
rocprofv3 --memory-copy-trace CSV, the union of HOST_TO_DEVICE copy
intervals inside each replay call (the replays are the long stretches of
slot copies; a gap of > 50 ms separates calls) and busy / span.

    python tools/copy_busy.py <rocprofv3 -d dir> [bench json]
"""
import csv
import glob
import json
import os
import sys


def main(d, bench=None):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(r)
    if not rows:
        print(json.dumps({"error": "no memory_copy_trace.csv under %s" % d}))
        return 1
    key_dir = next(k for k in rows[0] if k.lower() in ("direction", "operation"))
    h2d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r.get("Size", 0) or 0))
                 for r in rows if "HOST_TO_DEVICE" in r[key_dir].upper())
    d2h = [r for r in rows if "DEVICE_TO_HOST" in r[key_dir].upper()]
    # group into calls: the slot copies (>= 1 ms each; the trace has no sizes)
    # separated by > 50 ms
    big = [x for x in h2d if x[1] - x[0] >= 1_000_000]
    calls, cur = [], []
    for x in big:
        if cur and x[0] - cur[-1][1] > 50_000_000:
            calls.append(cur)
            cur = []
        cur.append(x)
    if cur:
        calls.append(cur)
    out = {"h2d_copies": len(h2d), "d2h_copies": len(d2h), "calls": []}
    for c in calls:
        t0, t1 = c[0][0], max(e for _, e, _ in c)
        inside = [x for x in h2d if x[0] >= t0 and x[1] <= t1]
        busy, last = 0, t0
        for s, e, _ in sorted(inside):
            if e > last:
                busy += e - max(s, last)
                last = e
        out["calls"].append(dict(span_s=round((t1 - t0) * 1e-9, 4), h2d_busy_s=round(busy * 1e-9, 4),
                                 busy_frac=round(busy / max(1, t1 - t0), 4), slot_copies=len(c),
                                 slot_copy_ms_mean=round(sum(e - s for s, e, _ in c) / len(c) * 1e-6, 3)))
    if bench and os.path.exists(bench):
        line = [x for x in open(bench).read().splitlines() if x.startswith("{")]
        if line:
            c5 = json.loads(line[-1]).get("c5") or {}
            out["bench_c5"] = {k: c5.get(k) for k in ("value", "GBps", "wall_s", "runs_wall_s", "htod_probe_GBps",
                                                        "htod_probe_1stream_GBps", "frac_of_htod_probe", "breakdown_s")}
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
