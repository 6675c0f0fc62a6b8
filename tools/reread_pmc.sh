# PMC passes of the re-read probe (tools/reread_probe.py), one process per mode.
# Usage: bash tools/reread_pmc.sh OUTDIR [pkt]
set -o pipefail
OUT=gpurun_out/$1; PKT=${2:-1500}
mkdir -p $OUT
export TMPDIR=/tmp
P="--kernel-include-regex probe_reread -f csv"
for m in 0 1 2 3; do
  A="tools/reread_probe.py --gib 32 --rounds 1 --steps 1 --modes $m --pkts $PKT"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE $P -d $OUT/m$m/fetch -o fetch -- python3 $A > /dev/null || exit 3
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum $P -d $OUT/m$m/hit -o hit -- python3 $A > /dev/null || exit 4
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum $P -d $OUT/m$m/ea -o ea -- python3 $A > /dev/null || exit 5
  echo "pmc mode $m done"
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, json
out = {}
for m in (0, 1, 2, 3):
    vals = {}
    for f in glob.glob(os.path.join(sys.argv[1], "m%d" % m, "*", "*", "*_counter_collection.csv")) + \
             glob.glob(os.path.join(sys.argv[1], "m%d" % m, "*", "*_counter_collection.csv")):
        per = {}
        for row in csv.DictReader(open(f)):
            per.setdefault(row["Dispatch_Id"], {}).setdefault(row["Counter_Name"], 0.0)
            per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
        for d in per.values():
            for k, v in d.items():
                vals[k] = v  # one dispatch per pass
    out["mode%d" % m] = vals
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(sys.argv[1], "reread_pmc.json"), "w"), indent=1)
PY
