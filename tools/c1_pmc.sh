# PMC A/B of the C1 kernels: the dword-aligned 5-chunk
# window (AL = 4, the default) against the 16-byte-aligned 6-chunk window
# (variant al16 = GPK_MID_W5=0), one pass per counter group.
# Usage: [SQ=1] bash tools/c1_pmc.sh OUTDIR "variants" [config]   (SQ=1: wave/instruction/LDS passes too)
set -o pipefail
OUT=gpurun_out/$1; VARS=${2:-"base al16"}; CFG=${3:-c1}
mkdir -p $OUT
export TMPDIR=/tmp
P="--kernel-include-regex decode_ -f csv"
for v in $VARS; do
  A="tools/ab_inproc.py --configs $CFG --rounds 1 --steps 2 $v"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE $P -d $OUT/$v/fetch -o fetch -- python3 $A > /dev/null || exit 3
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum $P -d $OUT/$v/hit -o hit -- python3 $A > /dev/null || exit 4
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum $P -d $OUT/$v/req -o req -- python3 $A > /dev/null || exit 5
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_BUBBLE_sum $P -d $OUT/$v/dram -o dram -- python3 $A > /dev/null || exit 6
  timeout -k 10 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum $P -d $OUT/$v/tcp -o tcp -- python3 $A > /dev/null || exit 7
  if [ -n "$SQ" ]; then
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS $P -d $OUT/$v/sq -o sq -- python3 $A > /dev/null || exit 8
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY $P -d $OUT/$v/lds -o lds -- python3 $A > /dev/null || exit 9
  fi
  echo "pmc $v done"
done
python3 - "$OUT" "$VARS" <<'PY'
import csv, glob, json, os, sys
out = {}
for v in sys.argv[2].split():
    vals, n = {}, {}
    for f in glob.glob(os.path.join(sys.argv[1], v, "*", "*", "*_counter_collection.csv")) + \
             glob.glob(os.path.join(sys.argv[1], v, "*", "*_counter_collection.csv")):
        per = {}
        for row in csv.DictReader(open(f)):
            per.setdefault(row["Dispatch_Id"], {}).setdefault(row["Counter_Name"], 0.0)
            per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
            n[row["Counter_Name"]] = row["Kernel_Name"]
        for d in per.values():  # the last dispatch of each pass
            vals.update(d)
    out[v] = dict(vals, kernel=sorted(set(n.values())))
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(sys.argv[1], "pmc.json"), "w"), indent=1)
PY
