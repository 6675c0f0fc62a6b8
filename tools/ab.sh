#!/bin/bash
# A/B kernel variants on the GPU box (run through gpurun from the repo root):
#   tools/ab.sh <out-tag> <configs> <variant>...   ("base" = gopacket_amd/libgpk.so)
# Each variant: one bench run (no CPU baseline, no parity sample) -> JSON line.
set -o pipefail
TAG=$1; CFGS=$2; shift 2
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for V in "$@"; do
  EXTRA=""
  case $V in
    base) unset GPK_LIB_VARIANT ;;
    global) unset GPK_LIB_VARIANT; EXTRA="--tables global" ;;
    *) export GPK_LIB_VARIANT=$V ;;
  esac
  timeout -k 10 300 python3 bench.py $EXTRA --no-cpu-baseline --no-parity --configs $CFGS --steps 10 --warmup 2 \
    > $OUT/$V.json 2> $OUT/$V.err || { echo "variant $V failed"; exit 1; }
  python3 - "$OUT/$V.json" "$V" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
line = "%-10s %s %.3f ms %.1f GB/s probe %s" % (sys.argv[2], "head", r["kernel_ms"], r["achieved"], r["probe_read_GBps"])
for k, v in d["configs"].items():
    line += " | %s %.3f ms %.1f GB/s probe %s" % (k, v["kernel_ms"], v["achieved_GBps"], v["probe_read_GBps"])
print(line)
PY
done
