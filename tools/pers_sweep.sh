# Persistent-kernel sweep: tiles per wave (GPK_PERS_TILES) for the given variants, in-process A/B
# against the one-tile kernel, then per-wave timings of the diagnostic build at one setting.
# Usage: bash tools/pers_sweep.sh OUTDIR "variants" "tile counts" configs DIAGLIB DIAGTILES
set -o pipefail
OUT=gpurun_out/$1; VARS=$2; TS=${3:-"2 4 8"}; CFGS=${4:-c4,c3}; DIAG=${5:-}; DT=${6:-4}
mkdir -p $OUT
export TMPDIR=/tmp
for T in $TS; do
  echo "== GPK_PERS_TILES=$T"
  GPK_PERS_TILES=$T timeout -k 10 300 python3 tools/ab_inproc.py --configs $CFGS --rounds 3 --steps 5 base $VARS > $OUT/ab_t$T.txt 2>&1 || { cat $OUT/ab_t$T.txt; exit 2; }
  grep -v amdgpu.ids $OUT/ab_t$T.txt
done
if [ -n "$DIAG" ]; then
  GPK_PERS_TILES=$DT timeout -k 10 300 python3 tools/wave_times.py --lib $DIAG --configs $CFGS > $OUT/waves.txt 2>&1 || { cat $OUT/waves.txt; exit 3; }
  grep -v amdgpu.ids $OUT/waves.txt
fi
