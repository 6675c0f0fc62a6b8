# Host-trap PC sampling of the decode kernel for one config (no counters, no tracing):
#   bash tools/pcsample.sh OUT CONFIG [interval_us]
# Output: gpurun_out/OUT/ (rocprofv3 pc-sampling CSV); summarise with tools/pcsample_summary.py
set -o pipefail
OUT=gpurun_out/$1
CFG=${2:-c4}
IV=${3:-100}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval $IV -f csv -d $OUT -o pcs -- python3 tools/ab_inproc.py --configs $CFG --rounds 1 --steps 3 base \
  > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
ls -R $OUT | head -20
