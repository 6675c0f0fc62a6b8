#!/bin/bash
# Profile the decode kernels on the GPU box (run through gpurun from the repo root).
#   tools/profile.sh <tag> [configs]
# 1. rocprofv3 --kernel-trace --stats of the headline bench command (C3) and
#    of the all-configs command: the average decode_kernel duration here must
#    agree with bench.py's HIP-event kernel_ms.
# 2. separate PMC passes per config (never combined with tracing), through the
#    in-process harness (tools/ab_inproc.py, 2 rounds x 2 steps = 4 dispatches
#    of the full-size batch): SQ instruction/cycle counters, FETCH_SIZE,
#    WRITE_SIZE.
# Summaries: python tools/make_profiles.py <tag> [configs]  (writes profiles/)
set -o pipefail
TAG=${1:-r03}
CFGS=${2:-c3,c2,c4,c1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt_c3 -o kt -- python3 bench.py --configs c3 --no-cpu-baseline --c5 0 --no-fields --no-narrow --steps 10 --warmup 2 > $OUT/kt_c3_bench.json || exit 1
BCFGS=$(echo $CFGS | tr , '\n' | grep -v '^c4f$' | grep -v 'n$' | paste -sd, -)
B="bench.py --no-cpu-baseline --no-parity --no-narrow --c5 0 --configs $BCFGS"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 $B --steps 5 --warmup 1 > $OUT/kt_bench.json || exit 1
P="--kernel-include-regex decode_(sb_|)kernel -f csv"
for c in $(echo $CFGS | tr , ' '); do
  # c4f: the fused decode + fields launch on C4's batch (gpk_decode_batch_fields)
  # c2n / c3n / ...: that config's batch through the narrow record (gpk_decode_batch_narrow)
  if [ "$c" = "c4f" ]; then A="tools/ab_inproc.py --configs c4 --fields --rounds 1 --steps 2 base";
  elif [ "${c: -1}" = "n" ]; then A="tools/ab_inproc.py --configs ${c%n} --rounds 1 --steps 2 base@narrow";
  else A="tools/ab_inproc.py --configs $c --rounds 1 --steps 2 base"; fi
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE $P -d $OUT/$c/fetch -o fetch -- python3 $A > /dev/null || exit 2
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE $P -d $OUT/$c/write -o write -- python3 $A > /dev/null || exit 3
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS $P -d $OUT/$c/sq1 -o sq1 -- python3 $A > /dev/null || exit 4
  timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE $P -d $OUT/$c/sq2 -o sq2 -- python3 $A > /dev/null || exit 5
  echo "pmc $c done"
done
echo done
