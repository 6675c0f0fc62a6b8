#!/bin/bash
# Profile the decode kernels on the GPU box (run through gpurun from the repo root).
#   tools/profile.sh <tag> [configs] [packets]
# 1. kernel trace + stats of the headline bench command (bench.py --configs c3)
#    and of the all-configs command: the average decode_kernel duration here
#    must agree with bench.py's HIP-event kernel_ms.
# 2. separate PMC passes (never combined with tracing): HBM bytes (FETCH_SIZE,
#    WRITE_SIZE) and SQ counters, one bench run per pass.
# Summaries: python tools/make_profiles.py <tag>  (writes profiles/)
set -o pipefail
TAG=${1:-r01}
CFGS=${2:-c3,c2,c4}
PK=${3:-16777216}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt_c3 -o kt -- python3 bench.py --configs c3 --no-cpu-baseline --steps 10 --warmup 2 > $OUT/kt_c3_bench.json || exit 1
B="bench.py --no-cpu-baseline --no-parity --configs $CFGS"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 $B --steps 5 --warmup 1 > $OUT/kt_bench.json || exit 1
P="--kernel-include-regex decode_kernel -f csv"
S="$B --no-probe --packets $PK --steps 2 --warmup 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE $P -d $OUT/fetch -o fetch -- python3 $S > /dev/null || exit 2
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE $P -d $OUT/write -o write -- python3 $S > /dev/null || exit 3
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS $P -d $OUT/sq1 -o sq1 -- python3 $S > /dev/null || exit 4
timeout -k 10 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE $P -d $OUT/sq2 -o sq2 -- python3 $S > /dev/null || exit 5
if [ -n "$EXTRA_PMC" ]; then
  timeout -k 10 400 rocprofv3 --pmc $EXTRA_PMC $P -d $OUT/extra -o extra -- python3 $S > /dev/null || exit 6
fi
echo done
