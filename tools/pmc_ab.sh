# PMC passes per (variant, config) through the in-process harness (one
# variant library loaded, 2 rounds x 2 steps = 4 dispatches per pass).
# Usage: bash tools/pmc_ab.sh OUTDIR "variants" "configs"
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
P="--kernel-include-regex decode_(sb_|)kernel -f csv"
for v in $2; do
  for c in $(echo $3 | tr , ' '); do
    A="tools/ab_inproc.py --configs $c --rounds 1 --steps 2 $v"
    timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM $P -d $OUT/${v}_${c}/sq1 -o sq1 -- python3 $A > /dev/null || exit 3
    timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $P -d $OUT/${v}_${c}/sq2 -o sq2 -- python3 $A > /dev/null || exit 4
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE $P -d $OUT/${v}_${c}/fetch -o fetch -- python3 $A > /dev/null || exit 5
    echo "pmc $v $c done"
  done
done
