set -o pipefail
OUT=gpurun_out/pmc_r04l
mkdir -p $OUT
export TMPDIR=/tmp
P="--kernel-include-regex decode_(sb_|)kernel -f csv"
for c in c4 c3 c1; do
  A="tools/ab_inproc.py --configs $c --rounds 1 --steps 2 base"
  timeout -k 10 300 rocprofv3 --pmc SQ_LEVEL_WAVES SQ_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_IFETCH $P -d $OUT/$c/a -o a -- python3 $A > /dev/null || exit 3
  timeout -k 10 300 rocprofv3 --pmc SQ_IFETCH_LEVEL SQ_LDS_UNALIGNED_STALL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC $P -d $OUT/$c/b -o b -- python3 $A > /dev/null || exit 4
  echo "pmc $c done"
done
