set -o pipefail
mkdir -p gpurun_out/diag1
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/ab_inproc.py --configs c4,c4x1,c4x3,c4x5,c1,c1x1,c2,c3 --rounds 3 --steps 5 base pbnull > gpurun_out/diag1/ab.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/diag1/kt_c1 -o kt -- python3 bench.py --configs c1 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/diag1/kt_c1_bench.json || exit 2
P="--kernel-include-regex decode_(sb_|)kernel -f csv"
S="bench.py --no-cpu-baseline --no-parity --no-probe --configs c1 --steps 2 --warmup 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE $P -d gpurun_out/diag1/fetch -o fetch -- python3 $S > /dev/null || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS $P -d gpurun_out/diag1/sq1 -o sq1 -- python3 $S > /dev/null || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE $P -d gpurun_out/diag1/sq2 -o sq2 -- python3 $S > /dev/null || exit 5
echo done
