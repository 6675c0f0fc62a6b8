# PMC per dispatch over tools/c3_alloc.py's five allocations (two passes, each its own process)
set -o pipefail
export TMPDIR=/tmp
P="--kernel-include-regex decode_(sb_|)kernel -f csv"
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL_sum $P -d gpurun_out/c3pmc/tlb -o tlb -- python3 tools/c3_alloc.py > gpurun_out/c3pmc/tlb.txt 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum $P -d gpurun_out/c3pmc/dram -o dram -- python3 tools/c3_alloc.py > gpurun_out/c3pmc/dram.txt 2>&1 || exit 2
grep -h "ms$" gpurun_out/c3pmc/tlb.txt gpurun_out/c3pmc/dram.txt
