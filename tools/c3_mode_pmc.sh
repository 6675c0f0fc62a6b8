#!/bin/bash
# C3 fast vs slow allocations under PMC: tools/c3_mode.py's
# allocations, one counter set per pass (each its own process, so its own
# allocations: every pass pairs its counters with its own timings), then a
# pass without profiling. Summary: python tools/c3_mode_summary.py gpurun_out/c3mode
set -o pipefail
OUT=gpurun_out/c3mode
mkdir -p $OUT
export TMPDIR=/tmp
P="--kernel-include-regex decode_(sb_|)kernel -f csv"
K=${1:-5}
timeout -k 10 240 python3 tools/c3_mode.py $K > $OUT/plain.txt 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum $P -d $OUT/ea -o ea -- python3 tools/c3_mode.py $K > $OUT/ea.txt 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL_sum TCP_TCC_READ_REQ_LATENCY_sum $P -d $OUT/tlb -o tlb -- python3 tools/c3_mode.py $K > $OUT/tlb.txt 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_LEVEL_sum $P -d $OUT/tcc -o tcc -- python3 tools/c3_mode.py $K > $OUT/tcc.txt 2>&1 || exit 4
cat $OUT/*.txt
