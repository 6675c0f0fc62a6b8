#!/bin/bash
# PMC passes over C4's memory skeleton in four write forms (tools/skeleton_pmc.py):
# where the stores' time goes (DESIGN.md §5 "What the writes cost"). Output: $1/<form>/<pass>.
OUT=${1:-gpurun_out/skel_pmc}
P="--kernel-include-regex probe_skeleton -f csv"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
for f in writes nowrite l2ring ring; do
  A="tools/skeleton_pmc.py --config c4 --form $f"
  mkdir -p $OUT/$f
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum $P -d $OUT/$f/tcc -o tcc -- python3 $A > $OUT/$f/tcc.txt 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_DRAM_sum $P -d $OUT/$f/req -o req -- python3 $A > $OUT/$f/req.txt 2>&1 || exit 4
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY $P -d $OUT/$f/sq -o sq -- python3 $A > $OUT/$f/sq.txt 2>&1 || exit 5
done
