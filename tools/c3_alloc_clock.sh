# effective clock per allocation (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) over tools/c3_alloc.py's five allocations
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex decode_(sb_|)kernel -f csv -d gpurun_out/c3clk -o clk -- python3 tools/c3_alloc.py > gpurun_out/c3clk/run.txt 2>&1 || exit 1
grep -h "ms$" gpurun_out/c3clk/run.txt
