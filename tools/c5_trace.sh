# C5 (pcapng replay, end to end) under rocprofv3 with the memory-copy and
# kernel traces: how busy the host->device copies keep the link during the
# replay (tools/copy_busy.py), beside the bench line's htod_probe_GBps.
# Usage: bash tools/c5_trace.sh OUTDIR [GiB]
set -o pipefail
OUT=gpurun_out/$1; G=${2:-10}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --configs c2 --packets 1048576 --steps 2 --warmup 1 --c5 $G --no-cpu-baseline --no-parity --no-probe"
timeout -k 10 400 python3 $B > $OUT/bench_plain.json 2> $OUT/bench_plain.err || { tail -20 $OUT/bench_plain.err; exit 2; }
timeout -k 10 400 rocprofv3 --memory-copy-trace --kernel-trace --stats -f csv -d $OUT/trace -o c5 -- python3 $B > $OUT/bench_traced.json 2> $OUT/bench_traced.err || { tail -20 $OUT/bench_traced.err; exit 3; }
python3 tools/copy_busy.py $OUT/trace $OUT/bench_traced.json > $OUT/copy_busy.json && cat $OUT/copy_busy.json
