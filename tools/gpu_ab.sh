# GPU step for a kernel variant: parity tests through the in-tree library and
# through the variant (GPK_LIB_VARIANT), then an in-process A/B and optional
# per-wave timings of a diagnostic build.
# Usage: bash tools/gpu_ab.sh OUTDIR VARIANT "configs" [DIAGLIB] [DIAGCONFIGS]
set -o pipefail
OUT=gpurun_out/$1; V=$2; CFGS=${3:-c4,c3,c1,c2}; DIAG=${4:-}; DCFGS=${5:-c4,c3}
mkdir -p $OUT
export TMPDIR=/tmp
PT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT tests/test_gpu_parity.py tests/test_table_streams_gpu.py > $OUT/pytest_base.log 2>&1 || { tail -30 $OUT/pytest_base.log; exit 1; }
tail -2 $OUT/pytest_base.log
GPK_LIB_VARIANT=$V timeout -k 10 600 $PT tests/test_gpu_parity.py > $OUT/pytest_$V.log 2>&1 || { tail -30 $OUT/pytest_$V.log; exit 1; }
tail -2 $OUT/pytest_$V.log
timeout -k 10 400 python3 tools/ab_inproc.py --configs $CFGS --rounds 3 --steps 5 base $V > $OUT/ab.txt 2>&1 || { cat $OUT/ab.txt; exit 2; }
cat $OUT/ab.txt
if [ -n "$DIAG" ]; then
timeout -k 10 300 python3 tools/wave_times.py --lib $DIAG --configs $DCFGS --json $OUT/waves_$DIAG.json > $OUT/waves_$DIAG.txt 2>&1 || { cat $OUT/waves_$DIAG.txt; exit 3; }
cat $OUT/waves_$DIAG.txt
fi
