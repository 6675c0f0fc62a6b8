# GPU step: parity tests of the decode path, then an in-process A/B of the
# given variants. Usage: bash tools/gpu_check.sh OUTDIR "variants" "configs" [pytest selection]
set -o pipefail
OUT=gpurun_out/$1
VARS=${2:-base}
CFGS=${3:-c4,c1,c3,c2}
SEL=${4:-tests/test_gpu_parity.py tests/test_table_streams_gpu.py}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$SEL" != "none" ]; then
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $SEL > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
fi
if [ "$VARS" != "none" ]; then
timeout -k 10 400 python3 tools/ab_inproc.py --configs $CFGS --rounds 3 --steps 5 $VARS > $OUT/ab.txt 2>&1 || { cat $OUT/ab.txt; exit 2; }
cat $OUT/ab.txt
fi
