#!/bin/bash
# The round's closing GPU check (run through gpurun from the repo root): the whole
# -m gpu suite, then smoke(), as the driver runs them at round end.
#   bash tools/closing_check.sh TAG   -> gpurun_out/TAG/gputest.log
set -o pipefail
OUT=gpurun_out/${1:?tag}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1050 python3 -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
tail -3 $OUT/gputest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" >> $OUT/gputest.log 2>&1 || { tail -20 $OUT/gputest.log; exit 2; }
tail -1 $OUT/gputest.log
