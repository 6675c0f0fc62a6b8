# C1 timing: the bench line alone, after C4, and the in-process harness (same box)
set -o pipefail
export TMPDIR=/tmp
for cf in c1 c4,c1; do
  timeout -k 10 300 python3 bench.py --configs $cf --no-cpu-baseline --no-full-parity --no-parity --c5 0 --steps 20 --warmup 3 > gpurun_out/c1t_$cf.json 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/c1t_$cf.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$cf head', r['kernel_ms'], [(k, v['kernel_ms']) for k,v in d['configs'].items()])"
done
timeout -k 10 300 python3 tools/ab_inproc.py --configs c1,c4,c1 --rounds 3 --steps 20 base || exit 2
