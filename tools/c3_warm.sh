# C3 timing vs warmup in one process: c3 twice (the second run follows the first's 20 steps), then warmup 30
export TMPDIR=/tmp
for args in "--configs c3,c3 --warmup 3" "--configs c3 --warmup 30"; do
  timeout -k 10 300 python3 bench.py $args --no-cpu-baseline --no-full-parity --no-parity --c5 0 --steps 20 > gpurun_out/c3w.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/c3w.json').read().strip().splitlines()[-1])
print('$args', d['roofline']['kernel_ms'], [(k, v['kernel_ms']) for k, v in d['configs'].items()])"
done
