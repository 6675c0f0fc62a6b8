cat /sys/fs/cgroup/cpu.max 2>&1; cat /sys/fs/cgroup/cpu/cpu.cfs_quota_us 2>&1; nproc; echo OMP=$OMP_NUM_THREADS; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
timeout -k 10 300 python3 -u -m pytest -q -x tests/test_replay_gpu.py --timeout 120 --timeout-method thread > gpurun_out/replay_tests.log 2>&1 || { tail -20 gpurun_out/replay_tests.log; exit 1; }
tail -1 gpurun_out/replay_tests.log
GPK_REPLAY_TRACE=1 timeout -k 10 400 python3 bench.py --configs c1 --no-cpu-baseline --no-full-parity --steps 3 --warmup 1 > gpurun_out/c5_pool.json 2>gpurun_out/c5_pool.err || { tail -20 gpurun_out/c5_pool.err; exit 2; }
python3 -c "
import json; d=json.loads(open('gpurun_out/c5_pool.json').read().strip().splitlines()[-1]); c=d['c5']; print(c['value'], c['wall_s'], c['runs_wall_s'], c['breakdown_s'], c['parity'])"
grep gpk_replay gpurun_out/c5_pool.err | tail -3
