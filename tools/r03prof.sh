set -o pipefail
bash tools/profile.sh r03 c3,c2,c4,c1 > gpurun_out/prof_r03.log 2>&1 || { tail -20 gpurun_out/prof_r03.log; exit 1; }
tail -3 gpurun_out/prof_r03.log
timeout -k 10 900 python3 bench.py > gpurun_out/bench_default_r03.json 2> gpurun_out/bench_default_r03.err || { tail -20 gpurun_out/bench_default_r03.err; exit 2; }
tail -c 3000 gpurun_out/bench_default_r03.json
