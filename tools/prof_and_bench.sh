# GPU step: profiles (tools/profile.sh TAG CFGS), then the default bench line.
#   bash tools/prof_and_bench.sh TAG [configs]
# Results: gpurun_out/prof_TAG/, gpurun_out/bench_default_TAG.json;
# summaries: python tools/make_profiles.py TAG configs
set -o pipefail
TAG=${1:?tag}
CFGS=${2:-c3,c2,c4,c1}
bash tools/profile.sh $TAG $CFGS > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -3 gpurun_out/prof_$TAG.log
timeout -k 10 900 python3 bench.py > gpurun_out/bench_default_$TAG.json 2> gpurun_out/bench_default_$TAG.err || { tail -20 gpurun_out/bench_default_$TAG.err; exit 2; }
tail -c 3000 gpurun_out/bench_default_$TAG.json
