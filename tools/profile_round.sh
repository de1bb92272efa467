#!/bin/bash
# Round profile of the bench command (run on the GPU box): kernel-trace stats + a separate
# --pmc FETCH_SIZE/WRITE_SIZE pass (counters never combined with tracing domains).
# Usage: tools/profile_round.sh <tag>   -> gpurun_out/prof_<tag>/..., gpurun_out/traffic_<tag>.json
set -e
TAG=${1:-rXX}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-oracle-check --no-recur --aux refit > $OUT/trace.log 2>&1
# one launch at a time (the roofline's per-launch figures): kernel-trace stats whose averages are single launches
ONE="--parts 1 --slots 1 --n1-batch 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/single -o run --output-format csv -- python bench.py --steps 10 --warmup 2 $ONE --no-cpu-baseline --no-oracle-check --no-recur --no-shadow --no-single --no-group --aux '' > $OUT/single.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc/fetch -o fetch --output-format csv -- python bench.py --steps 5 --warmup 1 $ONE --no-cpu-baseline --no-oracle-check --no-recur --no-shadow --no-single --no-group --aux '' > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc/write -o write --output-format csv -- python bench.py --steps 5 --warmup 1 $ONE --no-cpu-baseline --no-oracle-check --no-recur --no-shadow --no-single --no-group --aux '' > $OUT/pmc_write.log 2>&1
python tools/pmc_traffic.py $OUT/pmc gpurun_out/traffic_$TAG.json
