#!/bin/bash
# Kernel time + fabric traffic (separate FETCH_SIZE / WRITE_SIZE passes) of one config's traces.
# Usage: tools/pmc_config.sh c4 <outdir>
set -e
CFG=$1
OUT=${2:-gpurun_out/pmc_$CFG}
mkdir -p $OUT
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp && cd $ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python tools/prof_config.py $CFG > $OUT/trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc/fetch -o fetch --output-format csv -- python tools/prof_config.py $CFG --reps 1 > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc/write -o write --output-format csv -- python tools/prof_config.py $CFG --reps 1 > $OUT/write.log 2>&1
python tools/pmc_traffic.py $OUT/pmc $OUT/traffic.json
