#!/bin/bash
# Quick SQ counter passes for one kernel build. Usage: tools/pmc_quick.sh <outdir> [lib.so]
# (each pass its own rocprofv3 run; --pmc only, no tracing domains)
set -e
OUT=${1:-gpurun_out/pmcq}
[ -n "$2" ] && export TT_HIP_LIB=$(realpath $2)
mkdir -p $OUT
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp && cd $ROOT
run() { name=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python tools/prof_trace.py --reps 2 > $OUT/$name.log 2>&1; }
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA
