#!/bin/bash
# PMC passes for the unit-utilisation question (is the trace loop VALU-, TA/TD- or L1-bound?):
# one rocprofv3 --pmc run per counter group, no tracing domains. Usage: tools/pmc_units.sh <outdir>
set -e
OUT=${1:-gpurun_out/pmcu}
mkdir -p $OUT
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp && cd $ROOT
run() { name=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python bench.py --parts 1 --slots 1 --n1-batch 1 --steps 2 --warmup 1 --steady-steps 0 --no-group --no-single --no-cpu-baseline --no-oracle-check --no-shadow --no-recur --aux '' > $OUT/$name.log 2>&1; }
run u1 TA_TA_BUSY TA_BUSY GRBM_GUI_ACTIVE
run u2 TD_TD_BUSY TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ
run u3 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F SQ_INSTS_VALU_INT SQ_INSTS_VALU_ADD_F SQ_INSTS_VALU_MUL_F SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU
run u4 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD TA_BUFFER_READ_WAVEFRONTS TA_BUFFER_COALESCED_READ_CYCLES SQ_INSTS_VMEM_RD
python tools/pmc_units_summary.py $OUT $OUT/units.json
