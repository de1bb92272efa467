# Where do the trace waves wait? SQ wait/active counters on C4 and C2 (tools/prof_config.py), one
# rocprofv3 --pmc pass per group. Usage: bash tools/gpu/r03_stall.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-stall}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd $ROOT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_]*\|TCP_[A-Z_]*\|TCC_[A-Z_]*" $OUT/avail.txt | sort -u > $OUT/names.txt || true
run() { cfg=$1; name=$2; shift 2; timeout -s KILL 150 rocprofv3 --pmc "$@" -d $OUT/$cfg/$name -o $name --output-format csv -- python tools/prof_config.py $cfg --reps 1 > $OUT/$cfg.$name.log 2>&1; }
for cfg in c4 c2; do
  run $cfg a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_IFETCH || exit $?
  run $cfg b SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD || exit $?
  run $cfg c TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE || exit $?
done
echo done
