#!/bin/bash
# Diagnosis of the exit with live dedicated streams (tests/test_gpu_lifecycle.py): bash stream_exit_diag.sh TAG MODE
#   MODE plain    the child, no profiler
#   MODE prof     under rocprofv3 --kernel-trace, with the library's exit-time stream teardown
#   MODE profoff  the same without it (TT_STREAM_EXIT_HANDLER=0)
# One mode per gpurun call: a crash or a time limit ends the call (no GPU step after it). Outputs: gpurun_out/TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=gpurun_out/${1:-sexit}; mkdir -p "$O"
C=tests/native/stream_exit_child.py
case ${2:-prof} in
plain) timeout -k 10 120 python -u $C > "$O/plain.out" 2> "$O/plain.err" ;;
prof) timeout -k 10 60 rocprofv3 --kernel-trace -d "$O/prof_on" -o run -- python -u $C > "$O/prof_on.out" 2> "$O/prof_on.err" ;;
profoff) TT_STREAM_EXIT_HANDLER=0 timeout -k 10 60 rocprofv3 --kernel-trace -d "$O/prof_off" -o run -- python -u $C \
             > "$O/prof_off.out" 2> "$O/prof_off.err" ;;
esac
rc=$?
echo "${2:-prof} rc=$rc" | tee -a "$O/rc.txt"
exit $rc
