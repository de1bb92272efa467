#!/bin/bash
# Diagnosis of the exit with live dedicated streams under rocprofv3 (tests/test_gpu_lifecycle.py): the child
# plainly, under rocprofv3 --kernel-trace with the library's exit-time stream teardown, and without it.
# Every step has its own time limit; outputs in gpurun_out/$1/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=gpurun_out/${1:-sexit}; mkdir -p $O
C=tests/native/stream_exit_child.py
timeout -k 10 120 python -u $C > $O/plain.out 2> $O/plain.err; echo "plain rc=$?" >> $O/rc.txt
timeout -k 10 90 rocprofv3 --kernel-trace -d $O/prof_on -o run -- python -u $C > $O/prof_on.out 2> $O/prof_on.err
echo "prof_on rc=$?" >> $O/rc.txt
TT_STREAM_EXIT_HANDLER=0 timeout -k 10 90 rocprofv3 --kernel-trace -d $O/prof_off -o run -- python -u $C \
    > $O/prof_off.out 2> $O/prof_off.err
echo "prof_off (library exit teardown off) rc=$?" >> $O/rc.txt
timeout -k 10 90 rocprofv3 --kernel-trace -d $O/prof_keep -o run -- python -u $C keep-contexts > $O/prof_keep.out \
    2> $O/prof_keep.err
echo "prof_keep rc=$?" >> $O/rc.txt
cat $O/rc.txt
