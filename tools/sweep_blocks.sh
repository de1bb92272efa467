for b in 1 2 3 4 5; do echo "blocks/CU=$b"; TT_BLOCKS_PER_CU=$b timeout -k 10 120 python tools/prof_trace.py --reps 3 2>&1 | grep "launch ms"; done
