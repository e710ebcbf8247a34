#!/bin/bash
# SegFlush pool A/B, one box: shipped (1024 slots, store + atomics) vs 512 slots vs 512 slots with
# two store sub-slots; cfg4 f32 grm leg (PMC + time) then the cfg5 f32 part job (time).
set -e
bash tools/run_r05_ab_libs.sh r05p2 "head:-:" "old512:tools/libsnpmi_old512.so:" "sub2:tools/libsnpmi_sub2.so:"
bash tools/run_r05_ab_g5.sh r05p2g "head:-" "old512:tools/libsnpmi_old512.so" "sub2:tools/libsnpmi_sub2.so"
