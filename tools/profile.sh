#!/bin/bash
# Profiling recipe run ON THE GPU BOX (via gpurun).  Usage: tools/profile.sh <tag>
#  1. kernel trace + stats of the default bench (per-kernel average durations)
#  2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) -- TCC slots cannot hold both --
#     on a 1-step decode run and a short GRM run, for HBM traffic per launch.
# Outputs land in gpurun_out/prof_<tag>/; copy the summaries to profiles/<tag>/.
set -e
TAG=${1:-r01i}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
DEC="--steps 1 --warmup 1 --skip-cpu --skip-grm"
GRM="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-sid 30000"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --skip-cpu > $OUT/trace.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $OUT/dec_$C -o run --output-format csv -- python3 bench.py $DEC > $OUT/dec_$C.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $OUT/grm_$C -o run --output-format csv -- python3 bench.py $GRM > $OUT/grm_$C.log 2>&1
done
python3 tools/traffic_summary.py $OUT $OUT/traffic.json > $OUT/traffic.log 2>&1 || true
echo profile-done
