#!/bin/bash
# What do the SegFlush slot rounds cost in time?  cfg4 f32 grm leg and cfg5 f32 part with seg 12288
# (default) vs seg 0 (one chain per launch: no slot traffic, less accurate), same box, alternating.
set -e
out=gpurun_out/${1:-r05sc}
mkdir -p $out
A="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-f64 off --beta off --file off --e2e off"
for s in 12288 0 12288 0; do
  timeout -k 10 300 python -u bench.py $A --hook seg=$s > $out/b_$s.json 2>> $out/b_$s.err
  cat $out/b_$s.json >> $out/all_seg$s.jsonl
done
echo ok
