#!/bin/bash
# A/B of library builds on the cfg5 f32 whole part (bench grm5 leg), alternating, same box.
# Usage: tools/run_r05_ab_g5.sh <tag> "name:lib" ...
set -e
out=gpurun_out/$1
shift
mkdir -p $out
A="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --skip-grm --beta off --file off --e2e off"
for r in 1 2; do
  for spec in "$@"; do
    IFS=: read name lib <<< "$spec"
    if [ "$lib" = "-" ]; then timeout -k 10 300 python3 -u bench.py $A > $out/g5_${name}_$r.json 2> $out/g5_${name}_$r.err
    else SNPMI_LIB=$lib timeout -k 10 300 python3 -u bench.py $A > $out/g5_${name}_$r.json 2> $out/g5_${name}_$r.err; fi
  done
done
echo ok
