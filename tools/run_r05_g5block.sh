#!/bin/bash
# cfg5 f32 whole part: all-gathered SNP block 32768 (default) vs 65536, same box.
set -e
out=gpurun_out/${1:-r05g}
mkdir -p $out
A="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --skip-grm --beta off --file off --e2e off"
for b in 32768 65536 32768 65536; do
  timeout -k 10 300 python -u bench.py $A --grm5-block $b > $out/g5_$b.json 2>> $out/g5_$b.err
  cat $out/g5_$b.json >> $out/all.jsonl
done
echo ok
