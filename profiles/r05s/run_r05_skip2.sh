#!/bin/bash
# Round-5 A/B on one GPU box: the cfg4 SYRK's PMC read/write traffic and the bench grm leg time
# with the round-5 final library (tools/libsnpmi_r05q.so, built from 9e5008b) vs the current one
# (adaptive SegFlush on / off).  Usage: tools/run_r05_skip2.sh <tag>
set -e
out=gpurun_out/${1:-r05s3}
mkdir -p $out
export TMPDIR=/tmp
GRM="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-sid 125000 --grm-f64 off --grm5 off --e2e off --beta off --file off"
for C in FETCH_SIZE WRITE_SIZE; do
  mkdir -p $out/old $out/new16 $out/new0
  SNPMI_LIB=tools/libsnpmi_r05q.so timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $out/old/grm_$C -o run --output-format csv -- python3 bench.py $GRM > $out/old/grm_$C.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $out/new16/grm_$C -o run --output-format csv -- python3 bench.py $GRM --hook seg_skip=16 > $out/new16/grm_$C.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $out/new0/grm_$C -o run --output-format csv -- python3 bench.py $GRM --hook seg_skip=0 > $out/new0/grm_$C.log 2>&1
done
for v in old new16 new0; do
  python3 tools/traffic_summary.py $out/$v $out/$v/traffic.json 500000,2048 50000,62500 > $out/$v/traffic.log 2>&1 || true
done
T="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-f64 off --grm5 off --e2e off --beta off --file off"
for r in 1 2; do
  SNPMI_LIB=tools/libsnpmi_r05q.so timeout -k 10 200 python3 -u bench.py $T > $out/t_old_$r.json 2> $out/t_old_$r.err
  timeout -k 10 200 python3 -u bench.py $T --hook seg_skip=16 > $out/t_new16_$r.json 2> $out/t_new16_$r.err
  timeout -k 10 200 python3 -u bench.py $T --hook seg_skip=0 > $out/t_new0_$r.json 2> $out/t_new0_$r.err
done
[ "${2:-}" = sweep ] && timeout -k 10 300 python -u tools/exp_seg_skip.py 20000 48000 32,16,0 12288,8192 > $out/sweep_20k.jsonl 2> $out/sweep_20k.err
[ "${2:-}" = sweep ] && timeout -k 10 400 python -u tools/exp_seg_skip.py 50000 62500 32,16,0 12288,8192 > $out/sweep_50k.jsonl 2> $out/sweep_50k.err
echo ok
