#!/bin/bash
# A/B of the f64 squares' place around the cfg4 SYRK (hook diag_order 0 = before, 1 = after, as
# until round 5) and adaptive flushes, one box: SYRK PMC traffic + bench grm leg time.
set -e
out=gpurun_out/${1:-r05s4}
mkdir -p $out
export TMPDIR=/tmp
GRM="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-sid 125000 --grm-f64 off --grm5 off --e2e off --beta off --file off"
for C in FETCH_SIZE WRITE_SIZE; do
  for v in "o1 --hook seg_skip=0 --hook diag_order=1" "o0s0 --hook seg_skip=0" "o0s16 --hook seg_skip=16"; do
    set -- $v
    tag=$1; shift
    mkdir -p $out/$tag
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $out/$tag/grm_$C -o run --output-format csv -- python3 bench.py $GRM "$@" > $out/$tag/grm_$C.log 2>&1
  done
done
T="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-f64 off --grm5 off --e2e off --beta off --file off"
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py $T --hook seg_skip=0 --hook diag_order=1 > $out/t_o1_$r.json 2> $out/t_o1_$r.err
  timeout -k 10 200 python3 -u bench.py $T --hook seg_skip=0 > $out/t_o0s0_$r.json 2> $out/t_o0s0_$r.err
  timeout -k 10 200 python3 -u bench.py $T --hook seg_skip=16 > $out/t_o0s16_$r.json 2> $out/t_o0s16_$r.err
done
echo ok
