#!/bin/bash
# A/B of library builds on one GPU box: cfg4 SYRK PMC FETCH/WRITE + bench grm leg time.
# Usage: tools/run_r05_ab_libs.sh <tag> "name:lib:hook,hook" ...   (lib "-" = the in-tree library)
set -e
out=gpurun_out/$1
shift
mkdir -p $out
export TMPDIR=/tmp
GRM="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-sid 125000 --grm-f64 off --grm5 off --e2e off --beta off --file off"
T="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-f64 off --grm5 off --e2e off --beta off --file off"
run() {  # name lib hooks cmd...
  local name=$1 lib=$2 hooks=$3; shift 3
  local h=""
  for x in ${hooks//,/ }; do h="$h --hook $x"; done
  if [ "$lib" = "-" ]; then "$@" $h; else SNPMI_LIB=$lib "$@" $h; fi
}
for C in FETCH_SIZE WRITE_SIZE; do
  for spec in "$@"; do
    IFS=: read name lib hooks <<< "$spec"
    mkdir -p $out/$name
    run $name $lib "$hooks" timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $out/$name/grm_$C -o run --output-format csv -- python3 bench.py $GRM > $out/$name/grm_$C.log 2>&1
  done
done
for r in 1 2; do
  for spec in "$@"; do
    IFS=: read name lib hooks <<< "$spec"
    run $name $lib "$hooks" timeout -k 10 200 python3 -u bench.py $T > $out/t_${name}_$r.json 2> $out/t_${name}_$r.err
  done
done
echo ok
