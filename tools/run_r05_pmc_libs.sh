#!/bin/bash
# PMC diagnosis of library builds (cfg4 SYRK): L2 request counters from the instruction/scalar
# caches (SQC) and the vector L1 (TCP), one pass per counter group.
# Usage: tools/run_r05_pmc_libs.sh <tag> "name:lib:hook,hook" ...
set -e
out=gpurun_out/$1
shift
mkdir -p $out
export TMPDIR=/tmp
GRM="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-sid 125000 --grm-f64 off --grm5 off --e2e off --beta off --file off"
run() {
  local name=$1 lib=$2 hooks=$3; shift 3
  local h=""
  for x in ${hooks//,/ }; do h="$h --hook $x"; done
  if [ "$lib" = "-" ]; then "$@" $h; else SNPMI_LIB=$lib "$@" $h; fi
}
for P in "sqc:SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ" "tcp:TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum" "fetch:FETCH_SIZE"; do
  IFS=: read pn counters <<< "$P"
  for spec in "$@"; do
    IFS=: read name lib hooks <<< "$spec"
    mkdir -p $out/$name
    run $name $lib "$hooks" timeout -s KILL 90 rocprofv3 --pmc $counters --kernel-trace -d $out/$name/$pn -o run --output-format csv -- python3 bench.py $GRM > $out/$name/$pn.log 2>&1
  done
done
echo ok
