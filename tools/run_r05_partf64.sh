#!/bin/bash
# cfg5 f64 part SYRK: XCD-grouped moduli (0) vs the round-5 grid (88): time, FETCH, SQ clock.
set -e
out=gpurun_out/${1:-r05pf}
mkdir -p $out
export TMPDIR=/tmp
L=tools/libsnpmi_ubench.so
SNPMI_LIB=$L timeout -k 10 300 python -u tools/exp_part_f64.py 150000 32768 8 88,0 3 > $out/time.jsonl 2> $out/time.err
for v in 88 0; do
  SNPMI_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch_$v -o run --output-format csv -- python3 tools/exp_part_f64.py 150000 32768 8 $v 1 > $out/fetch_$v.log 2>&1
  SNPMI_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $out/sq_$v -o run --output-format csv -- python3 tools/exp_part_f64.py 150000 32768 8 $v 1 > $out/sq_$v.log 2>&1
done
echo ok
