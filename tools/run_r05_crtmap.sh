#!/bin/bash
# CRT SYRK workgroup mapping A/B (ubench variant 87 = XCD-grouped moduli vs 0): time at 50k x 62.5k,
# then FETCH_SIZE / SQ counters of each mapping.  Usage: tools/run_r05_crtmap.sh <tag>
set -e
out=gpurun_out/${1:-r05m}
mkdir -p $out
export TMPDIR=/tmp
SNPMI_LIB=tools/libsnpmi_ubench.so timeout -k 10 400 python -u tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants 0,87 --rounds 4 > $out/ubench_crtmap.jsonl 2> $out/ubench.err
for v in 0 87; do
  SNPMI_LIB=tools/libsnpmi_ubench.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch_$v -o run --output-format csv -- python3 tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants $v --rounds 1 > $out/fetch_$v.log 2>&1
  SNPMI_LIB=tools/libsnpmi_ubench.so timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $out/sq_$v -o run --output-format csv -- python3 tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants $v --rounds 1 > $out/sq_$v.log 2>&1
done
echo ok
