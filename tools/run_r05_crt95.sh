#!/bin/bash
# CRT grid A/B: 0 = XCD-grouped moduli (shipped), 95 = pairs of blocks per XCD; time + FETCH + SQ clock.
set -e
out=gpurun_out/${1:-r05c95}
mkdir -p $out
export TMPDIR=/tmp
L=tools/libsnpmi_ubench.so
SNPMI_LIB=$L timeout -k 10 400 python -u tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants 0,95 --rounds 4 > $out/ubench.jsonl 2> $out/ubench.err
for v in 0 95; do
  SNPMI_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch_$v -o run --output-format csv -- python3 tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants $v --rounds 1 > $out/fetch_$v.log 2>&1
  SNPMI_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $out/sq_$v -o run --output-format csv -- python3 tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants $v --rounds 1 > $out/sq_$v.log 2>&1
done
echo ok
