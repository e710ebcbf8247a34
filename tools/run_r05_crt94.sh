#!/bin/bash
set -e
out=gpurun_out/${1:-r05c94}
mkdir -p $out
SNPMI_LIB=tools/libsnpmi_ubench.so timeout -k 10 400 python -u tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants 0,94 --rounds 3 > $out/ubench.jsonl 2> $out/ubench.err
echo ok
