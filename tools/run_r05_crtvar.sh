#!/bin/bash
# CRT SYRK variants on the XCD-grouped mapping (ubench 0 = default MAP 1; 90-93 = MAP 1 with the
# round-4/5 schedule variants 78/79/83/84), 50k x 62.5k, alternating rounds.
set -e
out=gpurun_out/${1:-r05v2}
mkdir -p $out
SNPMI_LIB=tools/libsnpmi_ubench.so timeout -k 10 600 python -u tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants 0,90,91,92,93 --rounds 3 > $out/ubench_crtvar.jsonl 2> $out/ubench.err
echo ok
