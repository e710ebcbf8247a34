# round 5 A/B on the GPU box: the CRT ring variants (f64, 50k x 62.5k) and the f32 SYRK's rate
# against n at a fixed SNP count (does the packed pitch, i.e. the code panels' span, cost?)
set -e
out=gpurun_out/${1:-r05e}
mkdir -p $out
SNPMI_LIB=tools/libsnpmi_ubench.so timeout -k 10 400 python -u tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants 0,80,81,82,0 --rounds 3 > $out/ubench_crt_ring.jsonl 2> $out/ubench_crt.err
for n in 50000 100000 150000; do
  timeout -k 10 300 python -u tools/ubench.py syrk --dtype f32 --n $n --m 32768 --variants 0 --rounds 3 >> $out/ubench_f32_vs_n.jsonl 2>> $out/ubench_f32.err
done
echo ok
