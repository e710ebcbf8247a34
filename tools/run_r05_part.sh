# round 5: the cfg5 part kernel per block after supertile ownership, at 150k (1 part vs 8) and 500k
set -e
out=gpurun_out/${1:-r05f}
mkdir -p $out
for n in 150000 500000; do
  timeout -k 10 300 python -u tools/exp_part_locality.py $n >> $out/part_locality.jsonl 2>> $out/part.err
done
timeout -k 10 300 python -u tools/ubench.py syrk --dtype f32 --n 250000 --m 32768 --variants 0 --rounds 2 >> $out/ubench_f32_vs_n.jsonl 2>> $out/ubench.err
echo ok
