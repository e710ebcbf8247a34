set -e
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_crt.py --dtype f64 --n 50000 --m 62500 --rounds 5 --forms 1,3 > $OUT/ab_crt_n50k.jsonl 2> $OUT/ab_crt_n50k.err
timeout -k 10 300 python -u tools/ab_crt.py --dtype f64 --n 4100 --m 62500 --rounds 5 --forms 1,3 > $OUT/ab_crt_n4100.jsonl 2> $OUT/ab_crt_n4100.err
timeout -k 10 300 python -u tools/ab_crt.py --dtype f64 --n 500000 --m 8192 --rounds 2 --forms 1,3 --part 0/8 > $OUT/ab_crt_part.jsonl 2> $OUT/ab_crt_part.err
echo ab-done
