set -e
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
timeout -k 10 500 python -u tools/ab_crt.py --n 500000 --m 32768 --part 0/8 --rounds 2 --forms 0,1 > $OUT/ab_crt_part.jsonl 2> $OUT/ab_crt_part.err
timeout -k 10 500 python -u tools/ab_crt.py --dtype f32 --n 500000 --m 32768 --part 0/8 --rounds 2 --forms 0,1 > $OUT/ab_h2_part.jsonl 2> $OUT/ab_h2_part.err
echo ab-done
