set -e
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_crt.py --dtype f64 --n 50000 --m 62500 --rounds 4 --forms 1,3,4 > $OUT/ab_hold_n50k.jsonl 2> $OUT/ab_hold_n50k.err
echo ab-done
