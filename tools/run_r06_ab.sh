set -e
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_crt.py > $OUT/pytest_crt.log 2>&1
timeout -k 10 300 python -u tools/ab_crt.py --dtype f64 --n 50000 --m 62500 --rounds 3 --forms 1,3 > $OUT/ab_load2_n50k.jsonl 2> $OUT/ab_load2_n50k.err
echo ab-done
