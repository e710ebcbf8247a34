set -e
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_crt.py tests/test_gpu_parity.py tests/test_gpu_part_order.py tests/test_gpu_fuzz.py > $OUT/pytest_crt.log 2>&1
timeout -k 10 300 python -u tools/ab_crt.py --dtype f64 --n 50000 --m 62500 --rounds 3 --forms 1,2 > $OUT/ab_crt_n50k.jsonl 2> $OUT/ab_crt_n50k.err
timeout -k 10 400 python -u bench.py --grm5 off --beta off --file off --e2e off > $OUT/bench_grm.json 2> $OUT/bench_grm.err
echo ab-done
