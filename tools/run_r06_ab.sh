set -e
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_crt.py -k warp tests/test_gpu_specialised.py > $OUT/pytest_spec.log 2>&1
timeout -k 10 400 python -u tools/ab_crt.py --rounds 3 --forms 0,1,4 > $OUT/ab_crt.jsonl 2> $OUT/ab_crt.err
timeout -k 10 400 python -u tools/ab_crt.py --dtype f32 --rounds 3 --forms 0,1 > $OUT/ab_h2.jsonl 2> $OUT/ab_h2.err
echo ab-done
