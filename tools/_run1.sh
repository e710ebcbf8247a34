set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/bf3m
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "grm" > gpurun_out/bf3m/pytest.log 2>&1
timeout -k 10 200 python tools/ubench.py syrk --n 50000 --m 10000 --rounds 3 --variants 0,33,34,38,39 > gpurun_out/bf3m/ub.jsonl 2>&1
