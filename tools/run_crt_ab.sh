# f64 GRM (CRT) chunk ring A/B + tests, on the GPU box
set -e
mkdir -p gpurun_out/crt
timeout -k 10 300 python -u -m pytest tests/test_gpu_crt.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/crt/tests.log 2>&1
SNPMI_LIB=tools/libsnpmi_ubench.so timeout -k 10 400 python tools/ubench.py syrk --dtype f64 --n 50000 --m 10000 --variants 0,77 --rounds 5 --noassert 1 > gpurun_out/crt/ubench_f64_ring.jsonl 2> gpurun_out/crt/ubench.err
echo ok
