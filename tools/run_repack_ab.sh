set -e
mkdir -p gpurun_out/rp
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "repack or subsets" > gpurun_out/rp/tests.log 2>&1
for ix in rev2 sorted random; do
  timeout -k 10 120 python tools/ubench.py repack --index $ix --variants 0,17 --rounds 9 >> gpurun_out/rp/ubench.jsonl 2>>gpurun_out/rp/ubench.err
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rp/prof -o run --output-format csv -- python3 tools/ubench.py repack --index rev2 --variants 0,17 --rounds 7 > gpurun_out/rp/prof.log 2>&1
echo ok
