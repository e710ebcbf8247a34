set -e
mkdir -p gpurun_out/r05sub2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_f32_accuracy.py > gpurun_out/r05sub2/pytest_f32_acc.log 2>&1
bash tools/run_r05_ab_libs.sh r05sub2 "old:tools/libsnpmi_r05q.so:" "sub1:tools/libsnpmi_sub1.so:" "sub6:-:"
