# round 5: k_diag_sq with 4x the SNP slices, traced at 500k iids (the cfg5 part kernel) and 50k
set -e
out=gpurun_out/${1:-r05k}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/exp_part_locality.py 500000 > $out/part.jsonl 2> $out/part.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_accuracy.py tests/test_gpu_overlap_reduce.py tests/test_gpu_part_order.py tests/test_gpu_partitioned_kernel.py tests/test_gpu_checkpoint.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
echo ok
SNPMI_LIB=tools/libsnpmi_ubench.so timeout -k 10 300 python -u tools/ubench.py syrk --dtype f64 --n 50000 --m 62500 --variants 0,86,0,86 --rounds 3 > $out/ubench_crt_16w.jsonl 2> $out/ubench.err
echo ok2
