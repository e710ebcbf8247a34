# fp16x2 SYRK compiled with alternative LLVM scheduler strategies (syrk.hip only), one process per library
set -e
mkdir -p gpurun_out/sched
for lib in pysnptools_amd/libsnpmi.so tools/sched/libsnpmi_max-ilp.so tools/sched/libsnpmi_max-memory-clause.so tools/sched/libsnpmi_iterative-ilp.so pysnptools_amd/libsnpmi.so; do
  echo "$lib" >> gpurun_out/sched/syrk.jsonl
  SNPMI_LIB=$lib timeout -k 10 200 python tools/ubench.py syrk --n 50000 --m 10000 --variants 0 --rounds 4 >> gpurun_out/sched/syrk.jsonl 2>> gpurun_out/sched/err.txt
done
echo ok
