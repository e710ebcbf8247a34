#!/bin/bash
# Round-6 profiling recipe, run ON THE GPU BOX (via gpurun).  Usage: tools/profile_r06.sh <tag>
#  1. kernel trace + stats of the default bench (per-kernel average durations; tools/trace_summary.py)
#  2. separate PMC passes FETCH_SIZE / WRITE_SIZE on a decode-only run, a GRM-only run (cfg4 shape,
#     2 launches of 62500 SNPs) and the dense standardize (50k x 100k f32 in HBM, round-4 kernel)
#  3. one SQ pass on the GRM-only run: MFMA busy per SIMD and the loaded clock
# Every step has its own time limit and the chain stops at the first failure.
set -e
TAG=${1:-r06}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
DEC="--steps 1 --warmup 1 --skip-cpu --skip-grm --grm5 off --e2e off --beta off --file off"
GRM="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-sid 125000 --grm-f64 off --grm5 off --e2e off --beta off --file off"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --skip-cpu > $OUT/bench_under_rocprof.json 2> $OUT/trace.log
python3 tools/trace_summary.py $OUT/trace/run_kernel_trace.csv $OUT/bench_under_rocprof.json > $OUT/kernel_trace_summary.json 2>&1 || true
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/dec_$C -o run --output-format csv -- python3 bench.py $DEC > $OUT/dec_$C.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/grm_$C -o run --output-format csv -- python3 bench.py $GRM > $OUT/grm_$C.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/std_$C -o run --output-format csv -- python3 tools/exp_std_dense.py --only 0 --reps 1 > $OUT/std_$C.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $OUT/grm_SQ -o run --output-format csv -- python3 bench.py $GRM > $OUT/grm_SQ.log 2>&1
GRM64="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-sid 125000 --grm5 off --e2e off --beta off --file off"
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/crt_SQ -o run --output-format csv -- python3 bench.py $GRM64 > $OUT/crt_SQ.log 2>&1
python3 tools/pmc_summary.py $OUT/crt_SQ --match k_syrk_i8w > $OUT/pmc_sq_crt.json 2>&1 || true
python3 tools/traffic_summary.py $OUT $OUT/traffic.json 500000,2048 50000,62500 > $OUT/traffic.log 2>&1 || true
python3 tools/pmc_summary.py $OUT/grm_SQ --match k_syrk > $OUT/pmc_sq_grm.json 2>&1 || true
echo profile-done
