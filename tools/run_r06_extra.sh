set -e
OUT=gpurun_out/${1:-r06j}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --skip-grm --beta off --file off --e2e off --grm5-dtype f64 > $OUT/bench_grm5_f64.json 2> $OUT/grm5_f64.err
if [ "${2:-}" = rccl ]; then
  timeout -k 10 300 python -u bench.py --force-rccl --steps 1 --warmup 0 --n-sid 20000 --grm-sid 62500 --grm5-sid 65536 --file off --beta off --e2e off > $OUT/bench_force_rccl.json 2> $OUT/force_rccl.err
fi
echo extra-done
