# decode leg with a tight vs a 32 MB-pitch block buffer, alternating processes
set -e
mkdir -p gpurun_out/ld
Q="--skip-cpu --skip-grm --grm5 off --e2e off --steps 5 --warmup 2"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $Q > gpurun_out/ld/tight_$r.json 2>/dev/null
  timeout -k 10 200 python bench.py $Q --out-ld 8000000 > gpurun_out/ld/spread_$r.json 2>/dev/null
done
echo ok
