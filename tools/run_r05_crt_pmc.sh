set -e
out=gpurun_out/r05c1; mkdir -p $out; export TMPDIR=/tmp
GRM64="--n-iid 16384 --n-sid 16384 --steps 1 --warmup 0 --skip-cpu --grm-sid 125000 --grm5 off --e2e off --beta off --file off"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d $out/crt_$C -o run --output-format csv -- python3 bench.py $GRM64 > $out/crt_$C.log 2>&1
done
timeout -s KILL 180 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --kernel-trace -d $out/crt_tcp -o run --output-format csv -- python3 bench.py $GRM64 > $out/crt_tcp.log 2>&1
echo ok
