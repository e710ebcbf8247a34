set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r01f
timeout -k 10 300 python bench.py > gpurun_out/r01f/bench_default.json 2> gpurun_out/r01f/bench.err
timeout -k 10 300 python tools/bench_file.py > gpurun_out/r01f/bench_file.jsonl 2> gpurun_out/r01f/bench_file.err
bash tools/profile.sh r01f
