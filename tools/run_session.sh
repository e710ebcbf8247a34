# Full GPU check of HEAD on the box: tests, smoke, the driver-form bench, its rocprof kernel stats.
# Usage: bash tools/run_session.sh <tag>   (outputs under gpurun_out/<tag>/)
set -e
TAG=${1:-s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --skip-cpu > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err
echo session-done
