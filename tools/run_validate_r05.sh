#!/bin/bash
# Round-5 validation on one GPU box (via gpurun), in two calls that each fit gpurun's limit:
#   tools/run_validate_r05.sh tests <tag>   -> the -m gpu suite + smoke()
#   tools/run_validate_r05.sh bench <tag>   -> the default bench + tools/profile_r05.sh
# Every GPU step has its own limit; the chain stops at the first failure.
set -e
WHAT=${1:-tests}
TAG=${2:-r05}
OUT=gpurun_out/val_$TAG
mkdir -p $OUT
if [ "$WHAT" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
else
  timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench.err
  bash tools/profile_r05.sh $TAG
fi
echo validate-done
