#!/bin/bash
# Round-6 validation on one GPU box (via gpurun): the -m gpu suite + smoke(), then the default
# bench.  Every GPU step has its own limit; the chain stops at the first failure.
#   tools/run_validate_r06.sh <tag> [tests|bench|all]
set -e
TAG=${1:-r06}
WHAT=${2:-all}
OUT=gpurun_out/val_$TAG
mkdir -p $OUT
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench.err
fi
echo validate-done
