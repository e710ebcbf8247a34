#!/bin/bash
# Full validation on one GPU box (via gpurun): the -m gpu suite, smoke(), the default bench and the
# round-3 profiling recipe.  Usage: tools/run_validate.sh <tag>; outputs under gpurun_out/val_<tag>.
# Every GPU step has its own limit; the chain stops at the first failure.
set -e
TAG=${1:-val}
OUT=gpurun_out/val_$TAG
mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench.err
bash tools/profile_r03.sh $TAG
echo validate-done
