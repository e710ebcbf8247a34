#!/bin/bash
# GPU run (via gpurun): the seeded fuzz parity sweep, then the host-gather A/B.
set -e
OUT=gpurun_out/fg
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_fuzz.log 2>&1
timeout -k 10 400 python -u tools/exp_gather.py > $OUT/gather.jsonl 2> $OUT/gather.err
echo fg-done
