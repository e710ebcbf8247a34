#!/bin/bash
# GPU check of the GRM file path (via gpurun): new extraction tests, the full -m gpu suite, then a
# rocprofv3 kernel + memory-copy trace of tools/trace_file_grm.py.  Usage: tools/run_check_grm_path.sh <tag>
set -e
OUT=gpurun_out/${1:-tf2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_extract.log 2>&1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/trace -o run --output-format csv -- python3 tools/trace_file_grm.py > $OUT/out.jsonl 2> $OUT/err.txt
echo check-done
