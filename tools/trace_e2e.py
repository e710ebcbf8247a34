"""Run only bench.py's e2e leg (pinned host -> copy stream -> stats + decode on the compute stream)
so a rocprofv3 --kernel-trace --memory-copy-trace of it shows the copy/kernel overlap alone:
  rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o run --output-format csv -- python tools/trace_e2e.py
  python tools/overlap_summary.py DIR --kernels
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402

if __name__ == "__main__":
    args = bench.parse(sys.argv[1:])
    print(json.dumps(bench.leg_e2e(N, args)))
