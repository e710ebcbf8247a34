"""H2D rate of one pinned buffer by transfer shape: one 1 GB hipMemcpyAsync vs pieces of 64-512 MB,
on the compute or the copy stream (why grm5's upload runs at 30 GB/s while e2e's 256 MB chunks
run at 56).  Prints JSON lines."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import Dev, Events  # noqa: E402
from pysnptools_amd import _native as N  # noqa: E402

total = 1 << 30
host = ctypes.c_void_p()
N.call("snpmi_host_alloc", ctypes.byref(host), total)
dev = Dev(N, total)
N.call("snpmi_memcpy_d2h", host, dev.p, total)
ev = Events(N, 2)
for on_copy in (0, 1):
    for piece in (total, 512 << 20, 256 << 20, 128 << 20, 64 << 20):
        ts = []
        for rep in range(4):
            ev.record(0, on_copy)
            for off in range(0, total, piece):
                N.call("snpmi_memcpy_async", dev.at(off), ctypes.c_void_p(host.value + off), piece, 0, on_copy)
            ev.record(1, on_copy)
            N.call("snpmi_stream_sync")
            ts.append(ev.ms(0, 1))
        ts = sorted(ts)[1:]
        print(json.dumps({"stream": "copy" if on_copy else "compute", "piece_MB": piece >> 20,
                          "ms": min(ts), "GBps": total / (min(ts) * 1e-3) / 1e9}), flush=True)
N.call("snpmi_host_free", host)
dev.free()
