"""The aux compute stream (snpmi_set_stream, include/snpmi.h): block k's k_snp_stats enqueued on the
aux stream, its decode on the compute stream after an event wait, gives the values of the plain
serial order and of the oracle; the selector is per thread and rejects other stream ids."""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)
import bench
from oracle import oracle as O
from pysnptools_amd import _native as N

pytestmark = pytest.mark.gpu


def test_stats_on_aux_stream_then_decode_matches_serial_and_oracle():
    n, B, nblk = 3001, 256, 6
    m = B * nblk
    pitch = N.lib().snpmi_packed_pitch(n)
    ld = (n + 15) // 16 * 16
    packed = bench.Dev(N, pitch * m)
    bench.synth(N, packed.p, pitch, n, 0, m, 11, 0.05)
    lut, stats = bench.Dev(N, 2 * B * 16), bench.Dev(N, 2 * B * 8)
    out_a, out_s = bench.Dev(N, m * ld * 4), bench.Dev(N, m * ld * 4)
    ev = bench.Events(N, 4)
    rec = [False, False]
    try:
        for k in range(nblk):  # aux-stream stats, two LUT slots, cross-stream events
            sl, src = k & 1, packed.at(k * B * pitch)
            if rec[sl]:
                N.call("snpmi_stream_wait_event", ev.ev[2 + sl], 2)
            N.call("snpmi_set_stream", 2)
            N.call("snpmi_dev_snp_stats", src, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32,
                   stats.at(sl * B * 8), lut.at(sl * B * 16))
            N.call("snpmi_set_stream", 0)
            ev.record(sl, 2)
            N.call("snpmi_stream_wait_event", ev.ev[sl], 0)
            N.call("snpmi_dev_decode", src, pitch, n, B, lut.at(sl * B * 16), N.DT_F32, 0,
                   out_a.at(k * B * ld * 4), ld)
            ev.record(2 + sl)
            rec[sl] = True
        for k in range(nblk):  # serial reference order on the compute stream
            src = packed.at(k * B * pitch)
            N.call("snpmi_dev_snp_stats", src, pitch, n, B, 0, N.STD_UNIT, 0.0, 0.0, 0, N.DT_F32, stats.p, lut.p)
            N.call("snpmi_dev_decode", src, pitch, n, B, lut.p, N.DT_F32, 0, out_s.at(k * B * ld * 4), ld)
        N.call("snpmi_stream_sync")
        a = np.empty((m, ld), dtype=np.float32)
        s = np.empty((m, ld), dtype=np.float32)
        N.call("snpmi_memcpy_d2h", N.ptr(a), out_a.p, a.nbytes)
        N.call("snpmi_memcpy_d2h", N.ptr(s), out_s.p, s.nbytes)
        assert np.array_equal(a[:, :n], s[:, :n])
        host = np.empty((m, pitch), dtype=np.uint8)
        N.call("snpmi_memcpy_d2h", N.ptr(host), packed.p, host.nbytes)
        body = np.ascontiguousarray(host[:, :(n + 3) // 4]).reshape(-1)
        Z, _ = O.decode_standardize(body, n, m, dtype=np.float32)
        assert np.array_equal(a[:, :n].T, Z)
    finally:
        N.call("snpmi_set_stream", 0)
        ev.destroy()
        for d in (packed, lut, stats, out_a, out_s):
            d.free()


def test_set_stream_rejects_other_ids():
    with pytest.raises(Exception):
        N.call("snpmi_set_stream", 1)
    N.call("snpmi_set_stream", 0)
