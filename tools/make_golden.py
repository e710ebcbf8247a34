"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Runs only in the build container (it imports /root/reference, which never travels to the
GPU box).  The committed outputs are data: reference fixture files copied verbatim
(.bed/.bim/.fam) and small .npz files of inputs + expected outputs computed by the
reference's Python path (``force_python_only=True``).

Import harness: the reference's native dependency ``bed_reader``
(Rust, not installed, not vendored) is replaced by a stub module whose native entry points
raise, plus a pure gather for ``subset_*``; ``np.NAN`` is restored (util/__init__.py:329).
Decoding uses this script's own NumPy restatement of the BED format (Appendix B), pinned
bit-exactly against the reference fixture ``all_chr.maf0.001.N300.pst.npz``.

Usage:  python tools/make_golden.py
"""
import os
import shutil
import sys
import types
import warnings

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
DATA = os.path.join(OUT, "data")


def install_harness():
    np.NAN = np.nan
    stub = types.ModuleType("bed_reader")

    def _native(*a, **k):
        raise NotImplementedError("bed-reader native path unavailable offline")

    for n in ["open_bed", "to_bed", "standardize_f64", "standardize_f32"]:
        setattr(stub, n, _native)

    def _subset(val, rows, cols, out, num_threads):
        out[...] = val[np.ix_(rows, cols)]

    stub.subset_f64_f64 = stub.subset_f32_f64 = stub.subset_f32_f32 = _subset
    stub.get_num_threads = lambda n=None: n or 1
    sys.modules["bed_reader"] = stub
    sys.path.insert(0, REF)


def decode(path, n_iid, count_A1=False):
    b = np.fromfile(path, dtype=np.uint8)
    assert list(b[:3]) == [0x6C, 0x1B, 0x01]
    body = b[3:].reshape(-1, (n_iid + 3) // 4)
    codes = np.stack([(body >> s) & 3 for s in (0, 2, 4, 6)], -1).reshape(body.shape[0], -1)[:, :n_iid]
    lut = np.array([2, np.nan, 1, 0]) if count_A1 else np.array([0, np.nan, 1, 2])
    return lut[codes].T


def nlines(p):
    with open(p) as f:
        return sum(1 for line in f if line.strip())


def to_i8(val):
    out = np.where(np.isnan(val), -127, val).astype(np.int8)
    return out


def copy_triple(src_base, dst_name):
    for ext in ("bed", "bim", "fam"):
        shutil.copyfile(src_base + "." + ext, os.path.join(DATA, dst_name + "." + ext))


def main():
    install_harness()
    from pysnptools.snpreader import SnpData
    from pysnptools.snpreader.snpgen import SnpGen
    from pysnptools.standardizer import Unit, Beta, DiagKtoN
    from pysnptools.kernelreader import SnpKernel

    warnings.simplefilter("ignore")
    os.makedirs(DATA, exist_ok=True)

    def sd(val, n=None):
        n_iid, n_sid = val.shape
        return SnpData(iid=[["f%d" % i, "i%d" % i] for i in range(n_iid)],
                       sid=["s%d" % j for j in range(n_sid)], val=val)

    def std_py(val, std, dtype, order="F"):
        d = sd(np.array(val, dtype=dtype, order=order))
        d2, tr = d.standardize(std, return_trained=True, force_python_only=True)
        return d2.val, tr

    # ------------------------------------------------------------------ N300 (cfg1)
    base = REF + "/tests/datasets/all_chr.maf0.001.N300"
    copy_triple(base, "n300")
    n_iid, n_sid = nlines(base + ".fam"), nlines(base + ".bim")
    val = decode(base + ".bed", n_iid)
    fixture = np.load(base + ".pst.npz", allow_pickle=False)["val"]
    assert np.array_equal(val, fixture, equal_nan=True), "restated decoder disagrees with pst.npz"
    g = {"shape": np.array([n_iid, n_sid]), "val_i8": to_i8(fixture),
         "val_a1_i8": to_i8(decode(base + ".bed", n_iid, count_A1=True))}
    for dt, tag in ((np.float64, "f64"), (np.float32, "f32")):
        v, tr = std_py(val, Unit(), dt)
        g["unit_" + tag], g["unit_stats_" + tag] = v, tr.stats
        v, tr = std_py(val, Beta(1, 25), dt)
        g["beta_" + tag], g["beta_stats_" + tag] = v, tr.stats
    # trained: fit on iids 10.., apply to 0..9 (standardizer.py:31-42 doctest)
    for name, std in (("unit", Unit()), ("beta", Beta(1, 25))):
        _, tr = std_py(val[10:], std, np.float64)
        g[name + "_train_stats"] = tr.stats
        d = sd(np.array(val[:10], order="F"))
        d.standardize(tr, force_python_only=True)
        g[name + "_test"] = d.val
    # GRM (whole and blocked) + DiagKtoN, through the reference's own SnpKernel
    d = sd(np.array(val, order="F"))
    k_whole = d.read_kernel(Unit(), block_size=None, force_python_only=True).val
    k_block = d.read_kernel(Unit(), block_size=100, force_python_only=True).val
    assert np.abs(k_whole - k_block).max() < 1e-9
    g["K_unit"] = k_whole
    g["K_beta"] = d.read_kernel(Beta(1, 25), block_size=None, force_python_only=True).val
    kd = SnpKernel(d, Unit()).read(force_python_only=True)
    kd2, diag_tr = kd.standardize(DiagKtoN(), return_trained=True)
    g["diag_factor"] = np.array(diag_tr.factor)
    g["K_unit_diag"] = kd2.val
    np.savez_compressed(os.path.join(OUT, "n300.npz"), **g)

    # ------------------------------------------------------------------ snpgen / distributed X
    copy_triple(REF + "/tests/datasets/snpgen", "snpgen")
    sg = SnpGen(seed=0, iid_count=1000, sid_count=int(1e6), block_size=1000)[:, [0, 1, 200, 2200, 10]].read().val
    dec = decode(REF + "/tests/datasets/snpgen.bed", 1000)
    assert np.array_equal(sg, dec, equal_nan=True)
    g = {"val_i8": to_i8(sg)}
    for dt, tag in ((np.float64, "f64"), (np.float32, "f32")):
        v, tr = std_py(sg, Unit(), dt)
        g["unit_" + tag], g["unit_stats_" + tag] = v, tr.stats
        v, tr = std_py(sg, Beta(1, 25), dt)
        g["beta_" + tag], g["beta_stats_" + tag] = v, tr.stats
    np.savez_compressed(os.path.join(OUT, "snpgen.npz"), **g)

    copy_triple(REF + "/tests/datasets/distributed_bed_test1_X", "dist_x")
    dx = SnpGen(seed=0, iid_count=100, sid_count=100).read().val
    assert np.array_equal(dx, decode(REF + "/tests/datasets/distributed_bed_test1_X.bed", 100), equal_nan=True)
    g = {"val_i8": to_i8(dx)}
    for dt, tag in ((np.float64, "f64"), (np.float32, "f32")):
        v, tr = std_py(dx, Unit(), dt)
        g["unit_" + tag], g["unit_stats_" + tag] = v, tr.stats
    d = sd(np.array(dx, order="F"))
    g["K_unit"] = d.read_kernel(Unit(), force_python_only=True).val
    g["K_beta"] = d.read_kernel(Beta(1, 25), block_size=7, force_python_only=True).val
    np.savez_compressed(os.path.join(OUT, "dist_x.npz"), **g)

    # ------------------------------------------------------------------ toydata (500 x 10k)
    copy_triple(REF + "/pysnptools/examples/toydata.5chrom", "toydata")
    tv = decode(REF + "/pysnptools/examples/toydata.5chrom.bed", 500)
    t10 = np.load(REF + "/pysnptools/examples/toydata10.snp.npz", allow_pickle=False)["val"]
    assert np.array_equal(tv[:, :10], t10, equal_nan=True)
    kfix = np.load(REF + "/pysnptools/examples/toydata.kernel.npz", allow_pickle=False)["val"]
    shutil.copyfile(REF + "/pysnptools/examples/toydata.kernel.npz", os.path.join(DATA, "toydata.kernel.npz"))
    kref = sd(np.array(tv, order="F")).read_kernel(Unit(), block_size=1000, force_python_only=True).val
    assert np.abs(kref - kfix).max() < 1e-9
    np.savez_compressed(os.path.join(OUT, "toydata.npz"), K_rows=kfix[:64].copy(), K_diag=np.diag(kfix).copy(),
                        K_rowsum=kfix.sum(1), K00=np.array(kfix[0, 0]))

    # ------------------------------------------------------------------ writer-produced BEDs with N % 4 != 0
    # util/generate.py:207-240: gen1/gen4.bed were written by the reference (Bed.write of
    # snp_gen output, count_A1=False); they pin the encoder's bytes incl. the pad bits.
    from pysnptools.util.generate import snp_gen

    g = {}
    for name, kw in (("gen1", dict(fst=0, dfr=.5, iid_count=200, sid_count=20, maf_low=.05, seed=5)),
                     ("gen4", dict(fst=.1, dfr=.01, iid_count=200, sid_count=20, maf_low=.1, seed=5))):
        copy_triple(REF + "/tests/datasets/generate/" + name, name)
        sd_gen = snp_gen(**kw)
        assert np.array_equal(sd_gen.val, decode(REF + "/tests/datasets/generate/%s.bed" % name, sd_gen.iid_count),
                              equal_nan=True)
        g[name + "_val_i8"] = to_i8(sd_gen.val)
    np.savez_compressed(os.path.join(OUT, "generate.npz"), **g)

    # intersect_apply (util/__init__.py:18-173) on the reference's doctest inputs
    from pysnptools.snpreader import Pheno
    from pysnptools.util import intersect_apply, intersect_ids

    bed_iid = np.loadtxt(REF + "/tests/datasets/all_chr.maf0.001.N300.fam", dtype=str, usecols=(0, 1))
    pheno = Pheno(REF + "/tests/datasets/phenSynthFrom22.23.N300.randcidorder.txt", missing="").read()
    cov = Pheno(REF + "/tests/datasets/all_chr.maf0.001.covariates.N300.txt", missing="").read()
    rng = np.random.RandomState(1)
    drop = np.sort(rng.choice(300, 40, replace=False))
    sub_iid = np.delete(bed_iid, drop, axis=0)[::-1]
    g = {"bed_iid": bed_iid.astype("S"), "pheno_iid": pheno.iid.astype("S"), "pheno_val": pheno.val,
         "cov_iid": cov.iid.astype("S"), "cov_val": cov.val, "sub_iid": sub_iid.astype("S")}
    for tag, lists in (("a", [None, bed_iid, pheno.iid, cov.iid]), ("b", [sub_iid, bed_iid, pheno.iid]),
                       ("c", [pheno.iid, None, sub_iid])):
        g["ind_" + tag] = intersect_ids(lists)
        for sort in (True, False):
            outs = intersect_apply([None if x is None else (np.arange(len(x)), x) for x in lists],
                                   sort_by_dataset=sort)
            g["out_%s_%d" % (tag, sort)] = np.array([o[0] for o in outs if o is not None])
    np.savez_compressed(os.path.join(OUT, "intersect.npz"), **g)

    # DistributedBed written by the reference (distributedbed.py:285-300): 44 count_A1=True pieces
    dst = os.path.join(DATA, "distributed_bed_test1")
    if os.path.exists(dst):
        shutil.rmtree(dst)
    shutil.copytree(REF + "/tests/datasets/distributed_bed_test1", dst)
    for f in os.listdir(dst):
        os.chmod(os.path.join(dst, f), 0o644)

    # ------------------------------------------------------------------ edge matrices (kernelreader/test.py:56-111 style)
    g = {}
    np.random.seed(0)
    x0 = np.random.randint(3, size=[3, 20]).astype(np.float64)
    x1 = np.random.randint(3, size=[2, 20]).astype(np.float64)
    x0[:, 1] = 0          # SNC in training
    x0[0, 2] = np.nan     # missing
    x1[0, 2] = np.nan
    x0[:, 5] = np.nan     # all-missing column (Python-path semantics: NaN stats, zero column)
    g["x0"], g["x1"] = x0, x1
    for dt, tag in ((np.float64, "f64"), (np.float32, "f32")):
        for order in ("F", "C"):
            for name, std in (("unit", Unit()), ("beta", Beta(2, 10))):
                v, tr = std_py(x0, std, dt, order)
                key = "%s_%s_%s" % (name, tag, order)
                g[key + "_train"], g[key + "_stats"] = v, tr.stats
                d = sd(np.array(x1, dtype=dt, order=order))
                d.standardize(tr, force_python_only=True)
                g[key + "_apply"] = d.val
    # whole-matrix GRM on random ints (kernelreader/test.py:177-195)
    xr = np.random.randint(3, size=[7, 20]).astype(np.float64)
    xr[2, 3] = np.nan
    g["xr"] = xr
    for name, std in (("unit", Unit()), ("beta", Beta(1, 25))):
        d = sd(np.array(xr, order="F"))
        g["K_%s_xr" % name] = d.read_kernel(std, block_size=1, force_python_only=True).val
    np.savez_compressed(os.path.join(OUT, "edge.npz"), **g)
    print("goldens written to", OUT)


if __name__ == "__main__":
    main()
