"""Numerics study (CPU, NumPy + torch's float8_e4m3fn): can the fp16x2 GRM's correction terms
a0*b1 + a1*b0 run on the fp8 MFMA (2x the fp16 rate) without breaking f32-level K?

Emulates, in f64 accumulation (so only the representation error shows), on SnpGen-shaped data
(snpgen.py:140-151 MAF curve, --miss missing), K rows 0..R-1 of Unit-standardized Z (f32 LUT):
  exact3 : a0 b0 + a0 b1 + a1 b0                      (the shipped fp16x2 scheme)
  fp8    : a0 b0 + [e4m3(a0/s0) e4m3(b1/s1) + e4m3(a1/s1) e4m3(b0/s0)] s0 s1
           (s0, s1 = power-of-two scales per 32-SNP stage, or per launch with --global-scale)
against the f64 K; prints max|dK| / max diag per M.
"""
import argparse
import json

import numpy as np
import torch


def snpgen_mafs(rng, n, m):
    x = np.logspace(np.log10(0.1 / n), np.log10(0.5), 100)
    w = x ** -0.6482 * np.exp(-8.4979 * x)
    return rng.choice(x, size=m, p=w / w.sum())


def e4m3(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(torch.float8_e4m3fn).to(torch.float32).numpy().astype(np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--ms", default="1015,4096,16384,62500")
    ap.add_argument("--miss", type=float, default=0.218)
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--global-scale", action="store_true")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    n, R = a.n, a.rows
    for m in [int(v) for v in a.ms.split(",")]:
        maf = snpgen_mafs(rng, n, m)
        G = rng.binomial(2, maf, size=(n, m)).astype(np.float64)
        miss = rng.random((n, m)) < a.miss
        G[miss] = np.nan
        obs = ~miss
        cnt = obs.sum(0)
        mean = np.nansum(G, 0) / np.maximum(cnt, 1)
        std = np.sqrt(np.nansum(G * G, 0) / np.maximum(cnt, 1) - mean ** 2)
        std[std <= 0] = np.inf
        Z = ((G - mean) / std)
        Z[miss] = 0.0
        Z = Z.astype(np.float32).astype(np.float64)  # the f32 LUT values
        Kref = Z[:R] @ Z.T
        scale = np.abs(np.diag(Kref[:, :R])).max()
        a0 = Z.astype(np.float16).astype(np.float64)
        a1 = (Z - a0).astype(np.float16).astype(np.float64)
        out = {"n": n, "m": m, "miss": a.miss}
        K3 = a0[:R] @ a0.T + a0[:R] @ a1.T + a1[:R] @ a0.T
        out["exact3"] = float(np.abs(K3 - Kref).max() / scale)
        # per-stage (32 SNPs) or global power-of-two scales so the stage's largest |value| <= 448
        def scales(v):
            if a.global_scale:
                mx = np.full(m, np.abs(v).max())
            else:
                mx = np.repeat([np.abs(v[:, s:s + 32]).max() for s in range(0, m, 32)], 32)[:m]
            e = np.ceil(np.log2(np.maximum(mx, 1e-30) / 448.0))
            return np.exp2(e)
        s0, s1 = scales(a0), scales(a1)
        q0, q1 = e4m3(a0 / s0) * s0, e4m3(a1 / s1) * s1
        K8 = a0[:R] @ a0.T + q0[:R] @ q1.T + q1[:R] @ q0.T
        out["fp8_corr"] = float(np.abs(K8 - Kref).max() / scale)
        out["fp8_corr_diag_rel"] = float(np.max(np.abs(np.diag(K8[:, :R]) - np.diag(Kref[:, :R])) / np.abs(np.diag(Kref[:, :R]))))
        K1 = a0[:R] @ a0.T
        out["fp16_only"] = float(np.abs(K1 - Kref).max() / scale)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
