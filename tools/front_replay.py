"""Replay a GPU front that failed the front check (dense_gpu.hip, AA_FRONT_DUMP=<dir>).

The backend writes, for a front whose first factorization failed a check, the kept assembled
front and the first attempt's outputs (column-major doubles):
    front<s>_f<f>_p<p>_kept.bin        f x f   the assembled front (lower triangle used)
    front<s>_f<f>_p<p>_first_F.bin     f x f   L11 | L21 | Schur complement, in place
    front<s>_f<f>_p<p>_first_Linv.bin  p x p   L11^-1
    front<s>_f<f>_p<p>_first_M.bin     nb x p  M = L21 L11^-1
This factors the kept copy on the host (numpy) and names the outputs of the first attempt that
differ, with the first differing entries -- which kernel wrote wrong numbers (potrf: L11; trsm:
L21; syrk: the Schur complement; trtri: Linv; trmm: M).

    python tools/front_replay.py gpurun_out/front_dump/front12_f2844_p1422_kept.bin
"""
from __future__ import annotations

import json
import os
import re
import sys

import numpy as np

TOL = 1e-8


def _load(path, rows, cols):
    a = np.fromfile(path, dtype=np.float64)
    if a.size != rows * cols:
        raise ValueError(f"{path}: {a.size} doubles, expected {rows} x {cols}")
    return a.reshape(cols, rows).T   # column-major


def _cmp(name, got, want, lower=False):
    if lower:
        mask = np.tril(np.ones(got.shape, bool))
        got, want = np.where(mask, got, 0.0), np.where(mask, want, 0.0)
    scale = max(np.abs(want).max(), 1e-300)
    diff = np.abs(got - want)
    diff[~np.isfinite(got)] = np.inf
    dev = float(diff.max() / scale)
    idx = np.argwhere(diff > TOL * scale)
    out = {"output": name, "shape": list(got.shape), "rel_dev": dev, "n_wrong": int(len(idx)),
           "first_wrong": [[int(i), int(j), float(got[i, j]), float(want[i, j])] for i, j in idx[:5]]}
    if len(idx):   # where: bounding box and the 64 x 64 tiles holding wrong entries (a kernel's blocks)
        out["rows"] = [int(idx[:, 0].min()), int(idx[:, 0].max())]
        out["cols"] = [int(idx[:, 1].min()), int(idx[:, 1].max())]
        tiles, cnt = np.unique(idx // 64, axis=0, return_counts=True)
        out["tiles64"] = [[int(a), int(b), int(c)] for (a, b), c in zip(tiles[:40], cnt[:40])]
        out["n_tiles64"] = int(len(tiles))
    return out


def replay(kept_path: str) -> dict:
    m = re.search(r"front(\d+)_f(\d+)_p(\d+)_kept\.bin$", os.path.basename(kept_path))
    if not m:
        raise ValueError("expected a front<s>_f<f>_p<p>_kept.bin file")
    s, f, p = (int(x) for x in m.groups())
    nb = f - p
    base = kept_path[: -len("kept.bin")]
    K = _load(kept_path, f, f)
    K = np.tril(K) + np.tril(K, -1).T
    out = {"front": s, "order": f, "pivots": p, "kept_nonfinite": int((~np.isfinite(K)).sum())}
    try:
        L11 = np.linalg.cholesky(K[:p, :p])
        out["kept_factors"] = True
    except np.linalg.LinAlgError:
        out["kept_factors"] = False
        return out
    Linv = np.linalg.inv(L11)
    L21 = K[p:, :p] @ Linv.T
    S = K[p:, p:] - L21 @ L21.T
    F = _load(base + "first_F.bin", f, f)
    res = [_cmp("first_F[L11] (potrf)", F[:p, :p], L11, lower=True)]
    if nb:
        res.append(_cmp("first_F[L21] (trsm)", F[p:, :p], L21))
        res.append(_cmp("first_F[S] (syrk)", F[p:, p:], S, lower=True))
    res.append(_cmp("first_Linv (trtri)", _load(base + "first_Linv.bin", p, p), Linv, lower=True))
    if nb:
        res.append(_cmp("first_M (trmm)", _load(base + "first_M.bin", nb, p), L21 @ Linv))
    out["outputs"] = res
    out["differ"] = sorted({r["output"].split("[")[0].split(" ")[0] for r in res if r["rel_dev"] > TOL})
    return out


if __name__ == "__main__":
    for pth in sys.argv[1:]:
        print(json.dumps(replay(pth), indent=1))
