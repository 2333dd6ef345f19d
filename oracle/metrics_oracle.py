"""ORACLE — test infrastructure only.  numpy/scipy restatement of the SOD evaluation metrics.

Only ``tests/`` may import this module, as the checker of ``s3od_amd.metrics`` (the HIP path in
``csrc/metrics.hip``); the product never routes through it.

Restates ``synth_sod/src/synth_sod/model_training/metrics.py``:
  * ``EvaluationMetrics.step``  :227-283  MAE (float64), MaxF / AvgF over the 255 float32
    thresholds of ``_eval_pr`` :316-327 (float32 prec/recall/F as the reference's tensors hold
    them), S-measure :229-245 / :256-272 with ``_S_object`` :329-344, ``_S_region`` :346-356,
    ``_centroid`` :358-378, ``_ssim`` :405-424
  * ``EMeasure``               :14-137   changeable E-measure from the uint8 histograms (the curve
    mean is what ``get_metrics`` reports)
  * ``WeightedFMeasure``       :140-210  with scipy.ndimage's exact EDT (``return_indices``) and
    7x7 sigma-5 ``convolve`` — the reference's own dependency, used here unchanged.

Parity pin: ``tests/golden/metrics.npz`` (``make_golden.py --metrics`` ran the reference's
``EvaluationMetrics(device=None)`` on CPU); ``tests/test_oracle_golden.py`` checks this
restatement against it.  Where the reference computes in float32 (pred means/std, w1..w4, the
quadrant SSIM's pred terms) this restatement uses float64; the golden test bounds the gap.
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import convolve, distance_transform_edt

EPS = np.spacing(1)
KEYS = ("mae", "max_f", "avg_f", "s_score", "em", "wfm")


def thresholds():
    """torch.linspace(0, 1 - 1e-10, 255) in float32 (1 - 1e-10 rounds to 1.0f)."""
    import torch
    return torch.linspace(0, 1 - 1e-10, 255).numpy()


def gauss7():
    """WeightedFMeasure.matlab_style_gauss2D((7, 7), 5) (metrics.py:193-205)."""
    m = n = 3.0
    y, x = np.ogrid[-m:m + 1, -n:n + 1]
    h = np.exp(-(x * x + y * y) / (2 * 5.0 * 5.0))
    h[h < np.finfo(h.dtype).eps * h.max()] = 0
    return h / h.sum()


def _pr_f(pred, gt):
    thr = thresholds()
    ysum = gt.sum()
    f = np.empty(255, np.float32)
    for i, t in enumerate(thr):
        sel = pred >= t
        tp = gt[sel].sum()
        cnt = np.float32(sel.sum())
        den = np.float64(cnt) if cnt != 0 else np.float64(np.float32(1e-20))
        prec, rec = np.float32(tp / den), np.float32(tp / (ysum + 1e-20))
        with np.errstate(invalid="ignore", divide="ignore"):
            v = (np.float32(1.3) * prec) * rec / (np.float32(0.3) * prec + rec)
        f[i] = 0.0 if v != v else v
    return f


def _object(vals):
    with np.errstate(invalid="ignore", divide="ignore"):
        x = vals.mean() if vals.size else np.nan
        sd = vals.std(ddof=1) if vals.size > 1 else np.nan
        return 2.0 * x / (x * x + 1.0 + sd + 1e-20)


def _ssim(p, m):
    N = p.size
    with np.errstate(invalid="ignore", divide="ignore"):
        x, y = (p.mean(), m.mean()) if N else (np.nan, np.nan)
        sx2 = ((p - x) ** 2).sum() / (N - 1 + 1e-20)
        sy2 = ((m - y) ** 2).sum() / (N - 1 + 1e-20)
        sxy = ((p - x) * (m - y)).sum() / (N - 1 + 1e-20)
        a = 4 * x * y * sxy
        b = (x * x + y * y) * (sx2 + sy2)
        if a != 0:
            return a / (b + 1e-20)
        return 1.0 if b == 0 else 0.0


def s_measure(pred, gt):
    """S-measure with the reference's special cases; gt is binarised at 0.5 only in the general case."""
    p = pred.astype(np.float64)
    y = gt.mean()
    if y == 0:
        return float(1.0 - p.mean())
    if y == 1:
        return float(p.mean())
    m = (gt >= 0.5).astype(np.float64)
    u = m.mean()
    o_fg = _object(p[m == 1])
    o_bg = _object((1 - pred[m == 0]).astype(np.float64))
    so = u * o_fg + (1 - u) * o_bg
    H, W = m.shape
    if m.sum() == 0:
        X, Y = int(np.round(W / 2)), int(np.round(H / 2))
    else:
        X = int(np.round((m.sum(0) * np.arange(W)).sum() / m.sum()))
        Y = int(np.round((m.sum(1) * np.arange(H)).sum() / m.sum()))
    area = H * W
    w1, w2, w3 = X * Y / area, (W - X) * Y / area, X * (H - Y) / area
    w4 = 1 - w1 - w2 - w3
    sr = (w1 * _ssim(p[:Y, :X], m[:Y, :X]) + w2 * _ssim(p[:Y, X:], m[:Y, X:]) +
          w3 * _ssim(p[Y:, :X], m[Y:, :X]) + w4 * _ssim(p[Y:, X:], m[Y:, X:]))
    q = 0.5 * so + 0.5 * sr
    return 0.0 if q < 0 else float(q)


def e_measure(pred, gt):
    g = gt > 0
    size = g.size
    fgn = np.count_nonzero(g)
    q = (pred * np.float32(255)).astype(np.uint8)
    bins = np.linspace(0, 256, 257)
    ff = np.cumsum(np.flip(np.histogram(q[g], bins=bins)[0]))
    fb = np.cumsum(np.flip(np.histogram(q[~g], bins=bins)[0]))
    pf = ff + fb
    pb = size - pf
    if fgn == 0:
        s = pb
    elif fgn == size:
        s = pf
    else:
        bf = fgn - ff
        bb = pb - bf
        mp, mg = pf / size, fgn / size
        s = 0
        for part, (a, b) in zip((ff, fb, bf, bb), ((1 - mp, 1 - mg), (1 - mp, -mg), (-mp, 1 - mg), (-mp, -mg))):
            al = 2 * (a * b) / (a ** 2 + b ** 2 + EPS)
            s = s + (al + 1) ** 2 / 4 * part
    return float(np.mean(s / (size - 1 + EPS)))


def weighted_f(pred, gt):
    g = gt > 0
    if not g.any():
        return 0.0
    dst, idx = distance_transform_edt(g == 0, return_indices=True)
    E = np.abs(pred - g)
    Et = E.copy()
    Et[g == 0] = Et[idx[0][g == 0], idx[1][g == 0]]
    EA = convolve(Et, weights=gauss7(), mode="constant", cval=0)
    mn = np.where(g & (EA < E), EA, E)
    B = np.where(g == 0, 2 - np.exp(np.log(0.5) / 5 * dst), np.ones_like(g))
    Ew = mn * B
    tpw = np.sum(g) - np.sum(Ew[g == 1])
    fpw = np.sum(Ew[g == 0])
    R = 1 - np.mean(Ew[g == 1])
    P = tpw / (tpw + fpw + EPS)
    return float(2 * R * P / (R + P + EPS))


def step(pred: np.ndarray, gt: np.ndarray, sm_only: bool = False) -> dict:
    """One EvaluationMetrics.step on (pred float32 [H,W], gt {0,1} [H,W]) -> per-image values."""
    pred = np.asarray(pred, np.float32)
    gt = np.asarray(gt, np.float64)
    s = s_measure(pred, gt)
    if sm_only:
        return {"s_score": s}
    f = _pr_f(pred, gt)
    gb = (gt >= 0.5) if not (gt.mean() in (0.0, 1.0)) else gt > 0
    return {"mae": float(np.mean(np.abs(pred.astype(np.float64) - gt))), "max_f": float(f.max()),
            "avg_f": float(f.astype(np.float64).mean()), "s_score": s, "em": e_measure(pred, gb.astype(np.float64)),
            "wfm": weighted_f(pred, gb.astype(np.float64))}


def edt_nearest(fg: np.ndarray):
    """Pure-Python restatement of the distance-transform algorithm csrc/metrics.hip runs (column pass:
    nearest foreground row, ties -> lower row; row pass: Maurer lower envelope with strict remove /
    strict advance).  Returns (row index, column index) of the nearest foreground pixel per pixel;
    tests check it equals scipy's ``distance_transform_edt(fg == 0, return_indices=True)`` choice.
    Small images only (Python loops)."""
    H, W = fg.shape
    feat = np.full((H, W), -1)
    for x in range(W):
        rows = np.nonzero(fg[:, x])[0]
        for y in range(H):
            if rows.size:
                d = np.abs(rows - y)
                feat[y, x] = rows[d == d.min()].min()
    iy = np.full((H, W), -1); ix = np.full((H, W), -1)
    for y in range(H):
        g = []
        for x in range(W):
            if feat[y, x] < 0:
                continue
            dw = (feat[y, x] - y) ** 2
            while len(g) >= 2:
                (u, du), (v, dv) = g[-2], g[-1]
                a, b, c = v - u, x - v, x - u
                if c * dv - b * du - a * dw - a * b * c > 0:
                    g.pop()
                else:
                    break
            g.append((x, dw))
        if not g:
            continue
        l = 0
        for x in range(W):
            while l < len(g) - 1 and g[l][1] + (g[l][0] - x) ** 2 > g[l + 1][1] + (g[l + 1][0] - x) ** 2:
                l += 1
            ix[y, x] = g[l][0]; iy[y, x] = feat[y, g[l][0]]
    return iy, ix
