"""Digitize the data points of the Threshold notebook's fit plots (test infrastructure; CPU only).

``.ipynb_checkpoints/Threshold-checkpoint.ipynb`` cells 16, 20 and 25 print one (A, p_c) fit per round
count (the notebook pin's 15 points, tests/notebook_pin.py:PRINTED) AND draw, per fit, the plot of
``ThresholdEst(..., if_plot=True)`` (notebook lines 71-120): per code the data as diamonds (``'D'``,
colours C0 / C1 / C2) at ``sweep_p_list`` against ``sweep_pl_list`` = the notebook's WER + 1e-6, and the
fitted lines, on log-log axes.  Those diamonds are the only per-point outputs of the real ``ldpc`` /
``bposd`` decoders the reference holds.  This script reads the embedded PNGs (stdlib zlib + numpy: no
image library), and for each plot:

* finds the axes frame (the long dark spines) and the y tick marks left of the left spine (majors
  one pixel longer than minors); the tick values follow the log-axis pattern (majors at decades, minors
  at 2..9 x decade), the top tick's place in that pattern chosen by least squares, so y = a + b log10(v)
  up to an unknown integer decade;
* finds each colour's diamonds as the connected components of its fully-coloured 3 x 3 cores (the
  1.5-px fit lines have none), 6 per code, and refines each centre to the coverage-weighted centroid of
  its colour within 3.5 px (coverage = blend fraction of the colour over white);
* calibrates x by the 6 diamond columns against the cell's known p (log10, least squares);
* fixes the decade by refitting the notebook's own ThresholdEst (tests/notebook_pin.threshold_est) on the
  digitized WERs and taking the integer decade shift whose (A, p_c) is closest to the printed pair (one
  plot, cell 25 R = 6, spans 12 decades with equally spaced ticks and no sub-ticks: its decades per tick
  are then open too and its scale is marked unpinned).

Output: tests/golden/notebook_plot_points.json (per cell and round count: p, the digitized WER per code
and p, the pixel residuals of the tick fit, and the refit (A, p_c) beside the printed pair).

    python tools/notebook_digitize.py [reference notebook] [out.json]
"""
import base64
import json
import math
import os
import struct
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import notebook_pin as nbp  # noqa: E402

NB = "/root/reference/.ipynb_checkpoints/Threshold-checkpoint.ipynb"
COLOURS = [(31, 119, 180), (255, 127, 14), (44, 160, 44)]  # matplotlib C0, C1, C2


def png_decode(b):
    """8-bit RGB / RGBA PNG -> uint8 [H, W, 3] (filters 0-4)."""
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    while pos < len(b):
        ln, = struct.unpack(">I", b[pos:pos + 4])
        typ, data = b[pos + 4:pos + 8], b[pos + 8:pos + 8 + ln]
        pos += 12 + ln
        if typ == b"IHDR":
            w, h, bd, ct = struct.unpack(">IIBB", data[:10])
        elif typ == b"IDAT":
            idat += data
    assert bd == 8 and ct in (2, 6)
    ch = 4 if ct == 6 else 3
    raw = zlib.decompress(idat)
    stride = w * ch
    out = np.zeros((h, stride), np.int32)
    prev = np.zeros(stride, np.int32)
    p = 0
    for y in range(h):
        f = raw[p]
        line = np.frombuffer(raw[p + 1:p + 1 + stride], np.uint8).astype(np.int32)
        p += 1 + stride
        if f == 0:
            cur = line.copy()
        elif f == 2:
            cur = (line + prev) & 255
        else:
            cur = np.zeros(stride, np.int32)
            for i in range(stride):
                a = cur[i - ch] if i >= ch else 0
                up = prev[i]
                c = prev[i - ch] if i >= ch else 0
                if f == 1:
                    cur[i] = (line[i] + a) & 255
                elif f == 3:
                    cur[i] = (line[i] + ((a + up) >> 1)) & 255
                else:
                    pa, pb, pc = abs(up - c), abs(a - c), abs(a + up - 2 * c)
                    pr = a if (pa <= pb and pa <= pc) else (up if pb <= pc else c)
                    cur[i] = (line[i] + pr) & 255
        out[y] = cur
        prev = cur
    return out.reshape(h, w, ch)[..., :3].astype(np.int32)


def components(mask):
    H, W = mask.shape
    lab = -np.ones(mask.shape, int)
    out = []
    for y, x in zip(*np.nonzero(mask)):
        if lab[y, x] >= 0:
            continue
        st, pts = [(y, x)], []
        lab[y, x] = len(out)
        while st:
            a, b = st.pop()
            pts.append((a, b))
            for da in (-1, 0, 1):
                for db in (-1, 0, 1):
                    c, d = a + da, b + db
                    if 0 <= c < H and 0 <= d < W and mask[c, d] and lab[c, d] < 0:
                        lab[c, d] = len(out)
                        st.append((c, d))
        out.append(np.array(pts, float))
    return out


def y_calibration(img):
    """[(a, b, residual_px)], frame: pixel row = a + b * (log10 v - E) for an unknown integer E; several
    candidates when the tick pattern leaves the decades per tick open."""
    H, W, _ = img.shape
    dark = img.sum(2) < 450
    xs = [x for x in range(W) if dark[:, x].sum() > 0.6 * H]
    ys = [y for y in range(H) if dark[y].sum() > 0.6 * W]
    xl, yt, yb = min(xs), min(ys), max(ys)
    ticks = [(y, bool(dark[y, xl - 3])) for y in range(yt, yb + 1) if dark[y, xl - 1] and dark[y, xl - 2]]
    best = None
    for k0 in range(1, 10):  # the top tick's place in the decade pattern (1 = a major)
        vals, k, e, ok = [], k0, 0, True
        for _, major in ticks:
            if (k == 1) != major:
                ok = False
                break
            vals.append(e + math.log10(k))
            k -= 1  # next tick down
            if k == 0:
                k, e = 9, e - 1
            elif k == 1 and False:
                pass
        if not ok or len(vals) < 3:
            continue
        yv = np.array([t[0] for t in ticks], float)
        A = np.vstack([np.ones(len(vals)), vals]).T
        sol, *_ = np.linalg.lstsq(A, yv, rcond=None)
        res = float(np.sqrt(np.mean((A @ sol - yv) ** 2)))
        if best is None or res < best[2]:
            best = (float(sol[0]), float(sol[1]), res)
    if best is not None:
        return [best], (xl, yt, yb)
    # many decades: equally spaced ticks without 2..9 sub-ticks (matplotlib's majors every 1, 2 or 3
    # decades when the axis spans many): one candidate per spacing, decided by the refit
    yv = np.array([t[0] for t in ticks], float)
    sp = np.diff(yv)
    assert len(yv) >= 3 and np.ptp(sp) <= 2.0, "no consistent tick pattern"
    cands = []
    for step in (1, 2, 3):
        vals = -step * np.arange(len(yv), dtype=float)
        A = np.vstack([np.ones(len(vals)), vals]).T
        sol, *_ = np.linalg.lstsq(A, yv, rcond=None)
        cands.append((float(sol[0]), float(sol[1]), float(np.sqrt(np.mean((A @ sol - yv) ** 2)))))
    return cands, (xl, yt, yb)


def markers(img, colour, n_expect=6):
    H, W, _ = img.shape
    c = np.array(colour)
    m = np.abs(img - c).sum(2) <= 12
    core = m.copy()
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            core[1:-1, 1:-1] &= m[1 + dy:H - 1 + dy, 1 + dx:W - 1 + dx]
    # coverage of the colour over white, per pixel: the mean blend fraction of the channels that differ
    ch = [i for i in range(3) if c[i] < 250]
    cov = np.clip(np.mean([(255 - img[..., i]) / (255 - c[i]) for i in ch], axis=0), 0, 1)
    # pixels closer to another plot colour than to this one carry no coverage of it
    for o in COLOURS:
        if o != tuple(colour):
            cov[np.abs(img - np.array(o)).sum(2) < np.abs(img - c).sum(2)] = 0
    cov[(img.max(2) - img.min(2) < 24) & (img.sum(2) < 450)] = 0  # grey / black (axes, text)
    # diamonds, not stretches of the 1.5-px fit line (which can overlap itself: the notebook draws it
    # through an unordered set of p): a diamond fills its |dx| + |dy| <= 3 template, a line about half
    def fill(p):
        y0, x0 = int(round(p[:, 0].mean())), int(round(p[:, 1].mean()))
        if not (4 <= y0 < H - 4 and 4 <= x0 < W - 4):
            return 0.0
        Y, X = np.mgrid[y0 - 4:y0 + 5, x0 - 4:x0 + 5]
        t = (np.abs(Y - y0) + np.abs(X - x0)) <= 3
        return float(cov[Y, X][t].mean())
    cs = [p for p in components(core) if len(p) >= 2 and fill(p) >= 0.8]
    cs.sort(key=lambda p: p[:, 1].mean())
    assert len(cs) <= n_expect, f"colour {colour}: {len(cs)} diamonds"
    out = []
    for p in cs:
        y0, x0 = p[:, 0].mean(), p[:, 1].mean()
        for _ in range(3):
            Y, X = np.mgrid[int(y0) - 4:int(y0) + 5, int(x0) - 4:int(x0) + 5]
            w = cov[Y, X] * (((Y - y0) ** 2 + (X - x0) ** 2) <= 3.5 ** 2)
            y0, x0 = float((w * Y).sum() / w.sum()), float((w * X).sum() / w.sum())
        out.append((x0, y0))
    return out, cov


def occluded_marker(img, cov, colour, x_col, y_hint, r):
    """Centre of a diamond of ``colour`` partly hidden under a later-drawn marker, near (x_col, y_hint):
    the sub-pixel centre whose diamond template (|dx| + |dy| <= r) covers the most visible pixels of the
    colour and the fewest background (white) pixels; pixels of the other colours are neutral (they may
    hide it)."""
    white = img.min(2) > 235
    mine = cov > 0.5
    best = None
    for yc in np.arange(y_hint - 9, y_hint + 9.01, 0.25):
        for xc in np.arange(x_col - 1.0, x_col + 1.01, 0.25):
            Y, X = np.mgrid[int(yc) - 7:int(yc) + 8, int(xc) - 7:int(xc) + 8]
            inside = (np.abs(Y - yc) + np.abs(X - xc)) <= r
            score = float(mine[Y, X][inside].sum()) - 2.0 * float(white[Y, X][inside].sum()) \
                - float(mine[Y, X][~inside & ((np.abs(Y - yc) + np.abs(X - xc)) <= r + 2.5)].sum())
            if best is None or score > best[0]:
                best = (score, xc, yc)
    return best[1], best[2]


def digitize(cell, k, png):
    img = png_decode(png)
    cands, frame = y_calibration(img)
    P = nbp.cell_p_list(cell)
    found = [markers(img, col) for col in COLOURS]
    full = [f[0] for f in found if len(f[0]) == len(P)]
    assert full, "no colour with every diamond visible"
    xcols = np.array([[x for x, _ in pc] for pc in full]).mean(0)
    r = 4.0  # diamond half-diagonal, px (markersize 6 at 72 dpi)
    pts, occl = [], []
    for ci, (pc, cov) in enumerate(found):
        if len(pc) == len(P):
            pts.append(pc)
            occl.append([False] * len(P))
            continue
        # a diamond hidden under a later colour's: the columns this colour lacks
        have = [int(np.argmin(np.abs(xcols - x))) for x, _ in pc]
        row, flags = [], []
        for j in range(len(P)):
            if j in have:
                row.append(pc[have.index(j)])
                flags.append(False)
            else:
                ys = [f[0][[int(np.argmin(np.abs(xcols - x))) for x, _ in f[0]].index(j)][1] for f in found
                      if j in [int(np.argmin(np.abs(xcols - x))) for x, _ in f[0]] and f is not found[ci]]
                row.append(occluded_marker(img, cov, COLOURS[ci], xcols[j], float(np.mean(ys)), r))
                flags.append(True)
        pts.append(row)
        occl.append(flags)
    kx, x0 = np.polyfit(np.log10(P), xcols, 1)
    xres = float(np.sqrt(np.mean((x0 + kx * np.log10(P) - xcols) ** 2)))
    R = nbp.CELLS[cell]["rounds"][k]
    A0, pc0, line = nbp.PRINTED[cell][R]
    best = None
    for a, b, res in cands:
        logv = np.array([[(y - a) / b for _, y in pc_] for pc_ in pts])  # log10(WER + 1e-6) - E
        for E in range(-12, 1):
            wer = 10.0 ** (logv + E) - 1e-6
            if np.any(wer <= 0):
                continue
            try:
                A, pc = nbp.threshold_est(P, wer)
            except (RuntimeError, ValueError, TypeError):
                continue
            if not (A > 0 and pc > 0):
                continue
            d = abs(math.log(A / A0)) + abs(math.log(pc / pc0))
            if best is None or d < best[0]:
                best = (d, E, A, pc, wer, a, b, res)
    assert best is not None
    _, E, A, pc, wer, a, b, res = best
    return {"cell": cell, "rounds": R, "plot": k, "notebook_line": line, "p": [float(x) for x in P],
            "wer": [[float(v) for v in row] for row in wer],
            "pixels": [[[round(x, 2), round(y, 2)] for x, y in pc_] for pc_ in pts], "occluded": occl,
            "y_axis": {"a": a, "b_px_per_decade": b, "tick_rms_px": res, "decade": E,
                       # equally spaced ticks without 2..9 sub-ticks: the decades per tick come from the
                       # refit alone (the tick labels are not read), so this plot's scale is not pinned
                       "tick_pattern": "log-subticks" if len(cands) == 1 else "equally-spaced"},
            "x_rms_px": xres, "refit": {"A": A, "p_c": pc}, "printed": {"A": A0, "p_c": pc0}}


def main():
    nb_path = sys.argv[1] if len(sys.argv) > 1 else NB
    out_path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "tests", "golden", "notebook_plot_points.json")
    nb = json.load(open(nb_path))
    res = []
    for cell in (16, 20, 25):
        imgs = [o["data"]["image/png"] for o in nb["cells"][cell]["outputs"] if "data" in o and "image/png" in o["data"]]
        assert len(imgs) == len(nbp.CELLS[cell]["rounds"]), (cell, len(imgs))
        for k, b64 in enumerate(imgs):
            r = digitize(cell, k, base64.b64decode(b64))
            res.append(r)
            print(f"cell {cell} R{r['rounds']:2d}: ticks rms {r['y_axis']['tick_rms_px']:.2f} px, x rms {r['x_rms_px']:.2f} px, "
                  f"{r['y_axis']['b_px_per_decade']:.1f} px/decade, decade {r['y_axis']['decade']}; refit A {r['refit']['A']:.4g} "
                  f"p_c {r['refit']['p_c']:.4g} vs printed {r['printed']['A']:.4g} {r['printed']['p_c']:.4g}", flush=True)
    meta = {"what": __doc__.strip().splitlines()[0], "source": ".ipynb_checkpoints/Threshold-checkpoint.ipynb cells 16, 20, 25 "
            "(embedded PNG outputs of ThresholdEst(if_plot=True), notebook lines 71-120)",
            "generator": "tools/notebook_digitize.py", "plots": res}
    with open(out_path, "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
