"""spans_check.py (analysis only, not product, not test): a numpy restatement of
tile_row_spans (gsr_kernels.hip) on the oracle's preprocess records.  For each scene it
prints the fraction of (tile, splat) rect pairs the spans keep and the largest alpha any
DROPPED pair reaches on an in-box pixel of its tile (must stay < 1e-3: the drop is then
invisible).  `python tools/sim/spans_check.py c1` (config 1, four cameras) or `c2`
(config 2; needs /tmp/sim_1000000.ply from tools/sim/sim_blend.py)."""
import os, sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import gaussianrenderer_amd as gsr, _oracle as orc
from test_gpu_parity import rect_pairs, max_alpha_on_tiles, CAMS, cam_for
f32 = np.float32
def spans_np(want, W, H):
    v = want["status"] == 2
    n = len(want)
    cx = want["px_x"].astype(f32); cy = want["px_y"].astype(f32)
    a, b, c, e = [want["inv_covar"][:, i].astype(f32) for i in range(4)]
    op = want["opacity"].astype(f32)
    with np.errstate(all="ignore"):
        h = f32(0.5) * (b + c)
        pd = (a > 0) & (e > 0) & ((a * e - h * h) > f32(1e-4) * (a * e))
        cut = (np.log2(op * f32(1000)) * f32(1.38629436111989061)) * f32(1.00001) + f32(1e-3)
        S = np.abs(a) + np.abs(b) + np.abs(c) + np.abs(e)
        ok = pd & np.isfinite(cut) & np.isfinite(S) & v
        det = a * e - h * h
        ax0, ay0, ax1, ay1 = [want["aabb"][:, i].astype(np.int64) for i in range(4)]
        M = np.maximum(np.maximum(np.abs(ax0.astype(f32) - cx), np.abs(ax1.astype(f32) - cx)), np.maximum(np.abs(ay0.astype(f32) - cy), np.abs(ay1.astype(f32) - cy)))
        C = cut + (f32(4e-6) * S * M * M + f32(1e-3))
        rdet = f32(1) / det; ra = f32(1) / a
        xr = np.sqrt(C * e * rdet); ym = np.sqrt(C * a * rdet); yr = -h * xr * (f32(1) / e)
        k = a * e * rdet
        rel = np.sqrt(f32(6e-7) * (k + f32(1))) + f32(1e-4)
        padx = f32(1 / 64) + rel * xr; ymp = ym * (f32(1) + rel) + f32(1 / 64)
        aC = a * C
    tx, ty = (W + 15) // 16, (H + 15) // 16
    tx0 = ax0 // 16; tx1 = np.minimum(tx - 1, ax2 := ax1 // 16); ty0 = ay0 // 16; ty1 = np.minimum(ty - 1, ay1 // 16)
    w = tx1 - tx0 + 1
    code = np.zeros(n, np.uint32)
    for r in range(4):
        tyr = ty0 + r
        act = ok & (tyr <= ty1)
        y0 = np.maximum(tyr * 16, ay0); y1 = np.minimum(tyr * 16 + 15, ay1)
        with np.errstate(all="ignore"):
            dy0 = y0.astype(f32) - cy; dy1 = y1.astype(f32) - cy
            inr = ~((dy0 > ymp) | (dy1 < -ymp))
            u0 = np.minimum(np.maximum(dy0, -ym), ym); u1 = np.minimum(np.maximum(dy1, -ym), ym)
            inR = (yr >= u0) & (yr <= u1)
            uR = np.where(yr < u0, u0, u1)
            R = np.where(inR, xr, (-h * uR + np.sqrt(np.maximum(aC - det * uR * uR, f32(0)))) * ra)
            inL = (-yr >= u0) & (-yr <= u1)
            uL = np.where(-yr < u0, u0, u1)
            L = np.where(inL, -xr, (-h * uL - np.sqrt(np.maximum(aC - det * uL * uL, f32(0)))) * ra)
            xl = np.maximum(cx + L - padx, ax0.astype(f32)); xh = np.minimum(cx + R + padx, ax1.astype(f32))
            good = inr & (xl <= xh)
            c0 = np.where(good, np.maximum(tx0, np.floor(xl * f32(1 / 16)).astype(np.int64)), tx1 + 1)
            c1 = np.where(good, np.minimum(tx1, np.floor(xh * f32(1 / 16)).astype(np.int64)), tx0 - 1)
        empty = c0 > c1
        sl = np.where(empty, np.minimum(w, 3), np.minimum(c0 - tx0, 3)); sr = np.where(empty, np.minimum(w, 3), np.minimum(tx1 - c1, 3))
        code |= np.where(act, (sl | (sr << 2)).astype(np.uint32) << np.uint32(4 * r), 0).astype(np.uint32)
    return code, tx0, tx1, ty0
def listed(full, code, tx0, tx1, ty0, W):
    tx = (W + 15) // 16
    tile = (full >> np.uint64(32)).astype(np.int64); idx = (full & np.uint64(0xFFFFFFFF)).astype(np.int64)
    col = tile % tx; row = tile // tx
    ro = row - ty0[idx]
    sp = np.where(ro < 4, (code[idx] >> (4 * np.minimum(ro, 3)).astype(np.uint32)) & 0xf, 0)
    c0 = tx0[idx] + (sp & 3); c1 = tx1[idx] - (sp >> 2)
    return (col >= c0) & (col <= c1)
cfg = sys.argv[1]
if cfg == "c1":
    p = "/tmp/c1.ply"; soa = gsr.read_ply(p); W, H = 640, 480; cams = [cam_for(gsr, W, H, **kw) for kw in CAMS]
else:
    p = "/tmp/sim_1000000.ply"; soa = gsr.read_ply(p); W, H = 1920, 1080; cams = [gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H)]
for cam in cams:
    want = orc.preprocess(soa, cam, W, H, 3.0)
    order = orc.expected_depth_order(want)
    full = rect_pairs(want, order, W, H) if cfg == "c1" else None
    if full is None:
        # vectorized rect pairs for the big scene (order irrelevant here)
        vis = np.nonzero(want["status"] == 2)[0]; a = want["aabb"][vis].astype(np.int64)
        tx, ty = (W + 15) // 16, (H + 15) // 16
        x0 = a[:, 0] // 16; x1 = np.minimum(tx - 1, a[:, 2] // 16); y0 = a[:, 1] // 16; y1 = np.minimum(ty - 1, a[:, 3] // 16)
        cnt = (x1 - x0 + 1) * (y1 - y0 + 1); rep = np.repeat(np.arange(len(vis)), cnt); st = np.repeat(np.cumsum(cnt) - cnt, cnt)
        kk = np.arange(rep.size) - st; ww = (x1 - x0 + 1)[rep]
        tile = (y0[rep] + kk // ww) * tx + x0[rep] + kk % ww
        full = (tile.astype(np.uint64) << np.uint64(32)) | vis[rep].astype(np.uint64)
    code, tx0, tx1, ty0 = spans_np(want, W, H)
    keep = listed(full, code, tx0, tx1, ty0, W)
    dropped = full[~keep]
    al = max_alpha_on_tiles(want, dropped, W)
    print(f"pairs {full.size} kept {keep.mean():.3f} dropped {dropped.size} max alpha of dropped {al.max() if al.size else 0:.3e}", flush=True)
