"""Depth-split analysis (analysis only; AZ = orbit azimuth in degrees): how many (tile, splat) pairs and row items a
two-phase binning would list if phase A bins only the nearest fraction f of the
depth-ordered visible splats and phase B bins the rest for the tiles that phase A
did not saturate (every pixel's transmittance below 1e-3).  Oracle records, AABB
tile rects (no tile row spans).  N, W, H, SEED from the environment (config 3 by
default); FOURD=1 with T: config 5's 4D scene at time T (no temporal cull: 8 % of
its pixels saturate, no tile does, so the split turns itself off there)."""
import ctypes, os, subprocess, sys, time
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import gaussianrenderer_amd as gsr
import _oracle as orc

n = int(os.environ.get("N", 5_000_000)); W = int(os.environ.get("W", 1600)); H = int(os.environ.get("H", 1063))
seed = int(os.environ.get("SEED", 3))
so = os.path.join(HERE, "depth_split.so")
if not os.path.exists(so):
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fopenmp", "-shared", "-fPIC",
                           "-I" + os.path.join(ROOT, "include"), os.path.join(HERE, "depth_split.c"),
                           "-o", so, "-lm"])
four_d = os.environ.get("FOURD", "0") == "1"     # config 5: a 4D scene at time T (default 0.5)
ply = f"/tmp/sim_{n}_s{seed}{'_4d' if four_d else ''}.ply"
if not os.path.exists(ply):
    (gsr.write_synthetic_ply4d if four_d else gsr.write_synthetic_ply)(ply, n, seed)
soa = gsr.read_ply(ply, four_d=four_d)
if four_d:
    soa = orc.temporal(soa, float(os.environ.get("T", 0.5)))
cam = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H)
az = float(os.environ.get("AZ", 0))   # Camera::orbit azimuth (bench.py --orbit-step: frame i at i * step)
if az:
    gsr.orbit(cam, az)
t0 = time.time()
sp = orc.preprocess(soa, cam, W, H, 3.0)
vis = np.nonzero(sp["status"] == 2)[0]
order = vis[np.lexsort((vis, sp["depth_key"][vis]))]
s = sp[order]
m = len(s)
rec = np.zeros((m, 11), np.float32)
rec[:, 0] = s["px_x"]; rec[:, 1] = s["px_y"]
rec[:, 2:6] = s["inv_covar"]; rec[:, 6] = s["opacity"]
rec[:, 7:11] = s["aabb"]
sat = np.zeros(W * H, np.int32)
L = ctypes.CDLL(so)
L.sat_pos.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
L.sat_pos(rec.ctypes.data, m, W, H, sat.ctypes.data)
print(f"n {n} visible {m} ({time.time()-t0:.1f}s); pixels saturated {np.mean(sat >= 0):.3f}")

tx, ty = (W + 15) // 16, (H + 15) // 16
pad = np.full((ty * 16, tx * 16), -2, np.int64)
pad[:H, :W] = sat.reshape(H, W)
pad[pad == -1] = np.iinfo(np.int64).max     # never saturates
pad[pad == -2] = -1                          # outside the image
tile_sat = pad.reshape(ty, 16, tx, 16).max(axis=(1, 3))
x0 = np.clip(s["aabb"][:, 0] // 16, 0, tx - 1); x1 = np.clip(s["aabb"][:, 2] // 16, 0, tx - 1)
y0 = np.clip(s["aabb"][:, 1] // 16, 0, ty - 1); y1 = np.clip(s["aabb"][:, 3] // 16, 0, ty - 1)
cnt = ((x1 - x0 + 1) * (y1 - y0 + 1)).astype(np.int64)
rows = (y1 - y0 + 1).astype(np.int64)
pos = np.arange(m)
# pairs the blend reads today: a splat's pair is read while its tile is not saturated
consumed = 0
fin = tile_sat < np.iinfo(np.int64).max
print(f"pairs {cnt.sum()/1e6:.2f}M row items {rows.sum()/1e6:.2f}M; tiles never saturated "
      f"{np.mean(~fin):.3f}; tile saturation position / m: "
      + " ".join(f"p{q}={np.percentile(np.where(fin, tile_sat, m), q)/m:.3f}" for q in (10, 50, 90, 99)))
for f in (0.05, 0.1, 0.15, 0.2, 0.3, 0.5):
    d1 = int(f * m)
    unsat = (tile_sat >= d1).astype(np.int64)
    P = np.zeros((ty + 1, tx + 1), np.int64)
    P[1:, 1:] = unsat.cumsum(0).cumsum(1)
    b = pos >= d1
    xa, xb, ya, yb = x0[b], x1[b], y0[b], y1[b]
    pb = (P[yb + 1, xb + 1] - P[ya, xb + 1] - P[yb + 1, xa] + P[ya, xa]).sum()
    # phase-B row items: tile rows of the rect holding any unsaturated tile
    R = np.zeros((ty, tx + 1), np.int64)
    R[:, 1:] = unsat.cumsum(1)
    rb = 0
    for dy in range(int((yb - ya).max()) + 1 if b.any() else 0):
        ok = ya + dy <= yb
        yy = (ya + dy)[ok]
        rb += ((R[yy, xb[ok] + 1] - R[yy, xa[ok]]) > 0).sum()
    print(f"f={f:.2f}: phase A pairs {cnt[:d1].sum()/1e6:.2f}M rows {rows[:d1].sum()/1e6:.2f}M | "
          f"unsaturated tiles {unsat.mean():.3f} | phase B pairs {pb/1e6:.2f}M rows {rb/1e6:.2f}M | "
          f"total pairs {(cnt[:d1].sum()+pb)/1e6:.2f}M (now {cnt.sum()/1e6:.2f}M)", flush=True)
