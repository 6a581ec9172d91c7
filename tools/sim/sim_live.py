"""Live pixels per blend pair-iteration (analysis only): config-2 scene, oracle records,
16x16 tile lists in depth order, four 8x8 blocks per tile (tools/sim/sim_live.c).
Prices a "compact pair" schedule — both splats of a pair evaluated by one wave64 pass
over the live pixels when at most 32 are live — against the shipped packed pair loop,
in VALU issue cycles per wave (measured rates, profiles/r01_valu_rate.txt: v_fma_f32
0.348 / cycle, v_pk_fma_f32 0.212 / cycle).
Usage: python tools/sim/sim_live.py   (N=1000000 by default)"""
import ctypes, os, subprocess, sys, time
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import gaussianrenderer_amd as gsr  # noqa: E402
import _oracle as orc  # noqa: E402

n = int(os.environ.get("N", 1_000_000)); W, H = 1920, 1080
so = os.path.join("/tmp", "sim_live.so")
subprocess.run(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-o", so, os.path.join(HERE, "sim_live.c"), "-lm"],
               check=True)
ply = f"/tmp/sim_{n}.ply"
if not os.path.exists(ply):
    gsr.write_synthetic_ply(ply, n, 2)
soa = gsr.read_ply(ply)
cam = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H)
t0 = time.time()
sp = orc.preprocess(soa, cam, W, H, 3.0)
vis = np.nonzero(sp["status"] == 2)[0]
order = vis[np.lexsort((vis, sp["depth_key"][vis]))]
s = sp[order]
rec = np.zeros((len(s), 11), np.float32)
rec[:, 0] = s["px_x"]; rec[:, 1] = s["px_y"]
rec[:, 2:6] = s["inv_covar"]; rec[:, 6] = s["opacity"]
rec[:, 7:11] = s["aabb"]
tx, ty = (W + 15) // 16, (H + 15) // 16
x0 = np.clip(s["aabb"][:, 0] // 16, 0, tx - 1); x1 = np.clip(s["aabb"][:, 2] // 16, 0, tx - 1)
y0 = np.clip(s["aabb"][:, 1] // 16, 0, ty - 1); y1 = np.clip(s["aabb"][:, 3] // 16, 0, ty - 1)
cnt = ((x1 - x0 + 1) * (y1 - y0 + 1)).astype(np.int64)
rep = np.repeat(np.arange(len(s)), cnt)
start = np.repeat(np.cumsum(cnt) - cnt, cnt)
k = np.arange(rep.size) - start
w = (x1 - x0 + 1)[rep]
tile = (y0[rep] + k // w) * tx + x0[rep] + k % w
o = np.argsort(tile, kind="stable")
lists = rep[o].astype(np.int32)
toffs = np.zeros(tx * ty + 1, np.int64)
np.add.at(toffs, tile + 1, 1)
toffs = np.cumsum(toffs)
nb = tx * ty * 4
offs = np.zeros((nb, 2), np.int32); bxy = np.zeros((nb, 2), np.int32)
for sub in range(4):
    b = np.arange(tx * ty) * 4 + sub
    offs[b, 0] = toffs[:-1]; offs[b, 1] = toffs[1:]
    bxy[b, 0] = (np.arange(tx * ty) % tx) * 16 + (sub & 1) * 8
    bxy[b, 1] = (np.arange(tx * ty) // tx) * 16 + (sub >> 1) * 8
print(f"prep {time.time()-t0:.1f}s visible {len(s)} pairs {lists.size}", flush=True)
L = ctypes.CDLL(so)
P = ctypes.c_void_p
L.sim_live.argtypes = [P, P, P, ctypes.c_int, P, P, P]
hist = np.zeros(65); out = np.zeros(4)
t0 = time.time()
L.sim_live(rec.ctypes.data, lists.ctypes.data, offs.ctypes.data, ctypes.c_int(nb), bxy.ctypes.data,
           hist.ctypes.data, out.ctypes.data)
pit, batches, cblocks, active = out
print(f"pair-iterations {pit/1e6:.3f}M, batches {batches/1e3:.0f}K, blocks reaching <= 32 live {cblocks:.0f} of {nb} "
      f"({time.time()-t0:.1f}s)")
cum = np.cumsum(hist)
for L_ in (8, 16, 24, 32, 48, 64):
    print(f"  pair-iterations starting with <= {L_:2d} live pixels: {cum[L_]/pit:6.1%}")
# issue-cycle model per wave (profiles/r01_valu_rate.txt rates): shipped pair loop 25 packed +
# 21 scalar VALU; compact pair (one unpacked evaluation of both splats over <= 32 live
# pixels: dx dy, md2, exp, alpha ~ 24 scalar; a cross-half permute of alpha; two composites
# on the low half ~ 18 scalar; the in-box bit test per lane ~ 4 scalar) ~ 47 scalar
cyc_pk, cyc_sc = 1 / 0.212, 1 / 0.348
c_ship = 25 * cyc_pk + 21 * cyc_sc
c_comp = 47 * cyc_sc
c_cull = 135 * cyc_sc
small = cum[32]
base = pit * c_ship + batches * c_cull
new = (pit - small) * c_ship + small * c_comp + batches * c_cull + cblocks * 30 * cyc_sc
print(f"model: shipped {base/1e6:.1f}M issue-cycles, compact pairs {new/1e6:.1f}M ({(new/base - 1):+.1%})")
