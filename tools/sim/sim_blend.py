"""Blend schedule simulator driver (analysis only): config-2 scene, oracle records,
16x16 tile lists in depth order, four 8x8 blocks per tile."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import gaussianrenderer_amd as gsr
import _oracle as orc



def setup(n=None):
    """Config-2 scene (seed 2), oracle records in depth order, 16x16 tile lists, four 8x8
    blocks per tile: (rec n x 11, lists, offs nb x 2, nb, bxy nb x 2)."""
    n = n or int(os.environ.get("N", 1_000_000)); W, H = 1920, 1080
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
    # tile lists
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
    return rec, lists, offs, nb, bxy


def load_sim():
    so = os.path.join("/tmp", "sim_blend.so")
    import subprocess
    subprocess.run(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-o", so,
                    os.path.join(os.path.dirname(os.path.abspath(__file__)), "sim_blend.c"), "-lm"], check=True)
    L = ctypes.CDLL(so)
    P = ctypes.c_void_p
    L.sim.argtypes = [P, P, P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    return L


def run(L, data, G, B, pairs, cm):
    rec, lists, offs, nb, bxy = data
    out = np.zeros(5)
    L.sim(rec.ctypes.data, lists.ctypes.data, offs.ctypes.data, ctypes.c_int(nb), bxy.ctypes.data,
          ctypes.c_int(G), ctypes.c_int(B), ctypes.c_int(pairs), ctypes.c_int(cm), out.ctypes.data)
    return out


if __name__ == "__main__":
    data = setup()
    L = load_sim()
    for G, B, pairs, cm in [(1, 64, 1, 0), (1, 64, 1, 3), (1, 64, 1, 4)]:
        t0 = time.time()
        it, taken, active, loaded, _ = run(L, data, G, B, pairs, cm)
        print(f"G={G:2d} B={B} pairs={pairs} cull={cm}: iterations {it/1e6:.3f}M taken {taken/1e6:.1f}M active {active/1e6:.1f}M "
              f"taken/slots {taken/(64*it):.3f} active/slots {active/(64*it):.3f} ({time.time()-t0:.1f}s)", flush=True)
