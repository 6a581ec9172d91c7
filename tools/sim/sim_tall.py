"""VERDICT r05 #3, "also price": two (or four) pixels per lane, one wave per 8x16 (8x32)
block, against the shipped one pixel per lane (8x8), on the config-2 records and tile
lists (sim_blend.py setup), ideal per-block cull, 64-entry batches, pairs.  The cost model
is the kernel's measured mix per splat step: 18 VALU + 13.5 SALU per
splat for one pixel per lane; a second pixel per lane repeats the per-pixel VALU (md2, exp,
alpha, tests, colour: ~16 of the 18) and shares the scalar work.  Analysis only."""
import ctypes
import numpy as np
import sim_blend as sb

if __name__ == "__main__":
    rec, lists, offs, nb, bxy = sb.setup()
    L = sb.load_sim()
    P_ = ctypes.c_void_p
    L.sim_tall.argtypes = [P_, P_, P_, ctypes.c_int, P_, ctypes.c_int, ctypes.c_int, P_]
    tiles = nb // 4
    res = {}
    for P in (1, 2):
        if P == 1:
            o, b = offs, bxy
        else:   # one 8x16 block per half-tile column: sub-blocks 0 and 1 of each tile (top row)
            sel = np.concatenate([np.arange(tiles) * 4 + 0, np.arange(tiles) * 4 + 1])
            o, b = np.ascontiguousarray(offs[sel]), np.ascontiguousarray(bxy[sel])
        out = np.zeros(5)
        L.sim_tall(rec.ctypes.data, lists.ctypes.data, o.ctypes.data, ctypes.c_int(len(o)), b.ctypes.data,
                   ctypes.c_int(P), ctypes.c_int(64), out.ctypes.data)
        res[P] = out
        it, taken, active, loaded, batches = out
        print(f"{P} px/lane ({8}x{8 * P}): waves {len(o)}  splat iterations {it:.4g}  taken lanes {taken:.4g}  "
              f"lane-slots {it * 64 * P:.4g}  taken/slots {taken / (it * 64 * P):.3f}  batches {batches:.4g}", flush=True)
    valu1, salu = 18.0, 13.5
    for P in (1, 2):
        it = res[P][0]
        valu = it * (valu1 + (P - 1) * 16.0)
        sc = it * salu
        print(f"{P} px/lane: VALU {valu / 1e6:.1f}M  SALU {sc / 1e6:.1f}M  (loop only; issue bound ~ max(VALU, ...) "
              f"with SALU co-issued from other waves)")
    r = res[2][0] * (valu1 + 16.0) / (res[1][0] * valu1)
    print(f"2 px/lane loop VALU / 1 px/lane: {r:.3f}; SALU ratio {res[2][0] / res[1][0]:.3f}")
