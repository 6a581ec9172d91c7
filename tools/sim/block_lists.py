"""Analysis only: what per-8x8-block splat lists would save the blend (config 2 scene).

The blend runs four waves per 16x16 tile, one per 8x8 block, and each wave culls the
whole tile list in 64-record batches.  This replays the blend schedule (sim_blend.c,
G=1, pairs, saturation exits) over (a) the tile lists and (b) each block's own list,
filtered by the splat's pixel AABB (an exact filter: box_hit fails for every dropped
pair), and prints records loaded and batches.  profiles/r05_sim_block_lists.txt."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sim_blend as sb


def main():
    rec, lists, offs, nb, bxy = sb.setup()
    W, H = 1920, 1080
    tx, ty = (W + 15) // 16, (H + 15) // 16
    ntile = tx * ty
    toffs = np.concatenate([offs[0::4, 0], [offs[-1, 1]]])
    tile_of = np.repeat(np.arange(ntile), np.diff(toffs))
    a = rec[lists, 7:11]   # xmin ymin xmax ymax (px) per pair
    x0t, y0t = (tile_of % tx) * 16, (tile_of // tx) * 16
    parts, hits = [], 0
    for sub in range(4):
        bx, by = x0t + (sub & 1) * 8, y0t + (sub >> 1) * 8
        h = ~((a[:, 2] < bx) | (a[:, 0] > bx + 7) | (a[:, 3] < by) | (a[:, 1] > by + 7))
        hits += int(h.sum())
        sel = np.nonzero(h)[0]
        parts.append((lists[sel], np.bincount(tile_of[sel], minlength=ntile)))
    foffs = np.zeros((nb, 2), np.int32)
    vals, base = [], 0
    for sub, (v, cnt) in enumerate(parts):
        starts = base + np.concatenate([[0], np.cumsum(cnt)[:-1]])
        b = np.arange(ntile) * 4 + sub
        foffs[b, 0] = starts
        foffs[b, 1] = starts + cnt
        vals.append(v)
        base += v.size
    fl = np.concatenate(vals).astype(np.int32)
    L = sb.load_sim()
    o0 = sb.run(L, (rec, lists, offs, nb, bxy), 1, 64, 1, 0)
    o1 = sb.run(L, (rec, fl, foffs, nb, bxy), 1, 64, 1, 0)
    print(f"pairs {lists.size}; (pair, block) entries by AABB {hits} ({hits / (4 * lists.size):.3f} of 4 per pair)")
    for name, o in (("tile lists (shipped)", o0), ("block lists (AABB-filtered)", o1)):
        print(f"{name:30s} splat iterations {o[0]:.4g}  taken lanes {o[1]:.4g}  records loaded {o[3]:.4g}  batches {o[4]:.4g}")


if __name__ == "__main__":
    main()
