"""Prices the quadrant-list blend schedule (round-4 verdict item 4) with the round-4
issue costs before anything is built (analysis only, not product, not test).

tools/sim/sim_blend.c replays the config-2 blend on the oracle's records (16x16 tile
lists in depth order, four 8x8 blocks per tile, 64-record batches, render.cu:323-341
compositing and early termination) and counts splat-slot iterations for two schedules
with the ideal (exact) cull per lane group:
  G = 1  one 8x8 list per wave (the shipped kernel)
  G = 4  four 4x4 quadrant lists per wave (a wave step evaluates entry j of every list)
The counts are priced with the shipped fast loop's measured instruction mix
(DESIGN.md "Blend design": 36 VALU + 27 SALU per two-splat iteration; PMC of one launch:
99.4M VALU, 58.8M SALU, profiles/pmc_latest.json) and the quadrant loop's extra work,
in three variants (the loop is co-bound by VALU and SALU issue, so an iteration costs
max(VALU, SALU) issue slots in this model):
  A  per-group box masks combined on the scalar unit: 4 descriptor reads + 4 mask builds
     per splat (+14 SALU per pair), +2 VALU for the per-group slot index (LDS u8 lists)
  B  box test on the vector unit from per-lane descriptors: +8 VALU per pair (two
     range tests per splat), the scalar mask build gone (-10 SALU), +2 VALU for the index
  C  A or B plus the per-group cull: four exact block tests per batch instead of one (the
     launch's non-loop VALU -- cull, compaction, set-up, epilogue -- taken x4: an upper
     bound, the compaction and set-up do not all scale)
  D  A or B with the cheap per-group cull instead: the exact block test once, quadrant
     membership from the box only (sim cull mode 1: more iterations than the ideal cull,
     +3 VALU per batch for the four box tests)
Usage: python tools/sim/sim_quad.py  (N=1000000 by default; ~2 min on 8 cores)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import sim_blend  # noqa: E402

VALU_LOOP, SALU_LOOP = 36, 27          # per two-splat iteration, fast loop (round 4)
VALU_LAUNCH, SALU_LAUNCH = 99.4e6, 58.8e6


def main():
    data = sim_blend.setup()
    L = sim_blend.load_sim()
    res = {}
    for G, cm in ((1, 0), (4, 0), (4, 1)):
        t0 = time.time()
        it, taken, active, loaded, batches = sim_blend.run(L, data, G, 64, 1, cm)
        res[(G, cm)] = (it, taken, active, loaded, batches)
        print(f"G={G} cull={'ideal per group' if cm == 0 else 'block test + quadrant boxes'}: splat-slot iterations "
              f"{it / 1e6:.3f}M, taken lanes {taken / 1e6:.1f}M, batches {batches / 1e3:.1f}K, records loaded "
              f"{loaded / 1e6:.2f}M ({time.time() - t0:.1f}s)", flush=True)
    it1, _, _, _, b1 = res[(1, 0)]
    pairs1, pairs4, pairs4c = it1 / 2, res[(4, 0)][0] / 2, res[(4, 1)][0] / 2
    # the shipped launch: loop VALU / SALU from the mix, the rest (cull, setup, epilogue) per batch
    cull_valu = max(0.0, VALU_LAUNCH - pairs1 * VALU_LOOP)
    cull_salu = max(0.0, SALU_LAUNCH - pairs1 * SALU_LOOP)
    print(f"shipped: {pairs1 / 1e6:.3f}M pair iterations x ({VALU_LOOP} VALU, {SALU_LOOP} SALU); the rest of the "
          f"launch {cull_valu / 1e6:.1f}M VALU, {cull_salu / 1e6:.1f}M SALU over {b1 / 1e3:.1f}K batches")

    def price(pairs, dv, ds, cull_x, per_batch_v=0):
        v = pairs * (VALU_LOOP + dv) + cull_valu * cull_x + b1 * per_batch_v
        s = pairs * (SALU_LOOP + ds) + cull_salu
        return max(v, s), v, s

    base, bv, bs = price(pairs1, 0, 0, 1)
    rows = [("shipped (8x8 list)", pairs1, 0, 0, 1, 0),
            ("quadrants, ideal cull, no extra work (a floor)", pairs4, 0, 0, 1, 0),
            ("A: ideal cull at 1x cost, scalar per-group masks", pairs4, 2, 14, 1, 0),
            ("B: ideal cull at 1x cost, vector box test", pairs4, 10, -10, 1, 0),
            ("C-A: A + four exact block tests per batch", pairs4, 2, 14, 4, 0),
            ("C-B: B + four exact block tests per batch", pairs4, 10, -10, 4, 0),
            ("D-A: block test + quadrant boxes, scalar masks", pairs4c, 2, 14, 1, 3),
            ("D-B: block test + quadrant boxes, vector box test", pairs4c, 10, -10, 1, 3)]
    print(f"{'schedule':52s} {'pairs':>8s} {'VALU':>8s} {'SALU':>8s} {'issue-bound':>12s} {'vs shipped':>10s}")
    for name, p, dv, ds, cx, pb in rows:
        c, v, s = price(p, dv, ds, cx, pb)
        print(f"{name:52s} {p / 1e6:7.3f}M {v / 1e6:7.1f}M {s / 1e6:7.1f}M {c / 1e6:11.1f}M {c / base - 1:+9.1%}")
    print("stop rule (round-4 verdict item 4): build only if the schedule prices at >= 5 % under the shipped one")


if __name__ == "__main__":
    main()
