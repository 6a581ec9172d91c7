#!/usr/bin/env python3
"""bench.py — frames/sec of the MI355X 3DGS rasterizer (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|1]

One step = one full frame through the native pipeline (preprocess -> depth
sort -> tile binning: row pass + column pass -> blend) on the synthetic scene
of BASELINE config 2 (1M Gaussians, 1920x1080, seed 2, camera at (0,0,4),
fovY 50, k = 3), with the scene and the output image resident in HBM.

Multi-GPU (config 4 semantics, launched by torch.distributed.run): one process
per GPU, each rank renders its own orbit camera (azimuth 45 deg * rank) of the
replicated scene; frames shard with no collective inside the render (weak
scaling).  With --gather step (default for N > 1) every finished frame is
handed to rank 0 by an RCCL gather over xGMI (torch.distributed, backend
nccl), issued asynchronously and overlapped with the next frame's render
(double-buffered); --gather end hands over only the last frame, after the
timed region.  gaussianrenderer_amd/multi.py holds the per-rank logic.

Rank 0 prints ONE JSON line (contract in the task statement), including the
blend kernel's roofline (HIP events around every blend launch inside the timed
region) and the CPU-oracle baseline (rank 0, N = 1 only, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (n, W, H, seed)
    1: (10_000, 640, 480, 1),
    2: (1_000_000, 1920, 1080, 2),
    3: (5_000_000, 1600, 1063, 3),
    5: (2_000_000, 1920, 1080, 5),     # 4D (Spacetime-Gaussian style), 120 timesteps
}
TIMESTEPS_4D = 120
TIMING_STRIDE = 8
STAGE_FRAMES = 10     # untimed frames averaged for stages_ms
LEAD_IN = 8           # --orbit-step / orbit object: untimed frames per lane just before a timed region
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
# the blend (one 64-thread workgroup per 8x8 block): template <DIAG, STAMPS, FX, SPLIT>, FX = the
# fast-exp blend (GSR_TUNE_BLEND_EXP 1) or the exact one (0, the default); SPLIT 1 = the depth
# split's phase A (GSR_TUNE_DEPTH_SPLIT, on by default above 1.5M Gaussians), whose launch is
# the frame's blend; phase B (binning the rest of the depth order, resuming the blocks phase A
# left unsaturated) is the "resume" stage
BLEND_KERNELS = {1: "k_blend_w<false, false, true, 0>", 0: "k_blend_w<false, false, false, 0>",
                 "split": "k_blend_w<false, false, false, 1>"}
BLEND_KERNEL = BLEND_KERNELS[0]
SPLIT_STATES = {0: "one phase", 1: "whole order sorted", 2: "threshold partition, phase B queued",
                3: "threshold partition, speculative (no phase B)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--k", type=float, default=3.0)
    ap.add_argument("--warm-ms", type=float, default=1000.0,
                    help="untimed frames in flight for at least this long right before the timed regions")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-oracle sample length")
    ap.add_argument("--scene-dir", default=None)
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="N>1: nccl (= RCCL over xGMI, one GPU per rank) or gloo (rehearsal: ranks may share a GPU)")
    ap.add_argument("--gather", choices=("step", "end", "none"), default="step",
                    help="N>1: RCCL gather of finished frames to rank 0 every step (overlapped) or once at the end")
    ap.add_argument("--gather-every", type=int, default=1,
                    help="with --gather step: gather only every k-th chunk of frames to rank 0 (its inbound "
                         "xGMI budget at 8 ranks, DESIGN.md section 8); the others stay on their rank")
    ap.add_argument("--inflight", type=int, default=4,
                    help="frames in flight per GPU (gsr_render_path lanes); 1 = one frame at a time")
    ap.add_argument("--chunk", type=int, default=8,
                    help="N>1 with --gather step: frames per render_path call (one RCCL gather per frame)")
    ap.add_argument("--no-sh3-line", action="store_true",
                    help="config 2: skip the SH-3 sub-measurement (the 'sh3' object of the JSON line)")
    ap.add_argument("--sh3", action="store_true",
                    help="config 2 as BASELINE states it (SH degree 3): the opt-in SH-3 mode (all 45 f_rest, "
                         "bands 0-3; the reference evaluates bands 0-2)")
    ap.add_argument("--no-orbit-line", action="store_true",
                    help="config 2: skip the moving-camera sub-measurement (the 'orbit' object of the JSON line)")
    ap.add_argument("--orbit-step", type=float, default=0.0,
                    help="degrees of Camera::orbit per frame (a moving viewer: frame i at azimuth i * step); "
                         "0 = the fixed camera")
    ap.add_argument("--tune", default="",
                    help="gsr_set_tuning knob=value pairs, comma-separated (include/gsr.h GSR_TUNE_*; A/B runs)")
    return ap.parse_args()


def algorithmic_blend_bytes(ntiles: int, consumed: int, W: int, H: int, record: int = 48) -> int:
    """SURVEY.md 8d blend row: T*8 (tile ranges) + Pc*(4 index + 48 record) + 12*W*H
    (planar fp32 image) -- the roofline's `achieved`.  This design's blend gathers the
    whole 64-B splat record (4 x 16 B: conic, opacity + colour, centre + pixel box, cull
    word; gsr_kernels.hip k_blend_w), 68 B per pair: record=64 gives that figure
    (`algorithmic_bytes_design` beside it)."""
    return 8 * ntiles + (4 + record) * consumed + 12 * W * H


def algorithmic_stage_bytes(n: int, m: int, pairs: int, ntiles: int, consumed: int, W: int, H: int,
                            depth_passes: int = 4, tile_passes: int = 2, row_items: int = -1,
                            sh_floats: int = 27) -> dict:
    """Minimal bytes each stage of this design must move (per-stage table):
    preprocess N*152 read (38 fp32 SoA arrays; SH-3 mode: 48 SH floats, N*236) + M*64
    records + N*8 item + the tile rect (N*4 packed on the binning path, N*8 for the pair
    sort);
    blend as algorithmic_blend_bytes.
    Tile binning (row_items R >= 0): depth sort passes*N*32 (upsweep read 8, downsweep
    read 8 + 4 and write 8 + 4: item and its packed rect payload), or with the bucket
    sort (depth_passes 0, GSR_TUNE_DEPTH_BUCKETS) N*56 (count read 8; scatter read 8 + 4,
    write 8 + 4; local sort read 8 + 4, write 8 + 4);
    row pass ("emit") N*16 (4-B rects for the count, items + 4-B rects for the
    scatter) + R*8 row items; column pass ("tile_sort") R*16 (count + scatter reads)
    + P*4 values + T*8 ranges.
    Pair sort (R < 0): depth sort passes*N*24; emit N*40 (sorted items twice, rect
    gather, srect write/read) + P*6 (u16 key + u32 value); tile sort P*14 per
    non-final pass, P*12 for the final one (keys 2 up, 6 read, 6|4 write) + T*8."""
    out = {"preprocess": (152 + 4 * (sh_floats - 27)) * n + 64 * m + (12 if row_items >= 0 else 16) * n,
           "blend": algorithmic_blend_bytes(ntiles, consumed, W, H)}
    if row_items >= 0:
        out.update({"depth_sort": (depth_passes * 32 if depth_passes else 56) * n,
                    "emit": 16 * n + 8 * row_items,
                    "tile_sort": 16 * row_items + 4 * pairs + 8 * ntiles})
    else:
        out.update({"depth_sort": depth_passes * 24 * n,
                    "emit": 40 * n + 6 * pairs,
                    "tile_sort": 14 * pairs * (tile_passes - 1) + 12 * pairs + 8 * ntiles})
    return out


VALU_PEAK_PER_SIMD_CYCLE = 0.5   # wave64 non-packed VALU issue: one per 2 cycles per SIMD (32 lanes)
N_SIMDS = 256 * 4
CLOCK_HZ = 2.4e9


def load_pmc_counter(config: int, kernel: str, counter: str):
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None
    if d.get("config") != config:
        return None
    return d.get("kernels", {}).get(kernel, {}).get(counter)


def load_pmc_traffic(config: int, kernel: str):
    """HBM bytes per launch of `kernel` from the committed PMC summary of the same
    workload (tools/profile.sh: separate FETCH_SIZE / WRITE_SIZE passes, KiB x 1024,
    FETCH corrected per access pattern: x2 for wide coalesced streams (the guide's
    gfx950 correction), x1 for the blend's scattered 64-B record gathers, which our
    calibration shows are counted exactly — profiles/r01_fetch_calibration.txt), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None
    if d.get("config") != config or kernel not in d.get("kernels", {}):
        return None
    k = d["kernels"][kernel]
    if "fetch_bytes_corrected" not in k:
        return None
    return {"bytes_per_launch": int(k["fetch_bytes_corrected"] + k["write_bytes"]),
            "source": f"profiles/pmc_latest.json ({d.get('source', '')})"}


def dropin_rate(gsr, scene, cam, W, H, k, frames=20):
    """frames/sec through the reference's drop-in symbol preprocessCUDAGaussians:
    synchronous, header probe + full frame + 3*W*H float D2H into host memory
    (PCIe-inclusive; never reported as `value`)."""
    t = gsr.TilingInformation(50, 50, H, W)
    img = gsr.preprocessCUDAGaussians(scene.ptr, scene.n, cam, t.num_tile_y, t.num_tile_x, t.width_stride,
                                      t.height_stride, W, H, k)
    t0 = time.perf_counter()
    for _ in range(frames):   # one persistent pageable host image, like the viewer loop
        gsr.preprocessCUDAGaussians(scene.ptr, scene.n, cam, t.num_tile_y, t.num_tile_x, t.width_stride,
                                    t.height_stride, W, H, k, out=img)
    return frames / (time.perf_counter() - t0)


def cpu_baseline(soa, cam, W, H, k, seconds, four_d=False, sh3=False, cams=None):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle  # test infrastructure: CPU baseline leg only
    if sh3:
        with _oracle.sh3_mode():
            return cpu_baseline(soa, cam, W, H, k, seconds, four_d, False, cams)
    share = cpu_share()
    threads = share["threads"]
    frames, t0 = 0, time.perf_counter()
    while True:
        if four_d:   # temporal state of the frame, then the 3D render (no cull)
            _oracle.render(_oracle.temporal(soa, frame_time(frames)), cam, W, H, k, threads=threads)
        else:
            _oracle.render(soa, cams(frames) if cams else cam, W, H, k, threads=threads)
        frames += 1
        el = time.perf_counter() - t0
        if el >= seconds or frames >= 50:
            break
    # one frame on one thread beside it (single-thread and all-core runs)
    t1 = time.perf_counter()
    if four_d:
        _oracle.render(_oracle.temporal(soa, frame_time(0)), cam, W, H, k, threads=1)
    else:
        _oracle.render(soa, cam, W, H, k, threads=1)
    el1 = time.perf_counter() - t1
    return {"value": frames / el, "unit": "frames/sec", "cores": threads, "kind": "port",
            "sample": f"{frames} full frame(s) of the same workload by the C oracle (oracle/gsr_oracle.c, "
                      f"OpenMP {threads} threads), {el:.1f} s",
            "single_thread": {"value": 1.0 / el1, "unit": "frames/sec", "cores": 1,
                              "sample": f"1 full frame, {el1:.1f} s"},
            "host": dict(host_cpu(), **{k: v for k, v in share.items() if k != "threads"})}


def cpu_share() -> dict:
    """Host CPUs this process may run on: the affinity mask (os.sched_getaffinity),
    capped by the cgroup's CPU quota when one is set (cpu.max: a quota of 16 CPUs on
    a 256-CPU mask runs 16 at a time, so more OpenMP threads only time-slice)."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return {"threads": min(affinity, quota) if quota else affinity, "affinity_cpus": affinity,
            "cgroup_quota_cpus": quota}


def host_cpu() -> dict:
    """CPU model string and logical CPU count of the host the baseline ran on."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "logical_cpus": os.cpu_count()}


def gpu_telemetry(pci: str | None = None) -> dict | None:
    """Clocks, power and temperature of this rank's card (PCI address `pci`, e.g.
    "0000:75:00.0"; sysfs lists every card of the host), read in-process from sysfs
    (amdgpu's pp_dpm_* current levels and hwmon sensors) outside the timed region;
    None when unavailable.  No child process: a process that has initialised the GPU
    must not start programs that re-exec themselves (rocm-smi is a script)."""
    import glob
    cards = {}
    for dev in sorted(glob.glob("/sys/class/drm/card[0-9]*/device")):
        if not os.path.exists(os.path.join(dev, "pp_dpm_sclk")):
            continue
        if pci is None or os.path.basename(os.path.realpath(dev)).lower() != pci.lower():
            continue
        card = os.path.basename(os.path.dirname(dev))
        vals = {}
        for clk in ("sclk", "mclk", "fclk", "socclk"):
            try:
                with open(os.path.join(dev, f"pp_dpm_{clk}")) as f:
                    cur = [ln.split(":", 1)[1].strip().rstrip("*").strip() for ln in f if ln.rstrip().endswith("*")]
                if cur:
                    vals[f"{clk} (current dpm level)"] = cur[0]
            except OSError:
                pass
        for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
            for inp in sorted(glob.glob(os.path.join(hw, "temp*_input"))):
                try:
                    lab = inp.replace("_input", "_label")
                    name = open(lab).read().strip() if os.path.exists(lab) else os.path.basename(inp)
                    vals[f"temperature {name} (C)"] = int(open(inp).read()) / 1000.0
                except (OSError, ValueError):
                    pass
            for pw in ("power1_average", "power1_input"):
                try:
                    vals[f"{pw} (W)"] = int(open(os.path.join(hw, pw)).read()) / 1e6
                except (OSError, ValueError):
                    pass
        if vals:
            cards[card] = vals
    return cards or None


def sh3_line(gsr, torch, multi, args, ply, cam, W, H, F, stream, n) -> dict:
    """BASELINE config 2 as worded ("1M random Gaussians, 1920x1080, SH degree 3"): the same
    seed-2 .ply through the SH-3 scene block (48 SH floats per Gaussian, bands 0-3), the
    same K, warmup and camera, frames in flight and one at a time, and the preprocess
    stage's algorithmic rate.  The headline value stays the reference's bands 0-2
    (render.cu:506-530), the parity configuration."""
    scene3 = gsr.Scene.from_ply(ply, sh3=True)
    r3 = gsr.Renderer()
    for kv in filter(None, args.tune.split(",")):
        knob, val = kv.split("=")
        r3.set_tuning(int(knob), int(val))
    r3.set_frames_in_flight(F)
    shard3 = multi.FrameShard(None, r3, scene3, cam, W, H, k=args.k, steps=args.steps, gather="none", inflight=F,
                              chunk=args.chunk, stream=stream)
    for i in range(max(1, args.warmup)):
        shard3.frame(i)
    while r3.sync() != 0:
        shard3.frame()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) < 0.3:          # the card stays warm (the main run just ended)
        shard3.run(4 * F)
        torch.cuda.synchronize()
    r3.sync()
    r3.set_timing(2)
    for _ in range(STAGE_FRAMES):
        r3.render(scene3, cam, W, H, shard3.outs[0].data_ptr(), k=args.k, stream=stream)
    r3.sync()
    sums, frames = r3.stage_times()
    stages = {k: v / max(1, frames) for k, v in sums.items()}
    r3.set_timing(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        shard3.frame(i)
    torch.cuda.synchronize()
    seq = time.perf_counter() - t0
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        shard3.run(args.steps)
        shard3.drain()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if not shard3.finish("cuda"):
            break
    overflow = r3.sync()
    visible = int((r3.read_splats(n)["depth_key"] != 0xFFFFFFFF).sum())
    pre_bytes = algorithmic_stage_bytes(n, visible, 0, 1, 0, W, H, sh_floats=48)["preprocess"]
    out = {"value": round(args.steps / el, 3), "unit": "frames/sec", "ms_per_step": round(el / args.steps * 1e3, 4),
           "sequential": {"value": round(args.steps / seq, 3), "ms_per_frame": round(seq / args.steps * 1e3, 4)},
           "stages_ms": {k: round(v, 4) for k, v in stages.items()},
           "preprocess_gbs": round(pre_bytes / (stages["preprocess"] * 1e-3) / 1e9, 1) if stages.get("preprocess")
           else None,
           "preprocess_algorithmic_bytes": pre_bytes, "sh_floats": 48, "frames_in_flight": F,
           "overflow_after_timed": overflow,
           "note": "BASELINE config 2 as worded (SH degree 3): the same .ply's 45 f_rest through the SH-3 "
                   "scene block (bands 0-3, 48 SH floats), same K / warmup / camera; the headline value is "
                   "the reference's bands 0-2 (render.cu:506-530)"}
    r3.close()
    scene3.free()
    return out


ORBIT_LINE_STEP_DEG = 0.25    # the moving viewer of the 'orbit' object: Camera::orbit per frame
ORBIT_STATS_FRAMES = 40       # untimed frames whose bucket sizes give the splitter imbalance


def orbit_line(gsr, torch, multi, args, scene, W, H, F, stream) -> dict:
    """Config 2 on a moving camera: the same seed-2 scene, frame i orbited
    by 0.25 deg * i (Camera::orbit, camera.cpp:130-158), K frames in flight and one at a time
    after the same warmup, each timed region preceded by untimed lead-in frames -LEAD_IN..-1
    (per lane) so it starts from a viewer's history, not a jump.  The headline repeats one camera, the best case of every temporal cache
    in the path (the bucket splitters are the previous frame's depth quantiles, the depth
    pass budget, the depth split's speculation); this object reports the moving viewer's
    rate beside it, the items the bucket sort sent through its global path (buckets over
    the 2,048-item local capacity) in the timed frames, and the splitter imbalance (the
    largest live bucket / the mean) of ORBIT_STATS_FRAMES more frames."""
    import numpy as np
    pos = [0]
    cache = {}

    def cam_at(i):
        j = pos[0] + i
        if j not in cache:
            c = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H)
            gsr.orbit(c, ORBIT_LINE_STEP_DEG * j, 0.0)
            cache[j] = c
        return cache[j]

    ro = gsr.Renderer()
    for kv in filter(None, args.tune.split(",")):
        knob, val = kv.split("=")
        ro.set_tuning(int(knob), int(val))
    ro.set_frames_in_flight(F)
    sh = multi.FrameShard(None, ro, scene, cam_at(0), W, H, k=args.k, steps=args.steps, gather="none", inflight=F,
                          chunk=args.chunk, stream=stream, frame_cam=cam_at)
    for i in range(max(1, args.warmup)):
        sh.frame(i)
    pos[0] += max(1, args.warmup)
    while ro.sync() != 0:
        sh.frame(0)
        pos[0] += 1
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) < 0.3:          # the card stays warm, the orbit keeps moving
        sh.run(4 * F)
        pos[0] += 4 * F
        torch.cuda.synchronize()
    ro.sync()

    def lead_in(sequential):   # orbit frames -LEAD_IN .. -1 (per lane) before timed frames 0..K-1
        pos[0] = 0
        if sequential:
            for i in range(-LEAD_IN, 0):
                sh.frame(i)
        else:
            sh.path(-LEAD_IN * F, LEAD_IN * F, [j % F for j in range(LEAD_IN * F)])
        torch.cuda.synchronize()
        ro.sync()

    lead_in(True)
    over0 = ro.get_tuning(29)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        sh.frame(i)
    torch.cuda.synchronize()
    seq = time.perf_counter() - t0
    pos[0] += args.steps
    seq_rc = ro.sync()
    timed_frames = args.steps
    for _ in range(2):
        over1 = ro.get_tuning(29)
        lead_in(False)
        over0 += ro.get_tuning(29) - over1   # the lead-in's global-path items are not the timed frames'
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sh.run(args.steps)
        sh.drain()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        pos[0] += args.steps
        timed_frames += args.steps
        if not sh.finish("cuda"):
            break
    over_timed = ro.get_tuning(29) - over0
    # untimed: frames one at a time on lane 0 (its bucket totals after each), the orbit
    # continuing, with the per-stage events
    imb, glob, lsd = [], [], 0
    ro.set_timing(2)
    for i in range(ORBIT_STATS_FRAMES):
        o0 = ro.get_tuning(29)
        sh.frame(i)
        ro.sync()
        sizes = ro.bucket_sizes()
        if sizes is None:
            lsd += 1
            continue
        live = sizes[:-1].astype(np.float64)
        if live.sum() > 0:
            imb.append(float(live.max() / live.mean()))
        glob.append(ro.get_tuning(29) - o0)
    sums, frames = ro.stage_times()
    ro.set_timing(0)
    pos[0] += ORBIT_STATS_FRAMES
    ro.close()
    return {"value": round(args.steps / el, 3), "unit": "frames/sec", "ms_per_step": round(el / args.steps * 1e3, 4),
            "sequential": {"value": round(args.steps / seq, 3), "ms_per_frame": round(seq / args.steps * 1e3, 4)},
            "orbit_step_deg": ORBIT_LINE_STEP_DEG, "frames_in_flight": F,
            "depth_bucket_global_items": int(over_timed),
            "depth_bucket_global_items_per_frame": round(over_timed / max(1, timed_frames), 1),
            "splitter_imbalance": {"mean": round(float(np.mean(imb)), 3) if imb else None,
                                   "max": round(float(np.max(imb)), 3) if imb else None,
                                   "frames": len(imb),
                                   "global_items_per_frame": round(float(np.mean(glob)), 1) if glob else None,
                                   "lsd_frames": lsd,
                                   "note": "largest live bucket / mean live bucket of each bucket-sorted frame "
                                           "(gsr_bucket_sizes), ORBIT_STATS_FRAMES untimed frames one at a time "
                                           "after the timed ones"},
            "stages_ms": {k: round(v / max(1, frames), 4) for k, v in sums.items()},
            "overflow_after_timed": seq_rc,
            "note": "config 2 on a moving camera: frame i orbited by 0.25 deg * i around the scene (camera.cpp "
                    "Camera::orbit); the one-at-a-time and the in-flight regions each show frames 0..K-1 after "
                    "LEAD_IN untimed frames per lane just before them (-LEAD_IN .. -1), so every timed frame's "
                    "splitters are a moving viewer's; same scene, K, warmup as the headline"}


def frame_time(i: int) -> float:
    """Config 5: frame i renders timestep i mod 120 of [0, 1]."""
    return (i % TIMESTEPS_4D) / (TIMESTEPS_4D - 1)


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` (N > 1) started without RANK in the environment: start N
    ranks under torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1)
    as a CHILD process and return its exit code.  Nothing here touches the GPU: the
    parent only picks a free port and waits."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    import torch  # noqa: E402  (before gaussianrenderer_amd: one HIP runtime)
    from gaussianrenderer_amd import multi
    info = multi.rank_info()
    if info.world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {info.world}")
    rank, world, local_rank = info.rank, info.world, info.local_rank
    device = local_rank % max(1, torch.cuda.device_count())   # == local_rank on a full node
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
    import gaussianrenderer_amd as gsr

    n, W, H, seed = CONFIGS[args.config]
    scene_dir = args.scene_dir or os.path.join(tempfile.gettempdir(), "gsr_bench")
    os.makedirs(scene_dir, exist_ok=True)
    four_d = args.config == 5
    ply = os.path.join(scene_dir, f"config{args.config}_n{n}_s{seed}{'_4d' if four_d else ''}.ply")
    gloo = dist is not None and args.dist_backend == "gloo"
    scene = None
    if rank == 0:
        if not os.path.exists(ply):
            tmp = ply + f".tmp{os.getpid()}"
            (gsr.write_synthetic_ply4d if four_d else gsr.write_synthetic_ply)(tmp, n, seed)
            os.replace(tmp, ply)
        scene = gsr.Scene.from_ply(ply, sh3=args.sh3)   # the drop-in loader path (misc.cu:13-134)
    # N > 1: rank 0's device scene block reaches the other ranks in one broadcast
    # (over xGMI with RCCL), no rank but 0 reads the file
    load_s = time.perf_counter()
    scene = multi.broadcast_scene(dist, scene, gloo=gloo) if dist else scene
    broadcast_ms = (time.perf_counter() - load_s) * 1e3 if dist else None
    cam = multi.orbit_camera(rank, W, H)      # rank 0: camera (0,0,4); config 4: orbit 45 deg * rank
    frame_cam = None
    orbit_pos = [0]   # orbit index of region-relative frame 0 (untimed regions continue the orbit)

    def advance(m):
        orbit_pos[0] += m

    if args.orbit_step:
        # a moving viewer: orbit index j at azimuth 45 deg * rank + j * step (one Camera::orbit
        # call); region-relative frame i is j = orbit_pos + i.  Each timed region shows frames
        # 0..K-1 after a lead-in (lead_in below), so its views do not depend on how many
        # frames the time-based warmups rendered
        cam_cache = {}

        def frame_cam(i):
            j = orbit_pos[0] + i
            if j not in cam_cache:
                c = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H)
                gsr.orbit(c, multi.orbit_azimuth(rank) + args.orbit_step * j, 0.0)
                cam_cache[j] = c
            return cam_cache[j]

    r = gsr.Renderer()
    for kv in filter(None, args.tune.split(",")):
        knob, val = kv.split("=")
        r.set_tuning(int(knob), int(val))
    F = max(1, min(8, args.inflight))
    r.set_frames_in_flight(F)
    stream = torch.cuda.current_stream().cuda_stream
    shard = multi.FrameShard(dist, r, scene, cam, W, H, k=args.k, steps=args.steps, gather=args.gather,
                             inflight=F, chunk=args.chunk, gloo=gloo, frame_time=frame_time if four_d else None,
                             stream=stream, frame_cam=frame_cam, gather_every=args.gather_every)
    outs, frame, path = shard.outs, shard.frame, shard.path

    # warmup (+ grow every lane's pair buffer to the high-water mark)
    for i in range(max(1, args.warmup)):
        frame(i)
    advance(max(1, args.warmup))
    while r.sync() != 0:
        frame()
        advance(1)
    for _ in range(3):
        rc = path(0, max(F, args.warmup), [j % min(F, len(outs)) for j in range(max(F, args.warmup))])
        advance(max(F, args.warmup))
        if r.sync() == 0 and rc == 0:
            break
    torch.cuda.synchronize()

    def lead_in(sequential):
        """A moving camera's timed region shows orbit frames 0..K-1; untimed frames just
        before it (-LEAD_IN .. -1 per lane, one at a time or through the lanes) give the
        temporal caches (bucket splitters, pass budget) a viewer's history instead of a jump
        from wherever the orbit stood."""
        if not frame_cam:
            return
        orbit_pos[0] = 0
        if sequential:
            for i in range(-LEAD_IN, 0):
                frame(i)
        else:
            m = LEAD_IN * F
            path(-m, m, [j % min(F, len(outs)) for j in range(m)])
        torch.cuda.synchronize()
        r.sync()

    def warm(ms):
        """Untimed frames in flight for at least `ms` of wall time; returns the count.  A
        moving camera (--orbit-step) keeps moving through them."""
        frames, w0 = 0, time.perf_counter()
        while (time.perf_counter() - w0) * 1e3 < ms:
            m = 4 * F
            path(0, m, [j % min(F, len(outs)) for j in range(m)])
            advance(m)
            frames += m
            torch.cuda.synchronize()
        r.sync()
        return frames

    warm(min(300.0, args.warm_ms))   # stage times below are taken on a warm card too

    # untimed frames: the per-stage breakdown averaged over STAGE_FRAMES plain
    # frames (events between stages), then P, Pc and the blend counters from the
    # instrumented blend kernel
    t_mid = frame_time(TIMESTEPS_4D // 2) if four_d else None
    r.set_timing(2)
    for i in range(STAGE_FRAMES):
        r.render(scene, frame_cam(i) if frame_cam else cam, W, H, outs[0].data_ptr(), k=args.k, stream=stream,
                 time=t_mid)
    advance(STAGE_FRAMES)
    r.sync()
    stage_sums, stage_frames = r.stage_times()
    stages = {k: v / max(1, stage_frames) for k, v in stage_sums.items()}
    r.set_timing(0)
    r.set_diagnostics(True)
    r.render(scene, frame_cam(0) if frame_cam else cam, W, H, outs[0].data_ptr(), k=args.k, stream=stream,
             time=t_mid)
    advance(1)
    r.sync()
    pairs = r.pair_count()
    row_items = r.row_item_count()
    depth_passes = r.depth_passes()
    counters = r.blend_counters_ex()
    consumed = counters["records_loaded"]
    global BLEND_KERNEL
    blend_exp = r.get_tuning(22)
    split_state = r.get_tuning(26)                    # GSR_TUNE_DEPTH_SPLIT_STATE of the last frame
    split = split_state != 0
    BLEND_KERNEL = BLEND_KERNELS["split" if split else min(blend_exp, 1)]
    r.set_diagnostics(False)
    tiles_x, tiles_y = r.tile_grid()
    # visible Gaussians M (depth key != 0xFFFFFFFF), untimed
    visible = int((r.read_splats(n)["depth_key"] != 0xFFFFFFFF).sum())

    def timed(fn):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        shard.drain()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        return time.perf_counter() - t0

    # clocks and power before the timed regions (a ~1 s host-side child process, so it
    # runs before the sustained warmup, never between warmup and timing)
    props = torch.cuda.get_device_properties(device)
    pci = (f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
           if hasattr(props, "pci_bus_id") else None)
    telemetry_before = gpu_telemetry(pci) if rank == 0 else None
    # sustained warmup: the card leaves its idle power state over tens of ms, so a
    # short K (the driver's --steps 20 is ~10 ms of frames) would otherwise be timed on
    # the ramp.  Frames in flight for at least --warm-ms of wall time, untimed.
    warm_frames = warm(args.warm_ms)
    if dist:
        dist.barrier()

    # sequential segment: K frames one at a time on one stream (the viewer's use and the
    # frame latency), HIP events around the blend launch of every TIMING_STRIDE-th frame
    # (an event pair per frame costs ~7 us; every frame is the same workload, so the
    # sampled mean is the launch mean) -> roofline of the blend kernel running alone
    r.set_timing(1, TIMING_STRIDE)

    def run_sequential():
        for i in range(args.steps):
            frame(i)
    lead_in(True)
    seq_elapsed = timed(run_sequential)
    advance(args.steps)
    blend_times, timed_frames = r.stage_times()
    r.set_timing(0)
    seq_overflow = r.sync()

    # pipelined timed region (the reported value): the same K frames through
    # gsr_render_path with F frames in flight (no timing events in it: lane 0's blend
    # launches in flight are sampled in an untimed region after it)
    # Every rank checks its frames for GSR_E_OVERFLOW (an incomplete frame: pair buffer
    # grown, or a depth sort short of passes) and all ranks agree (shard.finish, a
    # collective); a region with one is timed again, once, on the grown buffers.
    dev_kind = "cpu" if gloo else "cuda"
    reruns = 0
    shard.time_gathers = dist is not None   # N > 1: per-chunk gather times for the 'scale' object
    if shard.validity:
        # per-step gathers carry each frame's validity word: the timed region includes
        # re-rendering and re-gathering exactly the chunks some rank got incomplete
        shard.overflowed, shard.gathers, shard.repaired = False, 0, 0
        clean = []
        lead_in(False)
        elapsed = timed(lambda: clean.append(shard.run_checked(args.steps, dev_kind)))
        advance(args.steps)
        reruns = shard.repaired
        if not clean[0]:
            sys.exit("bench.py: frames still incomplete after repairs")
    elif F > 1:
        for attempt in range(2):
            shard.overflowed, shard.gathers = False, 0
            lead_in(False)
            elapsed = timed(lambda: shard.run(args.steps))
            advance(args.steps)
            if not shard.finish(dev_kind):
                break
            reruns += 1
    else:
        elapsed = seq_elapsed
    overflow = r.sync() or seq_overflow
    split_after = (r.get_tuning(26), r.get_tuning(24))   # depth split state and point after the timed frames
    bucket_over = r.get_tuning(29)   # items the bucket sort's global path sorted so far (all lanes, sticky)
    telemetry_after = gpu_telemetry(pci) if rank == 0 else None
    if F > 1:
        # lane 0's blend launches while F frames are in flight: K more frames through the
        # same loop, untimed, with an event pair around every lane-0 blend (a collective at
        # N > 1: every rank runs it)
        shard.time_gathers = False
        r.set_timing(1, 1)
        shard.run(args.steps)
        shard.drain()
        torch.cuda.synchronize()
        advance(args.steps)
        blend_times_pipe, timed_frames_pipe = r.stage_times()
        r.set_timing(0)
        shard.finish(dev_kind)
    else:
        blend_times_pipe, timed_frames_pipe = blend_times, timed_frames

    max_elapsed = multi.max_over_ranks(dist, elapsed, "cpu" if gloo else "cuda")
    max_seq = multi.max_over_ranks(dist, seq_elapsed, "cpu" if gloo else "cuda")
    scale = None
    if dist:
        # what each rank renders with no gathers (a short region after the
        # headline, not part of it) and what the gathers cost, so the first SCALE record
        # can be read against DESIGN.md section 8's prediction
        gms = shard.gather_ms()
        shard.time_gathers = False
        ro = multi.FrameShard(dist, r, scene, cam, W, H, k=args.k, steps=args.steps, gather="none", inflight=F,
                              chunk=args.chunk, gloo=gloo, frame_time=frame_time if four_d else None,
                              stream=stream, frame_cam=frame_cam)
        ro.run(args.steps)               # warm: the lanes leave the gathered loop's rhythm
        torch.cuda.synchronize()
        advance(args.steps)
        r.sync()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ro.run(args.steps)
        torch.cuda.synchronize()
        render_el = time.perf_counter() - t0
        advance(args.steps)
        r.sync()
        scale = multi.scale_report(dist, render_el, args.steps, gms, world * args.steps / max_elapsed,
                                   "cpu" if gloo else "cuda")
    gather_ms = None
    if dist and args.gather == "end":
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        multi.gather_frames(dist, outs[0].cpu() if gloo else outs[0])
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = max_elapsed / args.steps * 1e3
    value = world * args.steps / max_elapsed
    blend_avg_ms = blend_times["blend"] / max(1, timed_frames)
    ntiles = tiles_x * tiles_y
    bytes_blend = algorithmic_blend_bytes(ntiles, consumed, W, H)
    achieved = bytes_blend / (blend_avg_ms * 1e-3) / 1e9
    img = outs[0].view(3, H, W)
    result = {
        "metric": ("frames/sec at 1920x1080, 1M Gaussians (config %d%s)"
                   % (args.config, ", SH degree 3" if args.sh3 else "")) if args.config == 2
        else (f"frames/sec at 1920x1080, 2M 4D Gaussians, {TIMESTEPS_4D} timesteps (config 5)" if four_d
              else f"frames/sec (config {args.config})"),
        "value": round(value, 3),
        "unit": "frames/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded 3DGS .ply, SURVEY.md 8d)",
        "config": {"workload": f"config{args.config}: {n} {'4D ' if four_d else ''}Gaussians, {W}x{H}, k={args.k}, "
                               + (f"frame i at t = (i mod {TIMESTEPS_4D})/{TIMESTEPS_4D - 1} with temporal cull, "
                                  if four_d else "")
                               + (f"one orbit camera per GPU, {'RCCL' if args.dist_backend == 'nccl' else 'gloo (rehearsal)'} "
                                  f"gather to rank 0 ({args.gather})" if world > 1
                                  else "camera (0,0,4) fovY 50")
                               + (f", moving camera: the i-th frame shown orbited by {args.orbit_step:g} deg * i "
                                  "(the orbit continues across warmup, stage sample and timed regions)"
                                  if args.orbit_step else "")
                               + (", SH degree 3 (opt-in SH-3 mode: 45 f_rest, bands 0-3)" if args.sh3
                                  else ", SH bands 0-2 as the reference evaluates (render.cu:506-530)")
                               + f", {F} frame(s) in flight per GPU (gsr_render_path)",
                   "sh_degree": 3 if args.sh3 else 2, "orbit_step_deg": args.orbit_step,
                   "gaussians": n, "width": W, "height": H, "parallelism": f"frames{world}"},
        "roofline": {"bound": "hbm", "kernel": BLEND_KERNEL, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None, "avg_launch_ms": round(blend_avg_ms, 4),
                     "algorithmic_bytes": bytes_blend,
                     "algorithmic_bytes_design": algorithmic_blend_bytes(ntiles, consumed, W, H, record=64),
                     "bytes_per_pair": {"survey": 52, "design": 68},
                     "measured_on": "sequential timed segment (K frames one at a time: the kernel does not share "
                                    "the GPU); avg_launch_ms_inflight = lane 0's launches with F frames in flight "
                                    "(K more frames after the timed regions, an event pair on each)",
                     "avg_launch_ms_inflight": round(blend_times_pipe["blend"] / max(1, timed_frames_pipe), 4)},
        "frames_in_flight": F,
        "sequential": {"value": round(world * args.steps / max_seq, 3), "unit": "frames/sec",
                       "ms_per_frame": round(max_seq / args.steps * 1e3, 4),
                       "note": "same K frames one at a time on one stream (gsr_render; the viewer's use)"},
        "stages_ms": {k: round(v, 4) for k, v in stages.items()},
        "depth_split": ({"split_permille": r.get_tuning(24), "unsaturated_blocks_after_phase_a": r.get_tuning(25),
                         "state": SPLIT_STATES[split_state],
                         "after_timed": {"state": SPLIT_STATES[split_after[0]], "split_permille": split_after[1]},
                         "note": "pairs / row_items / stages emit+tile_sort are phase A's (the nearest "
                                 "split_permille/1000 of the depth order); stage depth_sort = threshold "
                                 "partition + near sort; stage resume = phase B"}
                        if split else None),
        "pairs": pairs,
        "row_items": row_items,
        "depth_passes": depth_passes,
        "depth_sort": ("bucket sort: stable scatter into depth-quantile buckets + one LDS sort per bucket "
                       "(GSR_TUNE_DEPTH_BUCKETS)" if depth_passes == 0 else f"{depth_passes} LSD radix passes"),
        "depth_bucket_global_items": bucket_over,
        "pairs_consumed": consumed,
        "blend_exp": {1: "fast (v_exp_f32 alpha, exact alpha tests, guarded T tests, exact re-blend of "
                         "suspect pixels)", 0: "exact (gsr_blend_expf)"}[min(blend_exp, 1)],
        "blend_counters": counters,
        "blend_lane_efficiency": round(counters["active_lanes"] / max(1, counters["lane_slots"]), 4),
        "image_mean": float(img.mean().item()),
        "overflow_after_timed": overflow,
        "overflow_reruns": reruns,
        "overflow_reruns_unit": "chunks re-rendered and re-gathered inside the timed region (validity words)"
                                if shard.validity else "timed regions run again (whole region, untimed retry)",
    }
    result["gpu_telemetry"] = {"before_warmup": telemetry_before, "after_timed": telemetry_after}
    result["sustained_warmup"] = {"frames": warm_frames, "min_ms": args.warm_ms}
    if gather_ms is not None:
        result["gather_ms"] = round(gather_ms, 3)
    if scale is not None:
        result["scale"] = scale
    if dist:
        result["scene_broadcast_ms"] = round(broadcast_ms, 2)
        result["gathers_per_rank_timed"] = shard.gathers
        result["gather_every"] = args.gather_every
    sb = algorithmic_stage_bytes(n, visible, pairs, ntiles, consumed, W, H, depth_passes=depth_passes,
                                 row_items=row_items, sh_floats=48 if args.sh3 else 27)
    result["stages_gbs"] = {k: round(sb[k] / (stages[k] * 1e-3) / 1e9, 1) for k in sb if stages.get(k)}
    result["stages_gbs"]["blend"] = round(achieved, 1)     # timed frames, not the diagnostics frame
    result["stages_algorithmic_bytes"] = sb
    valu = load_pmc_counter(args.config, BLEND_KERNEL, "SQ_INSTS_VALU")
    if valu:
        rate = valu / (N_SIMDS * blend_avg_ms * 1e-3 * CLOCK_HZ)
        result["roofline_valu"] = {"bound": "valu", "kernel": BLEND_KERNEL, "achieved": round(rate, 4),
                                   "peak": VALU_PEAK_PER_SIMD_CYCLE, "unit": "wave64 VALU instr / SIMD / cycle @2.4GHz",
                                   "frac": round(rate / VALU_PEAK_PER_SIMD_CYCLE, 4),
                                   "instr_per_launch": valu,
                                   "measured_issue_peak": {"v_fma_f32": 0.348, "v_pk_fma_f32": 0.212,
                                                           "source": "profiles/r01_valu_rate.txt"},
                                   "source": "SQ_INSTS_VALU per launch from profiles/pmc_latest.json (one count "
                                             "per instruction, packed or not) / live blend time"}
    traffic = load_pmc_traffic(args.config, BLEND_KERNEL)
    if traffic is not None:
        result["roofline"]["traffic"] = traffic["bytes_per_launch"]
        result["roofline"]["traffic_source"] = traffic["source"]
    if world == 1 and args.config == 2 and not args.sh3 and not args.no_sh3_line:
        result["sh3"] = sh3_line(gsr, torch, multi, args, ply, cam, W, H, F, stream, n)
    if world == 1 and args.config == 2 and not args.sh3 and not args.orbit_step and not args.no_orbit_line:
        result["orbit"] = orbit_line(gsr, torch, multi, args, scene, W, H, F, stream)
    if world == 1:
        result["dropin_host_fps"] = round(dropin_rate(gsr, scene, cam, W, H, args.k), 2)
    if world == 1 and not args.no_cpu_baseline:
        soa = gsr.read_ply(ply, four_d=four_d, sh3=args.sh3)
        result["cpu_baseline"] = cpu_baseline(soa, cam, W, H, args.k, args.cpu_seconds, four_d=four_d, sh3=args.sh3,
                                              cams=frame_cam)
    print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
