/*
 * gsr.h — C ABI of the MI355X-native 3D Gaussian splatting rasterizer.
 *
 * Two groups of entry points:
 *
 *  1. DROP-IN BOUNDARY — the exact symbols the reference viewer links
 *     against.  A viewer built against the reference's
 *     render.cuh / misc.cuh links against libgsr.so unchanged:
 *
 *       preprocessCUDAGaussians   replaces render.cu:871-1157 (decl render.cuh:27-37)
 *       loadGaussianCudaFromPly   replaces misc.cu:13-134     (decl misc.cuh:4, C++ linkage)
 *       oneSweep3DGaussianSort    replaces render.cu:194-264  (decl render.cuh:8-11)
 *       oneSweepSort              replaces onesweep.cu:190-250 (decl onesweep.cuh:8)
 *
 *  2. NATIVE API (gsr_*) — stream-ordered, device-resident, no per-frame
 *     allocation: a persistent context (workspace sized by high-water mark),
 *     the three pipeline stages the reference names "Preprocess + Sort +
 *     Render" as separate calls, readback hooks used by the parity tests, and
 *     the host-side camera / PLY helpers that mirror the reference's
 *     camera.cpp and gaussians.cpp so tests and benches can build inputs
 *     exactly like the viewer does.
 *
 * Errors: every int-returning function returns 0 on success and a negative
 * GSR_E* code on failure; gsr_last_error() returns the message.  The void
 * drop-in functions keep the reference's behaviour (print the error to
 * stderr and return, render.cu:914-923).
 */
#ifndef GSR_H
#define GSR_H

#include <stddef.h>
#include <stdint.h>
#include "gsr_types.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    GSR_OK = 0,
    GSR_E_ARG = -1,        /* invalid argument */
    GSR_E_HIP = -2,        /* HIP runtime error (no device, OOM, launch failure) */
    GSR_E_IO = -3,         /* file missing / unreadable / truncated */
    GSR_E_FORMAT = -4,     /* unsupported PLY format */
    GSR_E_OVERFLOW = -5,   /* an earlier frame is incomplete and must be re-rendered: its pairs
                              overflowed the pair buffer (grown now), its depth sort needed more
                              digit passes than the adaptive pass budget launched (budget reset to
                              four), or it was a speculative depth-split frame (GSR_TUNE_DEPTH_SPLIT,
                              no phase B queued) whose phase A left an 8x8 block unsaturated
                              (speculation stopped).  Any of these can happen at any frame, not only
                              during warm-up; gsr_render_path_status names the frames.  The
                              code can arrive on a later call than the frame it refers to: every
                              frame rendered since the last call that returned GSR_OK (or since the
                              last gsr_sync) must be re-rendered. */
    GSR_E_DISPLAY = -6     /* display interop: no current GL context / GL registration failed (gsr_gl.h) */
};

/* Scene layout accepted by the render entry points. */
enum {
    GSR_LAYOUT_SCENE_BLOCK = 0,   /* our SoA block (gsr_scene_header + arrays) */
    GSR_LAYOUT_AOS = 1,           /* reference Gaussian[] (240 B records) */
    GSR_LAYOUT_SCENE_BLOCK_4D = 2, /* 4D SoA block (GSR_SCENE4D_NARRAYS), rendered at gsr_set_time() */
    GSR_LAYOUT_SCENE_BLOCK_SH3 = 3 /* SH-3 block (GSR_SCENE_SH3_NARRAYS): degree-3 colour, clamped at 0 */
};

/* PLY loading flags (gsr_ply_read_host_ex / gsr_load_ply_device_ex). */
enum {
    GSR_PLY_TYPED = 1,  /* hardened reader: declared property types, ascii and big-endian
                           formats, other elements skipped, "nx" accepted.
                           Off = the reference's reader exactly (every property a 4-B float). */
    GSR_PLY_SH3 = 2     /* "Inria-correct" SH: all 45 f_rest, channel-major, into a 59-array
                           block rendered with degree-3 SH (off = the reference's 24 f_rest) */
};

/* Stage indices for gsr_stage_times(). */
enum {
    GSR_STAGE_PREPROCESS = 0,     /* cull + SH colour + projection + covariance + AABB */
    GSR_STAGE_DEPTH_SORT = 1,     /* stable radix sort of (depth, index) */
    GSR_STAGE_EMIT = 2,           /* pair emission, or the binning row pass */
    GSR_STAGE_TILE_SORT = 3,      /* stable radix sort of pairs by tile, or the binning column pass */
    GSR_STAGE_RANGES = 4,         /* per-tile [start, end) from sorted pairs */
    GSR_STAGE_BLEND = 5,          /* front-to-back alpha compositing (with the depth split: phase A's) */
    GSR_STAGE_RESUME = 6,         /* depth split phase B: binning the rest of the depth order and
                                     resuming the blocks phase A left unsaturated (0 on other frames) */
    GSR_NUM_STAGES = 7
};

#define GSR_TILE_PX 16            /* internal tile edge (pixels); output is tile-invariant */
#define GSR_SPLAT_RECORD_BYTES 64 /* per-Gaussian splat record written by preprocess */

/* ---------------------------------------------------------------- drop-in */

/* render.cu:871-881.  d_gaussians: a device scene block from
 * loadGaussianCudaFromPly (our SoA layout) OR a device Gaussian[] array in
 * the reference's AoS layout (detected by the header magic).  out_pixels:
 * HOST buffer of 3*tile_W*tile_H floats, planar RGB, row 0 = bottom (NDC -1).
 * tile_W/tile_H are the image size; the num_tile / stride arguments follow
 * TilingInformation (gaussians.hpp:47-58) and only bound which pixels are
 * covered (pixels at x >= num_tile_x*width_stride or y >= num_tile_y*
 * height_stride stay 0 as in renderGaussians, render.cu:285-363).
 * Synchronous; uses a process-wide context guarded by a mutex. */
void preprocessCUDAGaussians(gsr_gaussian* d_gaussians, float* out_pixels, int num_gaussians,
                             gsr_camera cam, int num_tile_y, int num_tile_x, int width_stride,
                             int height_stride, int tile_W, int tile_H, float k);

/* C twin of loadGaussianCudaFromPly (misc.cu:13-134) for FFI callers:
 * returns a device scene block (free with hipFree or gsr_scene_free), or
 * NULL on failure; *out_numGaussians is set once the header is parsed. */
gsr_gaussian* gsr_load_ply_device(const char* filename, int* out_numGaussians);
/* Same with loader flags (GSR_PLY_TYPED | GSR_PLY_SH3).  If out_narrays is
 * non-NULL, a file carrying the 4D properties (trbf_center, trbf_scale,
 * motion_0..8) loads as a 4D scene block (*out_narrays = 49); GSR_PLY_SH3
 * gives an SH-3 block (59); else 38. */
gsr_gaussian* gsr_load_ply_device_ex(const char* filename, int* out_numGaussians, int flags, int* out_narrays);

/* render.cu:194-264: stable sort of N host-side lightWeightGaussian records
 * by the low num_bits bits of radix_id, in place; *kernel_ms = device time. */
void oneSweep3DGaussianSort(gsr_lwg* d_in, int N, int num_bits, float* kernel_ms);

/* onesweep.cu:190-250: sort N host ints (keys in [0, maxVal], non-negative)
 * ascending into output; *kernel_ms = device time of the sort passes. */
void oneSweepSort(int* input, int* output, int N, int maxVal, float* kernel_ms);

/* ---------------------------------------------------------------- context */

typedef struct gsr_context gsr_context;

gsr_context* gsr_create(void);
void gsr_destroy(gsr_context* ctx);

/* Pre-size the workspace for n Gaussians and `pairs` (tile, Gaussian) pairs. */
int gsr_reserve(gsr_context* ctx, int64_t n, int64_t pairs);

/* Whole frame, stream-ordered (stream = hipStream_t or NULL for the default
 * stream).  d_out: DEVICE buffer of 3*W*H floats (planar, row 0 = bottom).
 * Reference tiling arguments as in preprocessCUDAGaussians; pass
 * num_tile_x = num_tile_y = 1 and strides = W, H for "cover the image".
 * Returns GSR_E_OVERFLOW if an earlier frame was incomplete (pair buffer
 * overflow, grown; a depth sort short of passes, budget reset; or a speculative
 * depth-split frame that needed phase B): re-render every frame since the last
 * clean return, see GSR_E_OVERFLOW. */
int gsr_render(gsr_context* ctx, const void* d_scene, int layout, int64_t n,
               const gsr_camera* cam, int W, int H, int num_tile_x, int num_tile_y,
               int width_stride, int height_stride, float k, float* d_out, void* stream);

/* Offline camera path (config 4 on one GPU; the reference has no batch entry
 * point — it renders one frame per preprocessCUDAGaussians call, render.cu:871):
 * frame i renders cams[i] (at times[i] for 4D scenes; times may be NULL) into
 * the DEVICE buffer d_outs[i], each frame exactly as gsr_render would.  Up to
 * gsr_set_frames_in_flight() frames run concurrently: frame i goes to lane
 * i % F, lane 0 being this context on `stream` and lanes 1..F-1 private child
 * contexts (own workspaces) on their own streams, so one frame's latency-bound
 * sort and binning kernels overlap another frame's VALU-bound blend.
 * Stream-ordered: the frames start after the work already queued on `stream`
 * (fork event), and work queued on `stream` after the call sees all nframes
 * images (join events).  Outputs may repeat (e.g. a ring of buffers); a frame
 * whose output an in-flight frame of another lane also writes waits for it.
 * Readbacks, timing and diagnostics refer to lane 0's last frame.  Returns
 * GSR_E_OVERFLOW when an earlier frame of any lane was incomplete (see
 * GSR_E_OVERFLOW; every frame since the last clean return re-renders). */
#define GSR_MAX_FRAMES_IN_FLIGHT 8
int gsr_render_path(gsr_context* ctx, const void* d_scene, int layout, int64_t n, const gsr_camera* cams,
                    const float* times, int nframes, int W, int H, int num_tile_x, int num_tile_y,
                    int width_stride, int height_stride, float k, float* const* d_outs, void* stream);
/* gsr_render_path with per-frame completion events, for consumers that hand each
 * finished frame on (the multi-GPU gather) while later frames still render.
 * frame_events (may be NULL; entries may be NULL): hipEvent_t frame_events[i] is
 * recorded on frame i's lane right after its blend.  flags & GSR_PATH_NO_JOIN:
 * skip the join, so `stream` orders after lane 0's frames only and the lanes keep
 * running into the next call without a pipeline drain (a later call's lanes still
 * start after the work queued on `stream` before it).  Without the join the caller
 * orders everything else through the events: reading frame i, and re-using one of
 * this call's output buffers in a later call (wait for the buffer's last frame). */
#define GSR_PATH_NO_JOIN 1
/* flags & GSR_PATH_NO_FORK: lanes 1..F-1 do not wait for `stream` (lane 0 still runs
 * on it), so they are never held behind lane 0's frames of an earlier call (with the
 * fork, chunked calls cost ~4 % of the in-flight rate); the caller orders the frames
 * after its own work through wait_events instead. */
#define GSR_PATH_NO_FORK 2
/* wait_events (may be NULL; entries may be NULL): frame i's lane waits for
 * hipEvent_t wait_events[i] before rendering frame i (e.g. the hand-off of the frame
 * that last used d_outs[i]). */
int gsr_render_path_ex(gsr_context* ctx, const void* d_scene, int layout, int64_t n, const gsr_camera* cams,
                       const float* times, int nframes, int W, int H, int num_tile_x, int num_tile_y,
                       int width_stride, int height_stride, float k, float* const* d_outs, void* stream,
                       void* const* frame_events, void* const* wait_events, int flags);
/* gsr_render_path_ex with a validity word per frame, so a consumer that receives
 * frames asynchronously (the multi-GPU gather) knows exactly which ones to render
 * again instead of every frame since the last clean return.  d_status (may be NULL;
 * entries may be NULL): a uint32 DEVICE word per frame, written on frame i's lane
 * before its frame event: 0 if frame i is complete, else GSR_FRAME_* bits (the causes
 * of GSR_E_OVERFLOW, for that frame alone).  The word can sit right after the
 * frame's image in one buffer, so it travels with the frame.  The return code, the
 * buffer growth and the controller are exactly those of gsr_render_path_ex. */
#define GSR_FRAME_PAIR_OVERFLOW 1u   /* its pairs overflowed the pair buffer */
#define GSR_FRAME_DEPTH_PASSES 2u    /* its depth sort needed more passes than were launched */
#define GSR_FRAME_SPEC_MISS 4u       /* speculative depth-split frame that needed phase B */
int gsr_render_path_status(gsr_context* ctx, const void* d_scene, int layout, int64_t n, const gsr_camera* cams,
                           const float* times, int nframes, int W, int H, int num_tile_x, int num_tile_y,
                           int width_stride, int height_stride, float k, float* const* d_outs, void* stream,
                           void* const* frame_events, void* const* wait_events, int flags,
                           uint32_t* const* d_status);
/* Frames in flight for gsr_render_path: 1..GSR_MAX_FRAMES_IN_FLIGHT (default 3;
 * 1 = strictly sequential on `stream`).  Each extra lane holds its own workspace. */
int gsr_set_frames_in_flight(gsr_context* ctx, int frames);
int gsr_frames_in_flight(gsr_context* ctx);

/* The three stages of gsr_render, callable separately (same stream). */
int gsr_preprocess(gsr_context* ctx, const void* d_scene, int layout, int64_t n,
                   const gsr_camera* cam, int W, int H, int num_tile_x, int num_tile_y,
                   int width_stride, int height_stride, float k, void* stream);
int gsr_sort(gsr_context* ctx, void* stream);
int gsr_blend(gsr_context* ctx, float* d_out, void* stream);

/* Frame time t for GSR_LAYOUT_SCENE_BLOCK_4D scenes (config 5):
 * dt = t - trbf_center; position = xyz + m0..2*dt + m3..5*dt^2 + m6..8*dt^3;
 * opacity = sigmoid(opacity) * exp(-(dt / trbf_scale)^2).  Gaussians whose
 * temporal opacity is below 0.9e-3 (and whose 2D conic is robustly positive
 * definite) are culled in preprocess: they could never reach alpha >= 1e-3,
 * so the image equals the uncut render. */
int gsr_set_time(gsr_context* ctx, float t);

/* Wait for all work of the context (every lane); returns GSR_E_OVERFLOW if any
 * frame since the last clean check was incomplete — including one that a
 * non-blocking check inside a render call already reported — and grows the
 * buffer / resets the pass budget. */
int gsr_sync(gsr_context* ctx);

/* ---- readback (synchronous; for tests and tooling) ---- */

/* Number of (tile, Gaussian) pairs of the last frame's tile rects (before the capacity
 * clamp; an upper bound of the pairs listed when GSR_TUNE_TILE_SPANS drops some). */
int64_t gsr_pair_count(gsr_context* ctx);
/* Number of (tile row, Gaussian) items the last frame's row pass produced (tile
 * binning), or -1 if that frame used pair emission + the key-value tile sort. */
int64_t gsr_row_item_count(gsr_context* ctx);
/* Per-Gaussian splat records (n * GSR_SPLAT_RECORD_BYTES bytes):
 *   float inv_covar[4]; float opacity; float color[3];
 *   int32 px_x, px_y; uint32 x_range (xmin | xmax<<16); uint32 y_range;
 *   uint32 tile_x_range; uint32 tile_y_range; uint32 tile_count; uint32 depth_key.
 * Culled / invalid Gaussians have tile_count 0 and depth_key 0xFFFFFFFF;
 * their other fields are unspecified. */
int gsr_read_splats(gsr_context* ctx, void* host_records, int64_t n);
/* (depth_key << 32 | index) items after the depth sort, n of them.  A frame
 * that used the per-tile depth order has no global one: it is computed here
 * (stable sort of that frame's keys, the same kernels as the global path). */
int gsr_read_depth_order(gsr_context* ctx, uint64_t* host_items, int64_t n);
/* (tile << 32 | index) pairs the tile lists hold, in tile order; returns the count copied. */
int64_t gsr_read_pairs(gsr_context* ctx, uint64_t* host_pairs, int64_t cap);
/* Internal tile grid of the last frame and its [start, end) ranges. */
int gsr_tile_grid(gsr_context* ctx, int* tiles_x, int* tiles_y);
int gsr_read_tile_ranges(gsr_context* ctx, uint32_t* host_ranges, int64_t num_tiles);

/* ---- per-stage device timing with hipEvents on the render stream ----
 * mode 0 = off, 1 = blend only (two events per frame), 2 = every stage. */
int gsr_set_timing(gsr_context* ctx, int mode);
/* Same, recording the events on every `stride`-th frame only (frames 0, k, 2k, …
 * after the call); gsr_stage_times then averages over the recorded frames. */
int gsr_set_timing_stride(gsr_context* ctx, int mode, int stride);
/* Sums of per-stage device milliseconds and the number of frames timed since
 * the last call (synchronises, then resets). */
int gsr_stage_times(gsr_context* ctx, double* ms_out /* GSR_NUM_STAGES */, int64_t* frames);

/* Diagnostics (off by default): when on, the blend counts the splat records
 * it actually loads (Pc of SURVEY.md 8d: pairs consumed before every pixel of
 * a tile saturates); gsr_blend_records_loaded() returns the last frame's Pc. */
int gsr_set_diagnostics(gsr_context* ctx, int on);
int64_t gsr_blend_records_loaded(gsr_context* ctx);
/* All blend counters of the last diagnostics frame (8 values): {records
 * loaded (Pc), wave-splat iterations, active lanes (in AABB and not
 * saturated), lanes that composited, iterations on the exact one-splat
 * path (default schedule; batches without the fast-path proof),
 * iterations skipped by the per-splat md2 cutoff (variant 5), pixel-lane slots
 * (64 x pixels per lane x iterations), 0};
 * lane efficiency = active / slots. */
int gsr_blend_counters(gsr_context* ctx, int64_t* out8);
/* The first n (<= 16) blend counters: the 8 above, then {blocks the fast-exp blend
 * handed to the exact blend, their suspect pixels}. */
int gsr_blend_counters_ex(gsr_context* ctx, int64_t* out, int n);
/* Take map of the last diagnostics frame: per pixel (row-major, n = W * H), the
 * number of splats composited (low 32 bits) and the sum over them of
 * (gaussian index + 1) * 2654435761 mod 2^32 (high 32 bits).  The oracle's
 * orc_render_takes computes the same map, so the tests compare which splats
 * every pixel composited, not only the colours. */
int gsr_blend_take_map(gsr_context* ctx, uint64_t* out, int64_t n);
/* Blend schedule: 0 = one 64-thread workgroup per 8x8 pixel block (the
 * kernel); 3 = the same with per-wave timestamps instead of counters (see
 * gsr_blend_stamps; diagnostics frames only).  Other values are refused (the
 * tile-per-workgroup schedule, longest-tiles-first, several blocks per wave or
 * workgroup and LDS-capped occupancy were measured slower and removed). */
int gsr_set_blend_variant(gsr_context* ctx, int variant);
/* Tuning knobs for A/B experiments (all settings give bit-identical output, except
 * GSR_TUNE_BLEND_EXP: its modes composite the same splats on every pixel and differ in
 * the colours by < 1e-6). */
enum {
    GSR_TUNE_BLEND_SCHEDULE = 0,     /* as gsr_set_blend_variant */
    GSR_TUNE_TILE_SORT_ITEMS = 1,    /* tile sort items per thread: 8 | 16 (default 16) */
    GSR_TUNE_DEPTH_SORT_ITEMS = 2,   /* depth sort items per thread: 0 = by size | 8 | 16 (16 sorts one
                                        4,096-item tile per workgroup: a grid too small for that, e.g.
                                        capped by knob 4, sorts 8 per thread) */
    GSR_TUNE_TILE_SORT_GROUPS = 3,   /* tile sort workgroup cap (default 1024; 0 = one per tile of items) */
    GSR_TUNE_DEPTH_SORT_GROUPS = 4,  /* depth sort workgroup cap (0 = one per tile of items) */
    GSR_TUNE_TILE_SORT_SPLIT = 5,    /* tile sort digits: 1 = split evenly (default), 0 = 8 bits first */
    GSR_TUNE_DEPTH_SORT_SKIP = 6,    /* depth sort: 1 = skip trailing identity passes (default), 0 = run all 4 */
    GSR_TUNE_TILE_BINNING = 7,       /* 1 = row + column binning (default; tile grids <= 256 x 256),
                                        0 = pair emission + key-value tile sort */
    GSR_TUNE_BIN_ROW_ITEMS = 8,      /* binning row pass: items per thread per tile 4 | 8 | 16 (default 4) */
    GSR_TUNE_BIN_COL_ITEMS = 9,      /* binning column pass: items per thread per tile 4 | 8 | 16 (default 8) */
    GSR_TUNE_BIN_COL_GROUPS = 10,    /* binning column pass: workgroups (default 0 = n / 1024 clamped
                                        to 1024..4096) */
    GSR_TUNE_COMPLETION_EVENTS = 11, /* 1 (default): a completion event feeds the non-blocking overflow
                                        check; 0: none (frames captured into a graph).  With 0 the
                                        render calls report nothing: only gsr_sync (which drains the
                                        device, then reads the sticky overflow words) reports an
                                        incomplete frame, and no frame is rendered speculatively
                                        without the depth split's phase B (a graph would replay that
                                        choice) */
    /* 12 reserved (removed: longest tiles first) */
    GSR_TUNE_BLEND_BAND_TILES = 13,  /* blend schedule 0: tiles per spatial band, bands dealt round-robin
                                        to the 8 XCDs (default 4); 0 = one contiguous band per XCD */
    /* 14-17 reserved (removed, all measured slower: two blocks per workgroup, per-tile depth
       order after index-order binning (config 3: 1.53 ms vs 0.24 ms), several blocks per wave,
       LDS-capped blend occupancy) */
    GSR_TUNE_DEPTH_COMPACT = 18,     /* global depth sort on the binning path: 1 = stable partition of the
                                        visible Gaussians first, the passes sort only those; 0 = sort all;
                                        2 (default) = partition for 4D scenes only; same order, same image */
    GSR_TUNE_TILE_SPANS = 19,        /* binning path: 1 = list a splat in only the tiles of its first four
                                        tile rows it can composite on (conservative ellipse-vs-tile test);
                                        0 = every tile of its rect; 2 (default) = 1 up to 1.5M Gaussians;
                                        same image */
    GSR_TUNE_RANK_ATOMIC = 20,       /* stable digit ranks in the depth sort and both binning scatters:
                                        1 (default) = from returning LDS atomics, taken only on a gfx950
                                        device that passed the one-shot rank-order self-check
                                        (gsr_rank_order_check) when the context first ran; 0 = ballot
                                        matching.  The environment variable GSR_RANK_ATOMIC=0 makes 0
                                        the default.  Same order, same image */
    GSR_TUNE_RANK_ATOMIC_ACTIVE = 21, /* read-only: 1 if the atomic ranks are in use (knob 20 at 1 and the
                                        self-check passed), 0 if the kernels rank with ballots */
    GSR_TUNE_BLEND_EXP = 22,         /* blend exp.  1 (default since round 4) = hardware exp for
                                        alpha, with the alpha test exact on the exp argument and the
                                        transmittance test guarded by a proven band; pixels whose T
                                        decision the band cannot vouch for are blended again exactly.
                                        Every pixel composites exactly the oracle's splats (take map
                                        identical); colours within 1e-6 of the exact blend (measured
                                        <= 4e-7).  0 (environment GSR_BLEND_EXP=0 selects it) =
                                        gsr_blend_expf throughout: bit-exact with the oracle.  Depth-
                                        split frames (GSR_TUNE_DEPTH_SPLIT) always run the exact blend.
                                        2 = test hook: 1 with a 100 % guard band, so every block
                                        in which a pixel saturates is blended again exactly. */
    GSR_TUNE_DEPTH_SPLIT = 23,       /* binning path, exact blend, gsr_render / gsr_render_path: 1 = bin
                                        the nearest part of the depth order first and blend it (phase
                                        A), then bin the rest and resume only the 8x8 blocks phase A
                                        left unsaturated (phase B, skipped on the device when there are
                                        none).  After the first split frame the items are partitioned
                                        by a depth threshold and only the near part is sorted (phase B
                                        sorts the far part when it runs); the split point adapts to the
                                        frames seen, and once it cannot shrink further frames are
                                        rendered without phase B until one needs it (that frame returns
                                        GSR_E_OVERFLOW: render it again).  A split point grown to 1000
                                        turns it off; it is tried again 256+ frames later, only on
                                        another camera.  0 = one phase; 2 (default) =
                                        1 above 1.5M Gaussians.  Same image.  After a split frame
                                        gsr_read_pairs / gsr_read_tile_ranges hold the lists of its last
                                        phase, and after a threshold split gsr_read_depth_order is refused */
    GSR_TUNE_DEPTH_SPLIT_PERMILLE = 24, /* the current split point: phase A bins the nearest
                                        ceil(n * value / 1000) of the depth order (adapted per frame; a
                                        set value is a new starting point, 1..999) */
    GSR_TUNE_DEPTH_SPLIT_UNSAT = 25, /* read-only: 8x8 blocks the last completed split frame's phase A
                                        left unsaturated (0: its phase B did nothing); read after gsr_sync */
    GSR_TUNE_DEPTH_SPLIT_STATE = 26, /* read-only: how the last sorted frame ran: 0 one phase; 1 split,
                                        whole depth order sorted (count mode: the first split frame);
                                        2 split by a depth threshold (near part sorted, far part sorted
                                        in phase B); 3 as 2 with no phase B queued (speculative: a frame
                                        that then leaves a block unsaturated is reported as
                                        GSR_E_OVERFLOW and rendered again by the caller) */
    /* 27 reserved (removed, measured slower: the preprocess building the depth sort's pass-0
       histograms in 512-thread workgroups of 2048 Gaussians, pass 0 without its upsweep launch:
       preprocess 49.4 -> 60.3 us against the 5.7-us upsweep, -1.1 % one frame at a time and
       -1.2 % in flight, profiles/r04_ab_pre_hist.txt) */
    GSR_TUNE_DEPTH_BUCKETS = 28,     /* binning path, frames not split by a depth threshold: 1 (default) =
                                        bucket depth sort: one stable scatter of the preprocess order into
                                        depth buckets bounded by the previous frame's quantiles, then one
                                        workgroup per bucket sorts it in LDS.  Up to 2,097,152 Gaussians
                                        ~n/1024 buckets (at most 4,096) of up to 2,048 items per 256-thread
                                        workgroup (larger buckets are sorted through global memory by their
                                        workgroup); above, 512 buckets of up to 16,384 items per 1,024-thread
                                        workgroup (larger or wider-keyed ones go to the first kind's
                                        paths in a second launch).  A context's first frame of a scene size
                                        runs the LSD passes and takes the quantiles from them, and so does
                                        the first frame of another scene pointer, and the frame after one
                                        whose global path ran more than n/8 item-passes (a camera cut; knob
                                        33).  0 = LSD passes only; 2 = test hook: 1 with a 64-item local
                                        capacity in either kind (no reseeding on overflow); 3 = the first
                                        kind at any scene size (A/B).  Same order, same image;
                                        gsr_depth_passes is 0 after a bucket-sorted frame */
    GSR_TUNE_DEPTH_BUCKETS_OVER = 29, /* read-only: items the bucket sort's global path has sorted (buckets
                                        over the local capacity), summed over the lanes; sticky, read
                                        after gsr_sync */
    GSR_TUNE_BUCKET_ROWS = 30,       /* 1 (default): on a bucket-sorted frame binned once over the whole
                                        depth order, each bucket's workgroup also counts the row pass's
                                        items and pairs (the bucket is the row pass's chunk), so the row
                                        pass runs without its count kernel; 0 = the row pass counts.
                                        Same lists, same image */
    GSR_TUNE_COL_CHUNK = 31,         /* binning path: row items per column-pass chunk.  0 (default) =
                                        1024 for scenes of at most 2,097,152 Gaussians, else 2048;
                                        1024 or 2048 forces it.  Same lists, same image */
    GSR_TUNE_FAIL_FRAME = 32,        /* test hook: v > 0 makes the next gsr_render_path* call fail its
                                        frame v with GSR_E_ARG (once; 0 = off, the default).  The
                                        frames queued before it are still joined to the caller's
                                        stream */
    GSR_TUNE_DEPTH_BUCKETS_WORK = 33 /* read-only: the global path's items times the 8-bit passes each
                                        took (their bucket's key span; tied keys take none), summed
                                        over the lanes; sticky, read after gsr_sync.  A frame adding
                                        more than n/8 makes the next frame reseed the splitters */
};
int gsr_set_tuning(gsr_context* ctx, int knob, int value);
/* Current value of a knob (what gsr_set_tuning last set, else the default). */
int gsr_get_tuning(gsr_context* ctx, int knob, int* value);
/* Device self-check behind GSR_TUNE_RANK_ATOMIC: wave64 instructions whose lanes
 * add to the same LDS address with a returning atomic (ds_add_rtn_u32) on the
 * current device, over 24 digit patterns, compared lane by lane with the stable
 * ranks ballot matching gives.  *lane_ops = lanes checked, *mismatches = lanes
 * whose returned value was out of lane order.  The ISA does not document that
 * order; contexts run this once per process and device and rank with ballots if
 * any lane mismatches or the device is not gfx950.  Synchronous, < 1 ms. */
int gsr_rank_order_check(int64_t* lane_ops, int64_t* mismatches);
/* Depth-sort digit passes the last sorted frame ran (1..4; trailing identity
 * passes are skipped on the device), or a negative error code. */
int gsr_depth_passes(gsr_context* ctx);
/* Bucket depth sort diagnostics (GSR_TUNE_DEPTH_BUCKETS) of the last sorted frame of the
 * context (lane 0 of gsr_render_path): its bucket count B, or 0 when that frame was not
 * bucket-sorted, and each bucket's item count into sizes[0 .. min(B, cap)) (bucket B - 1
 * holds the items with key 0xFFFFFFFF: the culled ones).  Synchronizes the context. */
int gsr_bucket_sizes(gsr_context* ctx, uint32_t* sizes, int cap);
/* Schedule 3: with diagnostics on, the last frame's blend stores per wave
 * (launch order) {start of the 100 MHz s_memrealtime clock, duration (40 bits) |
 * placement << 40 (XCC id, HW_ID)}; read n values. */
int gsr_blend_stamps(gsr_context* ctx, uint64_t* out, int64_t n);

/* ---------------------------------------------------------------- scenes */

/* Upload a host SoA scene (GSR_SCENE_NARRAYS arrays of n floats, contiguous,
 * already activated as by the loader) into a new device scene block. */
void* gsr_scene_upload(const float* host_soa, int64_t n);
/* narrays = GSR_SCENE_NARRAYS (3D), GSR_SCENE4D_NARRAYS (4D) or GSR_SCENE_SH3_NARRAYS. */
void* gsr_scene_upload_ex(const float* host_soa, int narrays, int64_t n);
void gsr_scene_free(void* d_scene);
/* Bytes of a scene block (header + narrays arrays of n floats, padded), or a
 * negative error code. */
int64_t gsr_scene_bytes(int narrays, int64_t n);
/* Copy a whole device scene block (n Gaussians, narrays arrays: checked against its
 * header) into d_dst, a device buffer of gsr_scene_bytes(narrays, n) bytes, on
 * `stream` — e.g. into a buffer that a collective then broadcasts to the other
 * ranks (the multi-GPU scene replication; the copy is a valid scene block). */
int gsr_scene_copy(void* d_dst, const void* d_scene, int narrays, int64_t n, void* stream);
/* Copy a device scene block back into host SoA form (38 * n floats). */
/* Copies every array of the block (38, 49 for 4D, 59 for SH-3) into host_soa. */
int gsr_scene_download(const void* d_scene, float* host_soa, int64_t n);

/* ---------------------------------------------------------------- host helpers */

/* PLY reader with the semantics of loadGaussianCudaFromPly (misc.cu:13-134 +
 * storeGaussianFromProperty gaussians.cpp:17-30), host side only.  Call with
 * host_soa == NULL to get the count; then with a buffer of 38*n floats. */
int gsr_ply_read_host(const char* path, float* host_soa, int64_t capacity, int64_t* n_out);
/* Same with flags (GSR_PLY_TYPED, GSR_PLY_SH3) and narrays = 38, 49 (4D arrays
 * filled when present; defaults trbf_center 0, trbf_scale 1, motion 0) or 59
 * (with GSR_PLY_SH3); *is_4d (if non-NULL) reports whether the file has the 4D
 * properties. */
int gsr_ply_read_host_ex(const char* path, float* host_soa, int narrays, int64_t capacity, int64_t* n_out,
                         int flags, int* is_4d);

/* Seeded synthetic scene: writes a standard 62-property
 * binary_little_endian 3DGS .ply, or fills raw (pre-activation) property
 * values.  Same generator, same values, for a given (n, seed). */
int gsr_synth_write_ply(const char* path, int64_t n, uint64_t seed);
/* Config 5 4D synthetic scene: the 62 properties plus trbf_center U(0,1),
 * trbf_scale U(-3.5,-2) (log), motion_0..8 N(0, .5 | .2 | .1). */
int gsr_synth_write_ply4d(const char* path, int64_t n, uint64_t seed);

/* Camera (camera.cpp): Camera() ctor 8-13, updateCameraMatrices 36-57,
 * updateFrustumPlanes 59-121, zoom 123-128, orbit 130-158. */
void gsr_camera_default(gsr_camera* cam);
void gsr_camera_update(gsr_camera* cam);
void gsr_camera_update_frustum(gsr_camera* cam);
void gsr_camera_zoom(gsr_camera* cam, float delta);
void gsr_camera_orbit(gsr_camera* cam, float azimuth_deg, float elevation_deg);
/* fx, fy exactly as render.cu:620-621 (tanf computed correctly rounded). */
void gsr_camera_intrinsics(const gsr_camera* cam, float* fx, float* fy);

/* Device self-test used by the parity tests: for each (x, y) pair of host_in
 * (2n floats) evaluates on the GPU {gsr_expf(x), gsr_sinf(x), gsr_cosf(x),
 * gsr_atan2f(x, y), sqrtf(x), x / y, roundf(x), bits(gsr_f2i_sat(1000x)),
 * gsr_blend_expf(x)} into host_out (9n floats), so the CPU twins can be compared
 * bit for bit. */
int gsr_math_probe(const float* host_in, int n, float* host_out);
/* Exhaustive device checks of the blend's exp, over every float x in [x_lo, x_hi):
 * *violations = the number of x with gsr_blend_expf(x) > gsr_blend_expf(next x)
 * (0: the exact exp is monotone, so the alpha test is a threshold on -md2/2);
 * *err_all / *err_big = the largest |fast exp / gsr_blend_expf - 1|
 * (GSR_TUNE_BLEND_EXP 1) over the range / over x >= x_big (rounded up).
 * violations points at ONE int64 (the round-3 signature, unchanged). */
int gsr_exp_probe(float x_lo, float x_hi, float x_big, int64_t* violations, float* err_all, float* err_big);
/* gsr_exp_probe plus *packed_mismatches = the number of x in [-2e7, 5] (and of -x
 * there) where the packed compositing loop's exp differs from gsr_blend_expf
 * (0: the packed and scalar exps agree bit for bit).  Each pointer names one value. */
int gsr_exp_probe2(float x_lo, float x_hi, float x_big, int64_t* violations, int64_t* packed_mismatches,
                   float* err_all, float* err_big);
/* gsr_alpha_take_min_x (gsr_detmath.h) evaluated on the device for n opacities. */
int gsr_alpha_cut_probe(const float* host_op, int n, float* host_out);

const char* gsr_last_error(void);
const char* gsr_version(void);
/* 1 if a HIP device is usable, else 0 (never aborts). */
int gsr_device_available(void);

#ifdef __cplusplus
}  /* extern "C" */

#include <string>
/* misc.cuh:4 — C++ linkage, same mangled name as the reference's loader. */
gsr_gaussian* loadGaussianCudaFromPly(const std::string& filename, int* out_numGaussians);
#endif

#endif /* GSR_H */
