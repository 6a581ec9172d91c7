// gsr_internal.h — shared between the host runtime (gsr_runtime.cpp) and the
// gfx950 kernels (gsr_kernels.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "gsr_types.h"

namespace gsr {

// Set the thread's last error (gsr_last_error) and return `code`.
int set_error(int code, const char* fmt, ...);


// Per-frame constants, passed by value to the kernels.
struct Frame {
    float V[16];        // view matrix (camera.cpp:53, row-major)
    float P[16];        // projection (math.cpp:91-97)
    float Rc[9];        // r_cam
    float RcT[9];       // r_cam_T
    float campos[3];
    float znear;
    float fx, fy;       // render.cu:620-621 (host-computed, shared with the oracle)
    float k;            // sigma multiplier
    int W, H;           // image size (tile_W, tile_H of the reference ABI)
    int cover_w, cover_h;   // pixels covered by the reference tile grid
    int tiles_x, tiles_y;   // internal GSR_TILE_PX tiles
};

// Radix-sort geometry.
constexpr int kSortThreads = 256;
constexpr int kSortTile = kSortThreads * 16;           // largest tile (items = 16 per thread)
constexpr int kMaxSortGroups = 8192;                    // grid upper bound (hist: 256 x this)

// Device-side frame statistics block (device memory).
struct Stats {
    unsigned long long pairs_total;   // P before the capacity clamp
    uint32_t pairs_eff;               // min(P, capacity): what sort/ranges/blend consume
    uint32_t overflow;                // bit 0: P > capacity; bit 1: the depth sort needed more
                                      // passes than were launched (depth pass budget)
    uint32_t depth_passes;            // passes the depth sort's device plan needed (binning path; 0: n/a)
    uint32_t split_unsat;             // depth split: blocks the last phase-A blend left unsaturated
                                      // (written to the host-mapped copy by the phase-B blend)
    uint32_t split_pm;                // the split point of the frame whose split_unsat that is, | the
                                      // controller's epoch << 16 (gsr_runtime.cpp split_tag)
    uint32_t spec_miss;               // depth split without phase B (speculative): a phase-A blend
                                      // left a block unsaturated, the frame is incomplete (host copy,
                                      // sticky until the host reads it)
    unsigned int bkt_over;            // bucket depth sort: items of buckets over the local capacity,
                                      // sorted through global memory (host copy, sticky diagnostics)
    unsigned int bkt_over_work;       // ... times the 8-bit passes each needed (their keys' span): the
                                      // cost of the global path (tied keys cost none; host copy, sticky)
};

// Depth split (GSR_TUNE_DEPTH_SPLIT): the frame's tiles are binned over the nearest
// part of the depth order first (phase A); its blend saves the transmittance of
// every block it leaves unsaturated, and phase B bins the rest of the depth order
// and resumes those blocks.  phase: 1 = A (save), 2 = B (resume).
// Depth split, key mode: pass 0 of a depth sort reads the whole preprocess order and
// keeps key < *kcut (mode 1, the near part: the kept count goes to *count_out and the
// threshold is copied to *kcut_copy) or key >= *kcut (mode 2, the far part, written from
// the pass's base; with sat, only items whose tile rect holds a tile phase A left
// unsaturated — the summed-area table of k_split_sat, sat_w = tiles_x + 1 — and the kept
// count goes to *count_out).  mode 0 with count: a later far pass, length *count.
struct SortFilter {
    int mode;
    const uint32_t* kcut;
    uint32_t* count_out;
    uint32_t* kcut_copy;
    const uint32_t* sat;
    int sat_w;
    const uint32_t* count;
};

// Depth split, key mode: the preprocess writes splat records only for Gaussians nearer
// than the frame's threshold (mode 1; it copies *kcut to *kcut_frame for mode 2); mode
// 2 (phase B, or a frame that ends up not split) writes only the far ones' records and
// nothing else, and returns at once when *gate is 0 (gate nullptr: always runs).
struct RecSplit {
    int mode;
    const uint32_t* kcut;
    uint32_t* kcut_frame;
    const uint32_t* gate;
};

// Depth split with a threshold partition (the near part sorted, the far part sorted
// inside phase B): cut_mode 1 = the row pass reads [0, *cut), 2 = [*cut, n); na = the
// host's split point (positions), sizes phase A's grid.
struct RowSplit {
    int cut_mode;
    uint32_t na;
    const uint32_t* cut_n;            // mode 2: the far part's kept length (a masked far sort)
};

// The next frame's depth threshold (its partition puts keys < *kcut in the near part),
// computed by phase A's blend from this frame's near depth order (gsr_kernels.hip
// split_cut_update).  kcut == nullptr: no update.
struct SplitCut {
    const uint64_t* items0;
    const uint64_t* items1;
    const uint32_t* dstats;           // the near sort's pass plan (which buffer holds the result)
    const uint32_t* nnear;            // near count (nullptr: this frame sorted the whole order)
    uint32_t n, na;                   // items, the split point (positions)
    uint32_t* kcut;
};

struct BlendSplit {
    int phase;
    float* tbuf;                      // 64 floats per 8x8 block (4 blocks per tile)
    uint8_t* bflag;                   // per block: 1 = left unsaturated by phase A (tbuf valid)
    uint32_t* gate;                   // count of such blocks (cleared by phase A's row scan)
    Stats* host_st;                   // phase B publishes the count here (nullable)
    Stats* spec_host;                 // phase A with no phase B queued: an unsaturated block sets
                                      // spec_host->spec_miss (nullable)
    SplitCut cut;                     // phase A: the next frame's threshold; phase B: nnear and na only
                                      // (a near part short of the split point is tagged unmeasured)
    uint32_t pm;                      // phase B publishes it with the count (Stats::split_pm: the split
                                      // point | the controller's epoch << 16)
    uint32_t* fstatus;                // speculative phase A: an unsaturated block ors
                                      // GSR_FRAME_SPEC_MISS into the frame's validity word (nullable)
};

// ---- launch wrappers (gsr_kernels.hip) ----
hipError_t launch_aos_to_soa(const gsr_gaussian* aos, int64_t n, float* arrays, int64_t stride,
                             hipStream_t s);
hipError_t launch_preprocess(const float* arrays, int64_t stride, int64_t n, const Frame& fr,
                             uint4* rec, uint64_t* items, uint64_t* rect, bool packed, bool four_d, bool sh3,
                             float t, hipStream_t s, uint16_t* spans = nullptr,
                             const RecSplit* rs = nullptr);
// One stable LSD pass over u64 items on bits [shift, shift + bits) (bits <= 8).
// n = n_dev ? *n_dev : n_host.  hist: 256 * groups u32, totals: 256 u32.
// ranges (nullable, final tile-sort pass): per-tile {~start, end} of key (item >> 32),
// zeroed beforehand.
// items: 8 or 16 per thread (tile = 256 * items); groups from sort_groups().
// dstats (nullable): depth-sort pass plan, zeroed per frame; pass 0 fills it,
// passes >= 1 skip themselves when they would be identities (gsr_kernels.hip).
hipError_t launch_radix_pass(const uint64_t* in, uint64_t* out, const uint32_t* n_dev, uint32_t n_host,
                             int shift, int bits, int groups, int items, uint32_t* hist, uint32_t* totals,
                             uint2* ranges, hipStream_t s, uint32_t* dstats = nullptr, int pass = 0,
                             const uint32_t* rect = nullptr, int rect_direct = 0, uint32_t* pay0 = nullptr,
                             uint32_t* pay1 = nullptr, bool rank_atomic = false,
                             const uint32_t* base_dev = nullptr, const uint32_t* gate = nullptr,
                             const SortFilter* filter = nullptr);
// Bucket depth sort (binning path; gsr_kernels.hip "bucket depth sort"): the stable
// (depth key, index) order of the n items `in` (the preprocess order; rect = its packed
// tile rects by position) into items0 with the rects into pay0; items1 / pay1 are scratch.
// buckets: 256..4096 (a power of two); s_in: its buckets - 1 sorted splitters (the last
// 0xFFFFFFFF); s_out: the next frame's (quantiles of this order).  hist: groups x buckets
// u32 (groups <= kMaxBucketGroups), totals: 2 x buckets + 2 u32 (the totals, then the
// buckets' first positions and n, then a word raised when a live item has key 0xFFFFFFFF).  cap (<= kMaxBucketCap): largest bucket sorted in LDS (larger
// ones take the global path; over_host, host-mapped and nullable, counts their items, and
// over_host[1] their items times the passes they took).
constexpr int kMaxBuckets = 4096;
constexpr uint32_t kMaxBucketCap = 2048;
constexpr int kMaxBucketGroups = 512;    // chunks (workgroups) of the scatter; hist: groups x buckets
hipError_t launch_bucket_sort(const uint64_t* in, uint64_t* items0, uint64_t* items1, uint32_t n, int buckets,
                              int groups, const uint32_t* s_in, uint32_t* s_out, uint32_t* hist, uint32_t* totals,
                              const uint32_t* rect, uint32_t* pay0, uint32_t* pay1, bool rank_atomic, uint32_t cap,
                              unsigned int* over_host, hipStream_t s, int row_tiles_y, uint4* rec);
// rec: n 16-B records of scratch (the scatter's output, the local sorts' input).
// row_tiles_y > 0: the local kernel also writes the row pass's count histograms into hist
// (512 x buckets words: chunk g = bucket g, tile rows < row_tiles_y; the last bucket's chunk
// is empty unless a live item's key saturated to 0xFFFFFFFF), and the row pass then runs
// with buckets chunks, cstart = totals + buckets (the buckets' first positions) and no count
// kernel.
// Big buckets (scenes above 2M Gaussians): `buckets` (kBigBuckets = 512: ~n / 512 items each,
// sorted by one 1,024-thread workgroup in LDS, up to 16,384 items; or 1,024: ~n / 1,024 items
// by 512-thread workgroups, up to 8,192, two per CU) bounded by the previous frame's quantiles;
// larger or wider-keyed buckets are sorted by launch_bucket_sort's local kernel in a second
// launch.  The scatter writes each tile in bucket order (coalesced 12-B records).
// groups <= kBigBucketGroups.  No fused row count.
constexpr int kBigBuckets = 512;
constexpr int kBigBucketGroups = 1024;
hipError_t launch_bucket_sort_big(const uint64_t* in, uint64_t* items0, uint64_t* items1, uint32_t n, int buckets,
                                  int groups, const uint32_t* s_in, uint32_t* s_out, uint32_t* hist, uint32_t* totals,
                                  const uint32_t* rect, uint32_t* pay0, uint32_t* pay1, bool rank_atomic, uint32_t cap,
                                  unsigned int* over_host, hipStream_t s, uint4* rec);
// Splitters for launch_bucket_sort from an order the LSD passes sorted (depth_sorted of
// items0 / items1 under dstats); live_dev (nullable): its visible count.
hipError_t launch_bkt_splitters(const uint64_t* items0, const uint64_t* items1, const uint32_t* dstats, uint32_t n,
                                const uint32_t* live_dev, int buckets, uint32_t* s_out, hipStream_t s);
// Pair emission in depth order: tile counts (gathering each Gaussian's rect
// once into srect, and zeroing the tile ranges), scan, then keys (uint16_t if
// key16 else uint32_t) + values.
hipError_t launch_emit(const uint64_t* items0, const uint64_t* items1, const uint32_t* dstats, uint32_t n,
                       const uint64_t* rect, int groups, unsigned long long* wg_scratch, Stats* stats,
                       Stats* host_mapped_stats, uint32_t pair_capacity, int tiles_x, int tiles_y, void* keys,
                       bool key16, uint32_t* vals, uint2* ranges, hipStream_t s, uint32_t* fstatus = nullptr);
// One stable key-value LSD pass of the tile sort; keys_out == nullptr marks the
// final pass (values only, tile ranges recorded).
hipError_t launch_kv_pass(const void* keys_in, const uint32_t* vals_in, void* keys_out, uint32_t* vals_out,
                          bool key16, const uint32_t* n_dev, int shift, int bits, int groups, int items,
                          uint32_t* hist, uint32_t* totals, uint2* ranges, hipStream_t s);
// One wave per 8x8 block (k_blend_w).  consumed: optional device counters
// (diagnostics: 16 counters, then a u64 take map entry per pixel), or with stamps the
// per-wave timeline (tools/blend_timeline.py).  band_tiles > 0: bands of that many
// tiles dealt round-robin to the XCDs; 0: one contiguous run of blocks per XCD.
// blend_exp (GSR_TUNE_BLEND_EXP): 0 gsr_blend_expf; 1 hardware exp with exact alpha tests
// and guarded transmittance tests, blocks it cannot vouch for blended again exactly;
// 2 the same with the guard band at 100 % (test hook for the exact re-blend).
hipError_t launch_blend(const uint32_t* idx, const uint2* ranges, const uint4* rec, const Frame& fr,
                        float* out, unsigned long long* consumed, bool stamps, int band_tiles, int blend_exp,
                        hipStream_t s, const BlendSplit* split = nullptr);
// Stable partition of the preprocess items: visible first, culled last (both in
// index order), visible count into *n_live; culled tail to out only, with dead
// rects in srect (gsr_kernels.hip "live partition").  counts: groups words.
// Depth split, phase B: summed-area table of the tiles phase A left unsaturated
// ((tiles_y + 1) x (tiles_x + 1) words), gated.
hipError_t launch_split_sat(const uint8_t* bflag, int tiles_x, int tiles_y, uint32_t* sat, const uint32_t* gate,
                            hipStream_t s);
hipError_t launch_partition(const uint64_t* in, uint32_t n, int groups, uint32_t* counts, uint32_t* n_live,
                            uint64_t* out, const uint32_t* rect, uint32_t* pay0, uint32_t* pay1, hipStream_t s);
// Tile binning (row pass + column pass, tile grids <= 256 x 256): replaces
// launch_emit + the key-value tile sort.  hist: 512 x groups; row_items /
// row_pairs: 256 each; cbins: 256 x bin_col_chunks_max(); rows_buf: pair
// capacity 8-B row items; vals/ranges as the tile sort's final pass.
hipError_t launch_bin_rows(const uint64_t* items0, const uint64_t* items1, const uint32_t* dstats, uint32_t n,
                           const uint32_t* pay0, const uint32_t* pay1, int groups, uint32_t* hist,
                           uint32_t* row_items,
                           unsigned long long* row_pairs, uint32_t pair_capacity, int tiles_y, uint64_t* rows_buf,
                           int items, hipStream_t s, const uint16_t* spans = nullptr, bool rank_atomic = false,
                           uint32_t base = 0, uint32_t* gate = nullptr, int gate_mode = 0,
                           const uint32_t* cut = nullptr, const RowSplit* rs = nullptr,
                           const uint32_t* cstart = nullptr);
hipError_t launch_bin_cols(const uint64_t* rows_buf, const uint32_t* row_items, const unsigned long long* row_pairs,
                           uint32_t* cbins, int col_groups, uint32_t pair_capacity, int tiles_x, int tiles_y,
                           uint32_t* vals, uint2* ranges, Stats* stats, Stats* host_mapped_stats, int items,
                           hipStream_t s, const uint32_t* dstats = nullptr, int passes_launched = 4,
                           bool rank_atomic = false, const uint32_t* gate = nullptr, uint32_t* fstatus = nullptr,
                           int chunk = 2048);   // row items per column-pass chunk: 1024 or 2048
uint32_t bin_col_chunks_max(uint32_t pair_capacity, int tiles_y);
// Standalone sort ABI helpers (oneSweepSort / oneSweep3DGaussianSort).
hipError_t launch_items_from_keys(const int* keys, uint32_t n, uint64_t* items, hipStream_t s);
hipError_t launch_keys_from_items(const uint64_t* items, uint32_t n, int* keys, hipStream_t s);
hipError_t launch_items_from_lwg(const gsr_lwg* rec, const uint64_t* src_perm, uint32_t n, int shift,
                                 uint32_t mask, uint64_t* items, hipStream_t s);
hipError_t launch_gather_lwg(const gsr_lwg* in, const uint64_t* stage1, const uint64_t* stage2, uint32_t n,
                             gsr_lwg* out, hipStream_t s);

// Device self-check of the lane order of same-address returning LDS atomics (the
// RA rank path): runs k_rank_order_check synchronously on the current device and
// returns the lane-operations checked and how many returned a value out of lane order.
hipError_t rank_order_check(unsigned long long* lane_ops, unsigned long long* mismatches);

// Device math probe for the detmath GPU parity test.
hipError_t launch_math_probe(const float* in, int n, float* out, hipStream_t s);
hipError_t launch_exp_probe(uint32_t key_lo, uint32_t key_hi, float x_big, unsigned long long* viol, uint32_t* errs,
                            hipStream_t s);
hipError_t launch_xs_probe(const float* op, int n, float* out, hipStream_t s);

// Drop-in frame into a device image on the drop-in context (gsr_runtime.cpp);
// callers hold dropin_mutex().  `what` names the failing step for the message.
int dropin_render_device(gsr_gaussian* d_gaussians, int num_gaussians, const gsr_camera& cam, int num_tile_y,
                         int num_tile_x, int width_stride, int height_stride, int W, int H, float k,
                         float* d_out, const char** what);
std::mutex& dropin_mutex();
const char* last_error();

}  // namespace gsr
