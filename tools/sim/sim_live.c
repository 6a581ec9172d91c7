/* sim_live.c — analysis tool (not product, not test): how many of the blend's
 * pair-iterations run with few live pixels.  Replays the shipped schedule (one wave
 * per 8x8 block, 64-record batches, survivors of the ideal per-block cull, two
 * splats per iteration, render.cu:323-341 compositing and early termination) and
 * histograms, per pair-iteration, the pixels still live (T >= 1e-3) at its start.
 * A schedule that packs the live pixels of both splats of a pair into one wave64
 * evaluation when at most 32 are live would price those iterations lower.
 * build: gcc -O2 -fopenmp -shared -fPIC -o sim_live.so sim_live.c -lm */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    float cx, cy, a, b, c, e, op;
    int x0, y0, x1, y1;
} Sp;

static inline float alpha_at(const Sp* s, int px, int py) {
    const float dx = (float)px - s->cx, dy = (float)py - s->cy;
    const float md = dx * (s->a * dx + s->b * dy) + dy * (s->c * dx + s->e * dy);
    float al = s->op * expf(-0.5f * md);
    return fminf(al, 0.99f);
}

static inline void load(const float* r, Sp* s) {
    s->cx = r[0]; s->cy = r[1]; s->a = r[2]; s->b = r[3]; s->c = r[4]; s->e = r[5]; s->op = r[6];
    s->x0 = (int)r[7]; s->y0 = (int)r[8]; s->x1 = (int)r[9]; s->y1 = (int)r[10];
}

/* hist[L] (L = 0..64): pair-iterations that start with L live pixels; out[0] = pair
 * iterations, out[1] = batches, out[2] = blocks that ever reach <= 32 live pixels,
 * out[3] = in-box live lanes over all iterations (both splats) */
void sim_live(const float* rec, const int* lists, const int* offs, int nblocks, const int* bxy, double* hist,
              double* out) {
    double pit = 0, batches = 0, compact_blocks = 0, active = 0;
    double h[65];
    memset(h, 0, sizeof h);
#pragma omp parallel
    {
        double hl[65];
        memset(hl, 0, sizeof hl);
#pragma omp for schedule(dynamic, 64) reduction(+ : pit, batches, compact_blocks, active)
        for (int blk = 0; blk < nblocks; blk++) {
            const int bx = bxy[2 * blk], by = bxy[2 * blk + 1];
            float T[64];
            for (int l = 0; l < 64; l++) T[l] = 1.0f;
            const int beg = offs[2 * blk], end = offs[2 * blk + 1];
            int alive = 1, went_compact = 0;
            for (int base = beg; base < end && alive; base += 64) {
                const int cnt = end - base < 64 ? end - base : 64;
                batches += 1;
                int surv[64], ns = 0;
                for (int k = 0; k < cnt; k++) {
                    Sp s;
                    load(rec + 11 * (size_t)lists[base + k], &s);
                    int ok = 0;
                    for (int l = 0; l < 64 && !ok; l++) {
                        const int px = bx + (l & 7), py = by + (l >> 3);
                        if (px < s.x0 || px > s.x1 || py < s.y0 || py > s.y1 || T[l] < 1e-3f) continue;
                        if (alpha_at(&s, px, py) >= 1e-3f) ok = 1;
                    }
                    if (ok) surv[ns++] = lists[base + k];
                }
                for (int j = 0; j < ns && alive; j += 2) {
                    int live = 0;
                    for (int l = 0; l < 64; l++) live += !(T[l] < 1e-3f);
                    hl[live] += 1;
                    pit += 1;
                    if (live <= 32) went_compact = 1;
                    for (int q = j; q < j + 2 && q < ns; q++) {
                        Sp s;
                        load(rec + 11 * (size_t)surv[q], &s);
                        for (int l = 0; l < 64; l++) {
                            const int px = bx + (l & 7), py = by + (l >> 3);
                            if (px < s.x0 || px > s.x1 || py < s.y0 || py > s.y1 || T[l] < 1e-3f) continue;
                            active += 1;
                            const float al = alpha_at(&s, px, py);
                            if (al < 1e-3f) continue;
                            T[l] = T[l] * (1.0f - al);
                        }
                    }
                    alive = 0;
                    for (int l = 0; l < 64; l++) alive |= !(T[l] < 1e-3f);
                }
            }
            compact_blocks += went_compact;
        }
#pragma omp critical
        for (int i = 0; i <= 64; i++) h[i] += hl[i];
    }
    for (int i = 0; i <= 64; i++) hist[i] = h[i];
    out[0] = pit;
    out[1] = batches;
    out[2] = compact_blocks;
    out[3] = active;
}
