/* sim_blend.c — analysis tool (not product, not test): replays the blend's
 * per-8x8-block work for several wave schedules on real splat records and counts
 * splat-slot iterations (one wave evaluation of one splat) and lanes that
 * composite.  Compositing follows render.cu:323-341 (expf, 0.99 clamp, 1e-3
 * thresholds); the cull is the ideal one (a splat survives for a pixel group iff
 * some unsaturated in-box pixel of the group reaches alpha >= 1e-3).
 *
 * Schedules (G = lane groups of a wave, each group a sub-block with its own
 * survivor list; iterations of a batch = max over groups of its pair count):
 *   G=1: 8x8 (the shipped kernel)   G=2: 8x4 halves   G=4: 4x4 quadrants
 *   G=64: one list per lane (per-pixel streams)
 * Batches of B list entries; all groups sync at batch boundaries.
 * build: gcc -O2 -fopenmp -shared -fPIC -o sim_blend.so sim_blend.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
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

/* out[0] = splat-slot iterations, out[1] = taken lanes, out[2] = in-box live lanes,
 * out[3] = records loaded (batches * entries), out[4] = batches */
void sim(const float* rec /* n x 11 */, const int* lists, const int* offs, int nblocks, const int* bxy,
         int G, int B, int pairs, int cullmode, double* out) {
    double it = 0, taken = 0, active = 0, loaded = 0, batches = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : it, taken, active, loaded, batches)
    for (int blk = 0; blk < nblocks; blk++) {
        const int bx = bxy[2 * blk], by = bxy[2 * blk + 1];
        float T[64];
        for (int l = 0; l < 64; l++) T[l] = 1.0f;
        const int beg = offs[2 * blk], end = offs[2 * blk + 1];
        int alive = 1;
        for (int base = beg; base < end && alive; base += B) {
            const int cnt = end - base < B ? end - base : B;
            loaded += cnt;
            batches += 1;
            /* per-group survivor lists (lane group g covers lanes with grp(l) == g) */
            int surv[64][256];
            int ns[64];
            for (int g = 0; g < G; g++) ns[g] = 0;
            for (int k = 0; k < cnt; k++) {
                Sp s;
                const float* r = rec + 11 * (size_t)lists[base + k];
                s.cx = r[0]; s.cy = r[1]; s.a = r[2]; s.b = r[3]; s.c = r[4]; s.e = r[5]; s.op = r[6];
                s.x0 = (int)r[7]; s.y0 = (int)r[8]; s.x1 = (int)r[9]; s.y1 = (int)r[10];
                unsigned long long gmask = 0;
                int block_ok = 0;
                for (int l = 0; l < 64 && cullmode == 1; l++) {
                    const int px = bx + (l & 7), py = by + (l >> 3);
                    if (px < s.x0 || px > s.x1 || py < s.y0 || py > s.y1 || T[l] < 1e-3f) continue;
                    if (alpha_at(&s, px, py) >= 1e-3f) block_ok = 1;
                }
                for (int l = 0; l < 64 && cullmode == 2; l++) {
                    const int px = bx + (l & 7), py = by + (l >> 3);
                    if (px < s.x0 || px > s.x1 || py < s.y0 || py > s.y1 || T[l] < 1e-3f) continue;
                    if (alpha_at(&s, px, py) >= 1e-3f) block_ok = 1;
                }
                /* octagon: |u| <= U, |v| <= V around the centre, at the alpha cutoff */
                const double h = 0.5 * ((double)s.b + s.c), det = (double)s.a * s.e - h * h;
                const double cut = 2.0 * log(1000.0 * s.op);
                const double U = det > 0 ? sqrt(cut * (s.a - 2 * h + s.e) / det) : 1e30;
                const double V = det > 0 ? sqrt(cut * (s.a + 2 * h + s.e) / det) : 1e30;
                for (int l = 0; l < 64; l++) {
                    const int px = bx + (l & 7), py = by + (l >> 3);
                    if (px < s.x0 || px > s.x1 || py < s.y0 || py > s.y1 || T[l] < 1e-3f) continue;
                    if (cullmode == 0 && alpha_at(&s, px, py) < 1e-3f) continue;
                    if (cullmode == 1 && !block_ok) continue;
                    if (cullmode == 4) {
                        int gx0 = bx, gx1 = bx + 7, gy0 = by, gy1 = by + 7;
                        if (gx0 < s.x0) gx0 = s.x0;
                        if (gx1 > s.x1) gx1 = s.x1;
                        if (gy0 < s.y0) gy0 = s.y0;
                        if (gy1 > s.y1) gy1 = s.y1;
                        const double u0 = (gx0 - s.cx) + (gy0 - s.cy), u1 = (gx1 - s.cx) + (gy1 - s.cy);
                        const double v0 = (gx0 - s.cx) - (gy1 - s.cy), v1 = (gx1 - s.cx) - (gy0 - s.cy);
                        if (u0 > U || u1 < -U || v0 > V || v1 < -V) continue;
                    }
                    if (cullmode == 2) {
                        if (!block_ok) continue;
                        /* the pixel's group rectangle vs the octagon: test at group level by
                           testing each pixel (equivalent for the min over the rectangle) */
                        const double du = (px - s.cx) + (py - s.cy), dv = (px - s.cx) - (py - s.cy);
                        int grp_ok = 0;
                        /* group rect: expand to the group's pixel set */
                        int gx0, gx1, gy0, gy1;
                        if (G == 1) { gx0 = bx; gx1 = bx + 7; gy0 = by; gy1 = by + 7; }
                        else if (G == 2) { gx0 = bx; gx1 = bx + 7; gy0 = by + ((l >> 3) >= 4) * 4; gy1 = gy0 + 3; }
                        else if (G == 4) { gx0 = bx + ((l & 7) >= 4) * 4; gx1 = gx0 + 3; gy0 = by + ((l >> 3) >= 4) * 4; gy1 = gy0 + 3; }
                        else { gx0 = gx1 = px; gy0 = gy1 = py; }
                        if (gx0 < s.x0) gx0 = s.x0;
                        if (gx1 > s.x1) gx1 = s.x1;
                        if (gy0 < s.y0) gy0 = s.y0;
                        if (gy1 > s.y1) gy1 = s.y1;
                        const double u0 = (gx0 - s.cx) + (gy0 - s.cy), u1 = (gx1 - s.cx) + (gy1 - s.cy);
                        const double v0 = (gx0 - s.cx) - (gy1 - s.cy), v1 = (gx1 - s.cx) - (gy0 - s.cy);
                        grp_ok = !(u0 > U || u1 < -U || v0 > V || v1 < -V);
                        (void)du; (void)dv;
                        if (!grp_ok) continue;
                    }
                    int g;
                    if (G == 1) g = 0;
                    else if (G == 2) g = (l >> 3) >= 4;
                    else if (G == 4) g = ((l >> 3) >= 4) * 2 + ((l & 7) >= 4);
                    else g = l;
                    gmask |= 1ull << g;
                }
                for (int g = 0; g < G; g++)
                    if (gmask >> g & 1ull) surv[g][ns[g]++] = lists[base + k];
            }
            /* composite: iteration j evaluates entry j (pairs: entries 2j, 2j+1) of every group */
            int maxn = 0;
            for (int g = 0; g < G; g++) maxn = ns[g] > maxn ? ns[g] : maxn;
            int pos[64];
            for (int g = 0; g < G; g++) pos[g] = 0;
            const int step = pairs ? 2 : 1;
            for (int j = 0; j < maxn && alive; j += step) {
                int used = 0;
                for (int g = 0; g < G; g++) used = used > ns[g] - j ? used : ns[g] - j;
                it += used >= step ? step : used;
                for (int h = 0; h < step && j + h < maxn; h++) {
                    for (int l = 0; l < 64; l++) {
                        int g;
                        if (G == 1) g = 0;
                        else if (G == 2) g = (l >> 3) >= 4;
                        else if (G == 4) g = ((l >> 3) >= 4) * 2 + ((l & 7) >= 4);
                        else g = l;
                        if (j + h >= ns[g]) continue;
                        const float* r = rec + 11 * (size_t)surv[g][j + h];
                        Sp s;
                        s.cx = r[0]; s.cy = r[1]; s.a = r[2]; s.b = r[3]; s.c = r[4]; s.e = r[5]; s.op = r[6];
                        s.x0 = (int)r[7]; s.y0 = (int)r[8]; s.x1 = (int)r[9]; s.y1 = (int)r[10];
                        const int px = bx + (l & 7), py = by + (l >> 3);
                        if (px < s.x0 || px > s.x1 || py < s.y0 || py > s.y1 || T[l] < 1e-3f) continue;
                        active += 1;
                        const float al = alpha_at(&s, px, py);
                        if (al < 1e-3f) continue;
                        taken += 1;
                        T[l] = T[l] * (1.0f - al);
                    }
                }
                alive = 0;
                for (int l = 0; l < 64; l++) alive |= !(T[l] < 1e-3f);
            }
            (void)pos;
        }
    }
    out[0] = it;
    out[1] = taken;
    out[2] = active;
    out[3] = loaded;
    out[4] = batches;
}

/* Two pixels per lane (VERDICT r05 #3 "also price"): one wave per 8-wide x (8 * P)-tall
 * block, lane l holding pixels (l & 7, (l >> 3) + 8 p) for p < P.  The ideal per-block cull
 * (cullmode 1): a splat survives a batch iff some unsaturated in-box pixel of the block
 * reaches alpha >= 1e-3.  Batches of B entries of the tile list, pairs as the kernel.
 * blocks: bxy (top-left corners) with offs into lists.  out as sim(). */
void sim_tall(const float* rec, const int* lists, const int* offs, int nblocks, const int* bxy, int P, int B,
              double* out) {
    double it = 0, taken = 0, active = 0, loaded = 0, batches = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : it, taken, active, loaded, batches)
    for (int blk = 0; blk < nblocks; blk++) {
        const int bx = bxy[2 * blk], by = bxy[2 * blk + 1];
        const int np = 64 * P;
        float T[256];
        for (int l = 0; l < np; l++) T[l] = 1.0f;
        const int beg = offs[2 * blk], end = offs[2 * blk + 1];
        int alive = 1;
        for (int base = beg; base < end && alive; base += B) {
            const int cnt = end - base < B ? end - base : B;
            loaded += cnt;
            batches += 1;
            int surv[256], ns = 0;
            for (int k = 0; k < cnt; k++) {
                Sp s;
                const float* r = rec + 11 * (size_t)lists[base + k];
                s.cx = r[0]; s.cy = r[1]; s.a = r[2]; s.b = r[3]; s.c = r[4]; s.e = r[5]; s.op = r[6];
                s.x0 = (int)r[7]; s.y0 = (int)r[8]; s.x1 = (int)r[9]; s.y1 = (int)r[10];
                int ok = 0;
                for (int l = 0; l < np && !ok; l++) {
                    const int px = bx + (l & 7), py = by + (l >> 3);
                    if (px < s.x0 || px > s.x1 || py < s.y0 || py > s.y1 || T[l] < 1e-3f) continue;
                    if (alpha_at(&s, px, py) >= 1e-3f) ok = 1;
                }
                if (ok) surv[ns++] = lists[base + k];
            }
            for (int j = 0; j < ns && alive; j += 2) {
                it += ns - j >= 2 ? 2 : 1;
                for (int h = 0; h < 2 && j + h < ns; h++) {
                    const float* r = rec + 11 * (size_t)surv[j + h];
                    Sp s;
                    s.cx = r[0]; s.cy = r[1]; s.a = r[2]; s.b = r[3]; s.c = r[4]; s.e = r[5]; s.op = r[6];
                    s.x0 = (int)r[7]; s.y0 = (int)r[8]; s.x1 = (int)r[9]; s.y1 = (int)r[10];
                    for (int l = 0; l < np; l++) {
                        const int px = bx + (l & 7), py = by + (l >> 3);
                        if (px < s.x0 || px > s.x1 || py < s.y0 || py > s.y1 || T[l] < 1e-3f) continue;
                        active += 1;
                        const float a = alpha_at(&s, px, py);
                        if (a < 1e-3f) continue;
                        taken += 1;
                        T[l] *= 1.0f - a;
                    }
                }
                alive = 0;
                for (int l = 0; l < np; l++) alive |= !(T[l] < 1e-3f);
            }
        }
    }
    out[0] = it; out[1] = taken; out[2] = active; out[3] = loaded; out[4] = batches;
}
