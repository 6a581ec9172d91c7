/* Depth-split analysis (analysis only, not product code): for each pixel, the position
 * in the global depth order of the splat after which its transmittance falls below
 * 1e-3 (the blend stops there, render.cu:326-341), or -1 when it never does.
 * rec: m x 11 floats in depth order (px_x, px_y, inv_covar[4], opacity, aabb[4]),
 * as tools/sim/sim_blend.py builds them.
 * gcc -O2 -ffp-contract=off -fopenmp -shared -fPIC -I../../include depth_split.c -o depth_split.so -lm */
#include <stdint.h>
#include <stdlib.h>
#include "gsr_detmath.h"

void sat_pos(const float* rec, int64_t m, int W, int H, int32_t* out) {
    const int band = 8, nbands = (H + band - 1) / band;
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < nbands; b++) {
        const int y0 = b * band, y1 = (y0 + band < H ? y0 + band : H) - 1;
        float* T = (float*)malloc(sizeof(float) * band * W);
        for (int q = 0; q < band * W; q++) T[q] = 1.0f;
        for (int y = y0; y <= y1; y++)
            for (int x = 0; x < W; x++) out[(size_t)y * W + x] = -1;
        for (int64_t s = 0; s < m; s++) {
            const float* r = rec + 11 * s;
            const int ax0 = (int)r[7], ay0 = (int)r[8], ax1 = (int)r[9], ay1 = (int)r[10];
            if (ay1 < y0 || ay0 > y1) continue;
            const int ya = ay0 > y0 ? ay0 : y0, yb = ay1 < y1 ? ay1 : y1;
            const int xa = ax0 > 0 ? ax0 : 0, xb = ax1 < W - 1 ? ax1 : W - 1;
            for (int y = ya; y <= yb; y++)
                for (int x = xa; x <= xb; x++) {
                    float* t = &T[(y - y0) * W + x];
                    if (*t < 1e-3f) continue;
                    const float md2 = gsr_blend_md2((float)x - r[0], (float)y - r[1], r[2], r[3], r[4], r[5]);
                    float a = r[6] * gsr_blend_expf(-0.5f * md2);
                    a = a < 0.99f ? a : 0.99f;
                    if (a < 1e-3f) continue;
                    *t *= (1.0f - a);
                    if (*t < 1e-3f) out[(size_t)y * W + x] = (int32_t)s;
                }
        }
        free(T);
    }
}
