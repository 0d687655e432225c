/*
 * oracle/out_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's output step
 * after the bake, used to check the HIP kernel (csrc/fmgi_output.hip):
 *   normalisation   main.c:66-79 (photon modes only): level-0 texels *= 0.35 * tiles / (area * spa)
 *   tone map        rectangle.c:263-286 convert/convert2, :288-293 clamp, :295-321 saveAs_core
 *   floor tint      rectangle.c:313-330 (G *= 0.95, B *= 0.9 on floor walls; again with tintExtra)
 * Pinned against the reference's own saveAs() (tests/golden/output_ref.json via oracle/_ref/out_ref).
 * Arithmetic follows the C source's types: the luminance weights and exp() are double, the rest
 * float; byte conversions truncate (a NaN becomes 0, as x86's cvttss2si low byte does).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    float pos[4], width[4], height[4], n[4];
    int32_t lm[4];
} out_rect;

static float o_len3(const float *v) { return sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

static uint8_t o_byte(float d) {
    if (d != d) return 0;
    if (d < 0) d = 0;
    if (d > 255) d = 255;
    return (uint8_t)(int)d;
}

/* texels: float4 x num_texels, modified in place (normalisation); rgb: concatenated per-wall tiles */
void out_oracle(const void *walls_v, int nwalls, float *texels, int spa, int tint_extra, uint8_t *rgb) {
    const out_rect *walls = (const out_rect *)walls_v;
    if (spa > 0) {
        for (int i = 0; i < nwalls; i++) {
            const out_rect *w = &walls[i];
            const int tiles = w->lm[1] * w->lm[2];
            const float area = o_len3(w->width) * o_len3(w->height);
            const float per = tiles / (area * spa);
            const float f = (float)(0.35 * per);
            for (int j = 0; j < tiles; j++) {
                float *t = texels + 4 * (size_t)(w->lm[0] + j);
                t[0] = t[0] * f;
                t[1] = t[1] * f;
                t[2] = t[2] * f;
                t[3] = 0;
            }
        }
    }
    size_t at = 0;
    for (int i = 0; i < nwalls; i++) {
        const out_rect *w = &walls[i];
        const int tiles = w->lm[1] * w->lm[2];
        const int floor = w->pos[2] == 0 && w->width[2] == 0 && w->height[2] == 0;
        for (int j = 0; j < tiles; j++) {
            const float *t = texels + 4 * (size_t)(w->lm[0] + j);
            float r = t[0], g = t[1], b = t[2];
            const float lum = 0.2126 * r + 0.7152 * g + 0.0722 * b;
            const float per = 1 - exp(-2 * lum);
            r *= per / lum;
            g *= per / lum;
            b *= per / lum;
            uint8_t *px = rgb + at + 3 * (size_t)j;
            px[0] = o_byte(r * 255);
            px[1] = o_byte(g * 255);
            px[2] = o_byte(b * 255);
            if (floor) {
                px[1] = (uint8_t)(int)(px[1] * 0.95);
                px[2] = (uint8_t)(int)(px[2] * 0.9);
                if (tint_extra) {
                    px[0] = (uint8_t)(int)(px[0] * 1.0f);
                    px[1] = (uint8_t)(int)(px[1] * 0.95f);
                    px[2] = (uint8_t)(int)(px[2] * 0.9f);
                }
            }
        }
        at += 3 * (size_t)tiles;
    }
}
