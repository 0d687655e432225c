/*
 * oracle/out_ref_main.c -- TEST INFRASTRUCTURE ONLY. Linked by oracle/build_ref.sh against the
 * REFERENCE's rectangle.o / png_helper.o / vector3_cl.o (compiled in place from /root/reference).
 * Applies main.c:66-79's photon-mode normalisation (restated below, 4 lines) and then the reference's
 * own saveAs() (rectangle.c:338-345) to every wall, reads each PNG back with the reference's
 * read_png_file(), and writes the concatenated RGB8 tile bytes and the normalised texels.
 *
 *   out_ref <geometry.bin> <texels.bin> <spa, 0 = no normalisation> <tintExtra> <tmpdir> <rgb_out> <texels_out>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "geometry.h"
#include "png_helper.h"
#include "rectangle.h"

int main(int argc, char **argv) {
    if (argc != 8) return 2;
    FILE *f = fopen(argv[1], "rb");
    char magic[8];
    int hdr[4];
    if (!f || fread(magic, 1, 8, f) != 8 || memcmp(magic, "FMGIGEO1", 8) || fread(hdr, sizeof hdr, 1, f) != 1) return 3;
    size_t n = (size_t)hdr[0] + hdr[1] + hdr[2];
    Rectangle *all = NULL;
    if (posix_memalign((void **)&all, 16, (n ? n : 1) * sizeof(Rectangle)) || fread(all, sizeof(Rectangle), n, f) != n) return 4;
    fclose(f);
    Rectangle *walls = all + hdr[0] + hdr[1];
    const int nwalls = hdr[2], ntex = hdr[3];
    Vector3 *tex = NULL;
    if (posix_memalign((void **)&tex, 16, (size_t)(ntex ? ntex : 1) * sizeof(Vector3))) return 5;
    f = fopen(argv[2], "rb");
    if (!f || fread(tex, sizeof(Vector3), (size_t)ntex, f) != (size_t)ntex) return 6;
    fclose(f);
    const int spa = atoi(argv[3]), tint = atoi(argv[4]);
    if (spa > 0) { /* main.c:66-79 */
        for (int i = 0; i < nwalls; i++) {
            Rectangle *obj = &walls[i];
            float tilesPerSample = getNumTiles(obj) / (getArea(obj) * spa);
            int baseIdx = obj->lightmapSetup.s[0];
            for (int j = 0; j < getNumTiles(obj); j++) tex[baseIdx + j] = mul(tex[baseIdx + j], 0.35 * tilesPerSample);
        }
    }
    FILE *o = fopen(argv[6], "wb");
    if (!o) return 7;
    char path[4096];
    for (int i = 0; i < nwalls; i++) {
        snprintf(path, sizeof path, "%s/tile_%d.png", argv[5], i);
        saveAs(&walls[i], path, tex, tint);
        int w = 0, h = 0, ct = 0;
        uint8_t *px = NULL;
        read_png_file(path, &w, &h, &ct, &px);
        if (w != walls[i].lightmapSetup.s[1] || h != walls[i].lightmapSetup.s[2]) return 8;
        fwrite(px, 3, (size_t)w * h, o);
        free(px);
    }
    fclose(o);
    o = fopen(argv[7], "wb");
    if (!o || fwrite(tex, sizeof(Vector3), (size_t)ntex, o) != (size_t)ntex) return 9;
    fclose(o);
    return 0;
}
