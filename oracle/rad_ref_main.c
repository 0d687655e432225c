/*
 * oracle/rad_ref_main.c -- TEST INFRASTRUCTURE ONLY. A driver, linked by oracle/build_ref.sh against the
 * REFERENCE's own radiosityNative.o / rectangle.o / vector3_cl.o (compiled in place from
 * /root/reference), that seeds libc rand(), runs the reference's performRadiosityNative
 * (radiosityNative.c:92-268) on a FMGIGEO1 geometry fixture, and writes the resulting texels
 * (float4 x numTexels) followed by the next rand() value (int32: where the reference leaves the
 * libc stream). tests/golden/make_rad_fixtures.py records its output.
 *
 *   rad_ref <geometry.bin> <texels_out.bin> <seed>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "geometry.h"
#include "radiosityNative.h"

int main(int argc, char **argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s geometry.bin texels_out.bin seed\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 3;
    char magic[8];
    int hdr[4];
    if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "FMGIGEO1", 8) || fread(hdr, sizeof hdr, 1, f) != 1) return 4;
    Geometry geo;
    memset(&geo, 0, sizeof geo);
    geo.numWindows = hdr[0];
    geo.numLights = hdr[1];
    geo.numWalls = hdr[2];
    geo.numTexels = hdr[3];
    size_t n = (size_t)hdr[0] + hdr[1] + hdr[2];
    Rectangle *all = NULL;
    if (posix_memalign((void **)&all, 16, (n ? n : 1) * sizeof(Rectangle))) return 5;
    if (fread(all, sizeof(Rectangle), n, f) != n) return 6;
    fclose(f);
    geo.windows = all;
    geo.lights = all + hdr[0];
    geo.walls = all + hdr[0] + hdr[1];
    if (posix_memalign((void **)&geo.texels, 16, (size_t)(geo.numTexels ? geo.numTexels : 1) * sizeof(Vector3))) return 7;
    memset(geo.texels, 0, (size_t)geo.numTexels * sizeof(Vector3));
    srand((unsigned)atoi(argv[3]));
    performRadiosityNative(&geo);
    int next = rand();
    FILE *o = fopen(argv[2], "wb");
    if (!o || fwrite(geo.texels, sizeof(Vector3), (size_t)geo.numTexels, o) != (size_t)geo.numTexels) return 8;
    if (fwrite(&next, sizeof next, 1, o) != 1) return 9;
    fclose(o);
    return 0;
}
