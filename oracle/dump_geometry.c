/*
 * dump_geometry.c -- fixture generator (TEST INFRASTRUCTURE ONLY).
 *
 * Links against the reference's own layout parser (parseLayout.c:359 `parseLayout`,
 * image.c:210 `loadImage`), compiled from /root/reference by oracle/build_ref.sh, and writes
 * the resulting Geometry (geometry.h:7-15) as a flat binary fixture:
 *
 *   char magic[8] = "FMGIGEO1"
 *   int32 numWindows, numLights, numWalls, numTexels
 *   Rectangle windows[numWindows], lights[numLights], walls[numWalls]   (80 B each)
 *
 * Usage: dump_geometry <layout.png> <scale px/m> <out.bin>   (TILE_SIZE = 200 as in main.c:44)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parseLayout.h"
#include "geometry.h"
#include "image.h"

int main(int argc, char **argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s <layout.png> <scale> <out.bin>\n", argv[0]);
        return 2;
    }
    float scale = (float)atof(argv[2]);
    Image *img = loadImage(argv[1]);
    const float TILE_SIZE = 200;
    Geometry *geo = parseLayout(img, 1 / scale, TILE_SIZE);
    freeImage(img);
    FILE *f = fopen(argv[3], "wb");
    if (!f) return 1;
    fwrite("FMGIGEO1", 1, 8, f);
    int32_t hdr[4] = {geo->numWindows, geo->numLights, geo->numWalls, geo->numTexels};
    fwrite(hdr, sizeof hdr, 1, f);
    fwrite(geo->windows, sizeof(Rectangle), (size_t)geo->numWindows, f);
    fwrite(geo->lights, sizeof(Rectangle), (size_t)geo->numLights, f);
    fwrite(geo->walls, sizeof(Rectangle), (size_t)geo->numWalls, f);
    fclose(f);
    printf("windows=%d lights=%d walls=%d texels=%d sizeof(Rectangle)=%zu sizeof(Geometry)=%zu\n",
           geo->numWindows, geo->numLights, geo->numWalls, geo->numTexels, sizeof(Rectangle),
           sizeof(Geometry));
    freeGeometry(geo);
    return 0;
}
