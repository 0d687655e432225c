/*
 * oracle/photon_ref_main.c -- TEST INFRASTRUCTURE ONLY (bench.py's CPU baseline). A driver, linked by
 * oracle/build_ref.sh against the REFERENCE's own photonmap.o / rectangle.o / vector3_cl.o (compiled in
 * place from /root/reference), that times the reference's CPU photon mapper
 * performPhotonMappingNative (photonmap.c:408-435: one photon per sample, numSamplesPerArea x area per
 * emitter, BSP-tree scan, one core) on a FMGIGEO1 geometry fixture. The reference's progress lines go
 * to stdout; the last line is a JSON record {photons, seconds}.
 *
 *   photon_ref <geometry.bin> <numSamplesPerArea>
 */
#define _POSIX_C_SOURCE 199309L /* clock_gettime under -std=c99 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "geometry.h"
#include "global_illumination_native.h"
#include "rectangle.h"

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s geometry.bin numSamplesPerArea\n", argv[0]);
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
    const int spa = atoi(argv[2]);
    uint64_t photons = 0; /* photonmap.c:416-418 / 427-429: the same per-emitter sample counts */
    for (int i = 0; i < geo.numWindows + geo.numLights; i++) {
        const Rectangle *r = i < geo.numWindows ? &geo.windows[i] : &geo.lights[i - geo.numWindows];
        Vector3 xDir = getWidthVector(r), yDir = getHeightVector(r);
        float area = length(xDir) * length(yDir);
        photons += (uint64_t)(spa * area);
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    performPhotonMappingNative(&geo, spa);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    printf("\n{\"photons\": %llu, \"seconds\": %.6f}\n", (unsigned long long)photons, s);
    return 0;
}
