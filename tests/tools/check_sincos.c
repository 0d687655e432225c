/* Exhaustive check of fmgi_sincosf against glibc (float)sin((double)x) / (float)cos((double)x)
   over every phi = 6.283184f * rand() reachable by photonmap.cl:33/57 (rand = (float)s * 2^-32,
   photonmap.cl:21-25). Test infrastructure (tests/test_math.py). Prints: <checked> <mismatches>. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include "fmgi_math.h"

static float bits2f(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }

int main(int argc, char **argv) {
    uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 1;
    long long checked = 0, bad = 0;
    /* every float r in [0, 1] with r * 2^32 an integer == every value (float)s * 2^-32 can take */
#pragma omp parallel for reduction(+:checked,bad) schedule(dynamic, 65536)
    for (long long b = 0; b <= 0x3f800000LL; b += stride) {
        float r = bits2f((uint32_t)b);
        double sc = ldexp((double)r, 32);
        if (sc != floor(sc)) continue;
        float phi = 6.283184f * r;
        float s, c;
        fmgi_sincosf(phi, &s, &c);
        float gs = (float)sin((double)phi), gc = (float)cos((double)phi);
        checked++;
        if (memcmp(&s, &gs, 4) || memcmp(&c, &gc, 4)) {
            bad++;
            if (bad < 20) printf("mismatch phi=%.9g (0x%08x): mine %a %a glibc %a %a\n", phi,
                                 *(uint32_t *)&phi, s, c, gs, gc);
        }
    }
    printf("%lld %lld\n", checked, bad);
    return 0;
}
