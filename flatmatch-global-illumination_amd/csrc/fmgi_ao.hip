/*
 * fmgi_ao.hip -- ambient occlusion on the GPU, bit-identical to the reference's
 * performAmbientOcclusionNative (photonmap.c:435-490).
 *
 * One workgroup per level-0 texel, one lane per direction (481 geoSphere4 directions):
 *   - the lane builds its ray exactly as performAmbientOcclusionNativeOnWall does (:451-455);
 *   - it replays findClosestIntersection (:54-161) on the host-built BSP with an explicit stack;
 *   - it stores `dist * fac` (dist = 10 when nothing is hit, :458-462) to LDS.
 * Lane 0 then adds the terms in direction order, the reference's sequential fp32 sum, and applies
 * `distSum /= (facSum*1.5)` with the double promotion the C source implies (:468).
 *
 * Arithmetic: the native C path (rectangle.c, vector3_cl.c; gcc -O2 -msse3, no FMA) is IEEE fp32 in
 * source order. Contraction is off here, and every operation is written in the reference's order.
 */
#include <hip/hip_runtime.h>

#include "fmgi_ao.h"

#pragma clang fp contract(off)

#include "fmgi_rect_dev.h"

namespace {

using namespace fmgi_dev;

/* One stack frame of findClosestIntersection (photonmap.c:54-161). stage 0: test the node's items;
   stage 1: the nearer child (the side of the split plane the ray starts on) has returned `ret`;
   stage 2: the farther child, entered at its plane crossing with the distance shift, has returned. */
struct Frame {
    int node;
    float px, py, pz, shift;
    int hit, child_hit, stage;
};

__device__ int ao_find(const AoArgs &a, v3 pos0, v3 dir, float &dist) {
    Frame st[FMGI_AO_MAX_DEPTH];
    int sp = 0;
    st[0] = Frame{0, pos0.x, pos0.y, pos0.z, 0.0f, 0, 0, 0};
    int ret = 0;
    for (;;) {
        Frame &f = st[sp];
        const AoNode nd = a.nodes[f.node];
        const v3 pos = mk(f.px, f.py, f.pz);
        const v3 ppos = mk(nd.px, nd.py, nd.pz), pn = mk(nd.nx, nd.ny, nd.nz);
        if (f.stage == 0) {
            for (int i = 0; i < nd.nitems; i++) { /* :70-82 */
                const float dn = rect_intersects(a.items[nd.item0 + i], pos, dir, dist);
                if (dn == -1) continue;
                if (dn + f.shift < dist) {
                    dist = dn + f.shift;
                    f.hit = 1;
                }
            }
            if (nd.left < 0 && nd.right < 0) { /* :93-94 leaf */
                ret = f.hit;
                if (sp-- == 0) return ret;
                continue;
            }
            f.stage = 1;
            const int near = dot(sub(pos, ppos), pn) < 0 ? nd.left : nd.right; /* :106-108 */
            if (near >= 0) {
                st[sp + 1] = Frame{near, f.px, f.py, f.pz, f.shift, 0, 0, 0};
                sp++;
                continue;
            }
            ret = 0;
        }
        if (f.stage == 1) {
            f.child_hit = ret;
            f.stage = 2;
            const bool left_side = dot(sub(pos, ppos), pn) < 0;
            const int far = left_side ? nd.right : nd.left;
            v3 sn = pn; /* :98-101: the split normal facing the ray source */
            if (dot(sub(pos, ppos), sn) < 0) sn = mk(-sn.x, -sn.y, -sn.z);
            const bool faces_away = dot(sn, dir) >= 0;
            if (!f.child_hit && far >= 0 && !faces_away) { /* :121-129 / :142-149 */
                const float denom = dot(pn, dir); /* distanceOfIntersectionWithPlane rectangle.c:115 */
                float pd = -1;
                if (denom != 0) {
                    pd = dot(pn, sub(ppos, pos)) / denom;
                    if (pd < 0) pd = -1;
                }
                if (pd < 0) pd = 0;
                const v3 np = add(pos, mul(dir, pd));
                st[sp + 1] = Frame{far, np.x, np.y, np.z, f.shift + pd, 0, 0, 0};
                sp++;
                continue;
            }
            ret = 0;
        }
        /* stage 2 */
        f.hit |= ret;
        f.hit |= f.child_hit;
        ret = f.hit;
        if (sp-- == 0) return ret;
    }
}

__global__ __launch_bounds__(512) void k_ao(AoArgs a) {
    __shared__ float term[FMGI_AO_DIRS_MAX];
    const int64_t job = blockIdx.x;
    const AoWall w = a.walls[a.jobs[job]];
    const int tile = a.job_tile[job];
    const int k = threadIdx.x;
    if (k < a.ndirs) {
        const v3 g = mk(a.dirs[3 * k], a.dirs[3 * k + 1], a.dirs[3 * k + 2]);
        const float fac = g.z;
        /* transformToOrthoNormalBase (photonmap.c:29-44) with b0 = c1, b1 = c2, b2 = n */
        const v3 dir = mk(g.x * w.b1x + g.y * w.b2x + g.z * w.nx, g.x * w.b1y + g.y * w.b2y + g.z * w.ny,
                          g.x * w.b1z + g.y * w.b2z + g.z * w.nz);
        /* getTileCenter (rectangle.c:140-153): pos + vWidth*(tx+0.5) + vHeight*(ty+0.5) */
        const int tx = tile % w.s1, ty = tile / w.s1;
        const v3 c = add(add(mk(w.px, w.py, w.pz), mul(mk(w.vwx, w.vwy, w.vwz), (float)(tx + 0.5))),
                         mul(mk(w.vhx, w.vhy, w.vhz), (float)(ty + 0.5)));
        const v3 pos = add(c, mul(dir, 1E-5f));
        float dist = INFINITY;
        const int hit = ao_find(a, pos, dir, dist);
        if (!hit) dist = 10;
        term[k] = dist * fac;
    }
    __syncthreads();
    if (k == 0) {
        float s = 0;
        for (int i = 0; i < a.ndirs; i++) s += term[i];
        s = (float)((double)s / ((double)a.fac_sum * 1.5));
        float4 *t = (float4 *)a.texels + w.s0 + tile;
        *t = make_float4(s, s, s, 0.0f);
    }
}

} // namespace

hipError_t fmgi_launch_ao(const AoArgs &a, hipStream_t s) {
    if (a.njobs <= 0) return hipSuccess;
    if (a.ndirs > FMGI_AO_DIRS_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ao, dim3((unsigned)a.njobs), dim3(512), 0, s, a);
    return hipGetLastError();
}
