/*
 * fmgi_geosphere.h -- the ambient-occlusion direction table (the reference's geoSphere4, geoSphere.h:21),
 * regenerated instead of stored.
 *
 * The reference table is the output of its generator script geoSphere.py: the 4 upper faces of an
 * octahedron, each subdivided `levels` times by normalised edge midpoints, every vertex kept once in a
 * Python dict, z == 0 vertices dropped, printed in dict iteration order. The AO sum
 * (photonmap.c:448-465) runs over the table in that order, so the order is part of the result.
 *
 * The order is that of a CPython dict before 3.6: open addressing over the tuple hashes. This file
 * replays that dict:
 *   - float hash: _Py_HashDouble, the 3.x numeric hash modulo 2^61 - 1;
 *   - tuple hash: the pre-3.8 multiply/xor loop;
 *   - probing: i = 5i + perturb + 1, perturb >>= 5;
 *   - growth: used*2 + size/2 when the usable slots run out; a resize reinserts in slot order.
 * The vertex arithmetic is plain IEEE double: a midpoint (a + b) / 2, then v / sqrt(x*x + y*y + z*z).
 * The squares are correctly rounded products; the script's x**2 gave exactly that on the machine
 * that produced the reference table.
 *
 * oracle/geosphere_check.py checked every entry against the reference's geoSphere.c in this
 * container: identical for levels 3, 4 and 5, values and order. tests/test_ao.py pins this
 * generator to the SHA-256 of the float32 table.
 */
#ifndef FMGI_GEOSPHERE_H
#define FMGI_GEOSPHERE_H

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace fmgi_geo {

struct V3 {
    double x, y, z;
};

inline bool same(const V3 &a, const V3 &b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

/* CPython 3.x hash of a float (Objects/object.c _Py_HashDouble); the tuple (0, 0, 1) of the script
   holds ints, whose hashes equal those of the equal floats */
inline int64_t py_hash_double(double v) {
    const uint64_t M = (1ull << 61) - 1;
    if (std::isinf(v)) return v > 0 ? 314159 : -314159;
    if (std::isnan(v)) return 0;
    int e;
    double m = std::frexp(v, &e);
    int sign = 1;
    if (m < 0) {
        sign = -1;
        m = -m;
    }
    uint64_t x = 0;
    while (m != 0.0) {
        x = ((x << 28) & M) | x >> (61 - 28);
        m *= 268435456.0;
        e -= 28;
        const uint64_t y = (uint64_t)m;
        m -= (double)y;
        x += y;
        if (x >= M) x -= M;
    }
    e = e >= 0 ? e % 61 : 61 - 1 - ((-1 - e) % 61);
    x = ((x << e) & M) | x >> (61 - e);
    int64_t h = (int64_t)x * sign;
    return h == -1 ? -2 : h;
}

/* CPython < 3.8 tuple hash of a 3-tuple */
inline uint64_t py_hash_tuple3(const V3 &v) {
    const double c[3] = {v.x, v.y, v.z};
    uint64_t x = 0x345678ull, mult = 1000003ull;
    for (int i = 0; i < 3; i++) {
        const uint64_t y = (uint64_t)py_hash_double(c[i]);
        x = (x ^ y) * mult;
        mult += 82520ull + 2ull * (uint64_t)(3 - 1 - i);
    }
    x += 97531ull;
    if ((int64_t)x == -1) x = (uint64_t)-2;
    return x;
}

/* insertion-only CPython < 3.6 dict of V3 keys */
class PyDict {
  public:
    PyDict() : slots_(8), used_(8, false), usable_((2 * 8 + 1) / 3) {}

    void insert(const V3 &k) {
        const uint64_t h = py_hash_tuple3(k);
        if (find(k, h)) return;
        if (usable_ <= 0) resize(count_ * 2 + slots_.size() / 2);
        place(k, h);
        count_++;
        usable_--;
    }

    std::vector<V3> keys() const {
        std::vector<V3> out;
        for (size_t i = 0; i < slots_.size(); i++)
            if (used_[i]) out.push_back(slots_[i].k);
        return out;
    }

  private:
    struct Slot {
        uint64_t h;
        V3 k;
    };
    std::vector<Slot> slots_;
    std::vector<bool> used_;
    long usable_;
    size_t count_ = 0;

    bool find(const V3 &k, uint64_t h) const {
        const uint64_t mask = slots_.size() - 1;
        uint64_t i = h & mask, perturb = h;
        while (used_[i]) {
            if (slots_[i].h == h && same(slots_[i].k, k)) return true;
            i = (i * 5 + perturb + 1) & mask;
            perturb >>= 5;
        }
        return false;
    }

    void place(const V3 &k, uint64_t h) {
        const uint64_t mask = slots_.size() - 1;
        uint64_t i = h & mask, perturb = h;
        while (used_[i]) {
            i = (i * 5 + perturb + 1) & mask;
            perturb >>= 5;
        }
        slots_[i] = Slot{h, k};
        used_[i] = true;
    }

    void resize(size_t minused) {
        size_t n = 8;
        while (n <= minused) n <<= 1;
        std::vector<Slot> old;
        for (size_t i = 0; i < slots_.size(); i++)
            if (used_[i]) old.push_back(slots_[i]);
        slots_.assign(n, Slot{});
        used_.assign(n, false);
        usable_ = (long)((2 * n + 1) / 3) - (long)old.size();
        for (const Slot &s : old) place(s.k, s.h);
    }
};

inline V3 midpoint_dir(const V3 &a, const V3 &b) {
    const V3 m{(a.x + b.x) / 2.0, (a.y + b.y) / 2.0, (a.z + b.z) / 2.0};
    const double len = std::sqrt(m.x * m.x + m.y * m.y + m.z * m.z);
    return V3{m.x / len, m.y / len, m.z / len};
}

inline void subdivide(PyDict &d, const V3 &a, const V3 &b, const V3 &c, int n) {
    if (n <= 0) return;
    const V3 ab = midpoint_dir(a, b), bc = midpoint_dir(b, c), ca = midpoint_dir(c, a);
    if (n == 1) {
        for (const V3 &v : {a, b, c, ab, bc, ca}) d.insert(v);
        return;
    }
    subdivide(d, a, ab, ca, n - 1);
    subdivide(d, b, ab, bc, n - 1);
    subdivide(d, c, bc, ca, n - 1);
    subdivide(d, ab, bc, ca, n - 1);
}

/* the table of `levels` subdivisions as float xyz triples, in the reference's order */
inline std::vector<float> geosphere(int levels) {
    const double pi = 3.141592653589793;
    const V3 top{0, 0, 1};
    V3 eq[5];
    const double deg[5] = {90, 180, 270, 360, 90};
    for (int i = 0; i < 4; i++) eq[i] = V3{std::sin(deg[i] / 180 * pi), std::cos(deg[i] / 180 * pi), 0};
    eq[4] = eq[0];
    PyDict d;
    for (int f = 0; f < 4; f++) subdivide(d, top, eq[f], eq[f + 1], levels);
    std::vector<float> out;
    for (const V3 &v : d.keys()) {
        if (v.z == 0.0) continue;
        out.push_back((float)v.x);
        out.push_back((float)v.y);
        out.push_back((float)v.z);
    }
    return out;
}

} // namespace fmgi_geo

#endif
