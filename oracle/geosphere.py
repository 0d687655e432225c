"""oracle/geosphere.py -- TEST INFRASTRUCTURE ONLY: the ambient-occlusion direction table (the
reference's geoSphere4, geoSphere.h:21), regenerated the way the reference's generator script
geoSphere.py produced it, for checking the product's own generator (csrc/fmgi_geosphere.h).

The script subdivides the 4 upper faces of an octahedron, keeps every vertex once in a Python dict
and prints the dict's keys with z != 0. Its output order is the slot order of a CPython dict before
3.6 (open addressing over tuple hashes), replayed here by `Dict35`. Squares are correctly rounded
products (x*x); the script's x**2 gave exactly that on the machine that generated the reference.
oracle/geosphere_check.py compares this output with the reference's geoSphere.c."""
import math

import numpy as np

_M61 = (1 << 61) - 1
_U64 = (1 << 64) - 1


def hash_float(x: float) -> int:
    """CPython 3.x numeric hash of a float (== hash(x) on any 3.x)."""
    return hash(float(x))


def hash_tuple35(t) -> int:
    """CPython < 3.8 tuple hash (tupleobject.c), as an unsigned 64-bit value."""
    x, mult, n = 0x345678, 1000003, len(t)
    for i, item in enumerate(t):
        x = ((x ^ (hash_float(item) & _U64)) * mult) & _U64
        mult = (mult + 82520 + 2 * (n - 1 - i)) & _U64
    x = (x + 97531) & _U64
    return (-2) & _U64 if x == _U64 else x


class Dict35:
    """Insertion-only CPython < 3.6 dict: iteration order = slot order."""

    def __init__(self):
        self.slots = [None] * 8
        self.used = 0
        self.usable = (2 * 8 + 1) // 3

    def _probe(self, slots, h):
        mask = len(slots) - 1
        i, perturb = h & mask, h
        while slots[i] is not None:
            yield i
            i = (i * 5 + perturb + 1) & mask
            perturb >>= 5
        yield i

    def insert(self, k):
        h = hash_tuple35(k)
        for i in self._probe(self.slots, h):
            e = self.slots[i]
            if e is not None and e[0] == h and e[1] == k:
                return
        if self.usable <= 0:
            self._resize(self.used * 2 + len(self.slots) // 2)
        for i in self._probe(self.slots, h):
            pass
        self.slots[i] = (h, k)
        self.used += 1
        self.usable -= 1

    def _resize(self, minused):
        n = 8
        while n <= minused:
            n <<= 1
        old = [e for e in self.slots if e is not None]
        self.slots = [None] * n
        self.usable = (2 * n + 1) // 3 - len(old)
        for h, k in old:
            for i in self._probe(self.slots, h):
                pass
            self.slots[i] = (h, k)

    def keys(self):
        return [e[1] for e in self.slots if e is not None]


def generate(levels: int) -> np.ndarray:
    """float32 [n, 3] table of `levels` subdivisions, in the reference's order."""

    def add(a, b):
        return (a[0] + b[0], a[1] + b[1], a[2] + b[2])

    def mid(a, b):
        m = add(a, b)
        m = (m[0] / 2.0, m[1] / 2.0, m[2] / 2.0)
        n = math.sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2])
        return (m[0] / n, m[1] / n, m[2] / n)

    d = Dict35()

    def sub(a, b, c, n):
        if n <= 0:
            return
        ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
        if n == 1:
            for v in (a, b, c, ab, bc, ca):
                d.insert(v)
        else:
            sub(a, ab, ca, n - 1)
            sub(b, ab, bc, n - 1)
            sub(c, bc, ca, n - 1)
            sub(ab, bc, ca, n - 1)

    pi = math.pi
    top = (0, 0, 1)
    eq = [(math.sin(deg / 180 * pi), math.cos(deg / 180 * pi), 0) for deg in (90, 180, 270, 360)]
    for f in range(4):
        sub(top, eq[f], eq[(f + 1) % 4], levels)
    return np.array([k for k in d.keys() if k[2] != 0.0], dtype=np.float64).astype(np.float32)
