// acmmp_delaunay.cpp — DelaunayTriangulation (src/ACMMP.cpp:896-918) of the
// planar prior's support points, host code (the rest of the planar-prior
// construction is on the GPU, acmmp_planar.hip).
//
// Pin: cv::Subdiv2D is replaced by an exact Delaunay
// triangulation seeded with Subdiv2D's own bounding triangle (3·max(w,h),
// from OpenCV's initDelaunay) so hull behaviour matches; co-circular ties
// keep the existing triangulation (strict in-circle test).
#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/acmmp.h"

namespace {

// ---------------------------------------------------------------- Delaunay
// Bowyer-Watson over integer points with exact orientation / in-circle
// predicates (coordinates are pixel integers, |c| < 2^20, so int64 / int128
// arithmetic is exact). Triangles are counter-clockwise; nb[i] is the
// triangle across the edge opposite v[i].
struct Delaunay {
    struct Tri {
        int v[3];
        int nb[3];
        int mark;
        bool alive;
    };
    std::vector<int64_t> X, Y;
    std::vector<Tri> T;

    int64_t orient(int a, int b, int c) const {
        return (X[b] - X[a]) * (Y[c] - Y[a]) - (Y[b] - Y[a]) * (X[c] - X[a]);
    }
    // > 0 when d lies strictly inside the circumcircle of CCW (a, b, c)
    bool in_circle(const Tri &t, int d) const {
        const __int128 adx = X[t.v[0]] - X[d], ady = Y[t.v[0]] - Y[d];
        const __int128 bdx = X[t.v[1]] - X[d], bdy = Y[t.v[1]] - Y[d];
        const __int128 cdx = X[t.v[2]] - X[d], cdy = Y[t.v[2]] - Y[d];
        const __int128 det = (adx * adx + ady * ady) * (bdx * cdy - cdx * bdy) +
                             (bdx * bdx + bdy * bdy) * (cdx * ady - adx * cdy) +
                             (cdx * cdx + cdy * cdy) * (adx * bdy - bdx * ady);
        return det > 0;
    }

    int locate(int p, int t) const {
        for (size_t guard = 0; guard < 4 * T.size() + 16; ++guard) {
            const Tri &tr = T[t];
            int next = -1;
            for (int i = 0; i < 3; ++i)
                if (orient(tr.v[(i + 1) % 3], tr.v[(i + 2) % 3], p) < 0) {
                    next = tr.nb[i];
                    break;
                }
            if (next < 0) return t;
            t = next;
        }
        return -1;
    }

    bool insert(int p, int &last, int stamp) {
        const int t0 = locate(p, last);
        if (t0 < 0) return false;
        for (int i = 0; i < 3; ++i)
            if (X[T[t0].v[i]] == X[p] && Y[T[t0].v[i]] == Y[p]) return true;  // duplicate point
        std::vector<int> bad{t0}, stack{t0};
        T[t0].mark = stamp;
        while (!stack.empty()) {
            const int t = stack.back();
            stack.pop_back();
            for (int i = 0; i < 3; ++i) {
                const int nb = T[t].nb[i];
                if (nb >= 0 && T[nb].mark != stamp && in_circle(T[nb], p)) {
                    T[nb].mark = stamp;
                    bad.push_back(nb);
                    stack.push_back(nb);
                }
            }
        }
        struct NewTri {
            int a, b, id;
        };
        std::vector<NewTri> made;
        for (const int t : bad) {
            for (int i = 0; i < 3; ++i) {
                const int nb = T[t].nb[i];
                if (nb >= 0 && T[nb].mark == stamp) continue;
                const int a = T[t].v[(i + 1) % 3], b = T[t].v[(i + 2) % 3];
                Tri nt{{a, b, p}, {-1, -1, nb}, 0, true};
                const int id = (int)T.size();
                if (nb >= 0)
                    for (int j = 0; j < 3; ++j)
                        if (T[nb].nb[j] == t) T[nb].nb[j] = id;
                T.push_back(nt);
                made.push_back({a, b, id});
            }
        }
        for (const int t : bad) T[t].alive = false;
        for (const NewTri &m : made) {
            for (const NewTri &o : made) {
                if (o.a == m.b) T[m.id].nb[0] = o.id;  // edge (b, p) shared with (b, c, p)
                if (o.b == m.a) T[m.id].nb[1] = o.id;  // edge (p, a) shared with (z, a, p)
            }
        }
        last = made.empty() ? last : made.back().id;
        return true;
    }
};

}  // namespace

extern "C" {

int acmmp_delaunay_triangulation(int width, int height, const int32_t *xy, int npoints, int32_t *tris,
                                 int capacity, int *ntris) {
    if (!ntris || width <= 0 || height <= 0 || npoints < 0 || (npoints > 0 && !xy) || capacity < 0 ||
        (capacity > 0 && !tris))
        return ACMMP_ERR_ARG;
    *ntris = 0;
    if (npoints == 0) return ACMMP_OK;  // :898-900
    Delaunay dt;
    const int64_t big = 3 * (int64_t)std::max(width, height);  // Subdiv2D::initDelaunay(rect)
    dt.X = {big, 0, -big};
    dt.Y = {0, big, -big};
    dt.X.reserve(npoints + 3);
    dt.Y.reserve(npoints + 3);
    for (int i = 0; i < npoints; ++i) {
        if (xy[2 * i] < 0 || xy[2 * i] >= width || xy[2 * i + 1] < 0 || xy[2 * i + 1] >= height)
            return ACMMP_ERR_ARG;
        dt.X.push_back(xy[2 * i]);
        dt.Y.push_back(xy[2 * i + 1]);
    }
    dt.T.reserve((size_t)npoints * 7 + 16);
    dt.T.push_back({{0, 1, 2}, {-1, -1, -1}, 0, true});
    int last = 0;
    for (int i = 0; i < npoints; ++i)
        if (!dt.insert(i + 3, last, i + 1)) return ACMMP_ERR_STATE;
    int n = 0;
    for (const auto &t : dt.T) {
        if (!t.alive || t.v[0] < 3 || t.v[1] < 3 || t.v[2] < 3) continue;
        if (n < capacity)
            for (int k = 0; k < 3; ++k) {
                tris[6 * n + 2 * k] = (int32_t)dt.X[t.v[k]];
                tris[6 * n + 2 * k + 1] = (int32_t)dt.Y[t.v[k]];
            }
        ++n;
    }
    *ntris = n;
    return n > capacity ? ACMMP_ERR_ARG : ACMMP_OK;
}

}  // extern "C"
