// tt_synth.cpp — seeded synthetic scenes shaped like the BASELINE.json configs (the Sponza,
// Bistro and San Miguel assets are not in the reference tree: .MISSING_LARGE_BLOBS:14-15).
// Every generator is deterministic for a given seed (std::mt19937_64 + explicit transforms,
// no std:: distributions, whose output is implementation-defined).
#include "tt_synth.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <random>
#include <vector>

struct tt_synth_mesh {
    std::vector<float> pos, nrm, uv;
    std::vector<int32_t> idx, mat;
};

namespace {

struct Rng {
    std::mt19937_64 g;
    explicit Rng(uint64_t s) : g(s) {}
    double u01() { return (double)(g() >> 11) * (1.0 / 9007199254740992.0); }
    double uni(double a, double b) { return a + (b - a) * u01(); }
    double normal() {  // Box-Muller
        double u1 = u01();
        if (u1 < 1e-300) u1 = 1e-300;
        const double u2 = u01();
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
    double lognormal(double median, double sigma) { return median * std::exp(sigma * normal()); }
};

struct D3 {
    double x, y, z;
};
static D3 d3(double x, double y, double z) { return D3{x, y, z}; }
static D3 add(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
static D3 sub(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
static D3 scl(D3 a, double s) { return d3(a.x * s, a.y * s, a.z * s); }
static D3 crs(D3 a, D3 b) { return d3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static D3 nrmz(D3 a) {
    const double l = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return l > 0 ? scl(a, 1.0 / l) : d3(0, 1, 0);
}

struct Builder {
    tt_synth_mesh* m;
    int32_t vert(D3 p, D3 n, double u, double v) {
        const int32_t id = (int32_t)(m->pos.size() / 3);
        m->pos.push_back((float)p.x); m->pos.push_back((float)p.y); m->pos.push_back((float)p.z);
        m->nrm.push_back((float)n.x); m->nrm.push_back((float)n.y); m->nrm.push_back((float)n.z);
        m->uv.push_back((float)u); m->uv.push_back((float)v);
        return id;
    }
    void tri(int32_t a, int32_t b, int32_t c, int32_t mat) {
        m->idx.push_back(a); m->idx.push_back(b); m->idx.push_back(c);
        m->mat.push_back(mat);
    }
    size_t ntri() const { return m->idx.size() / 3; }
    // Parametric grid surface f(s,t), s,t in [0,1], nu x nv quads.
    template <class F>
    void grid(int nu, int nv, int32_t mat, F f) {
        const int32_t base = (int32_t)(m->pos.size() / 3);
        for (int j = 0; j <= nv; j++) {
            for (int i = 0; i <= nu; i++) {
                const double s = (double)i / nu, t = (double)j / nv;
                const D3 p = f(s, t);
                const double e = 1e-4;
                const D3 ds = sub(f(s + e, t), f(s - e, t)), dt = sub(f(s, t + e), f(s, t - e));
                vert(p, nrmz(crs(ds, dt)), s, t);
            }
        }
        for (int j = 0; j < nv; j++) {
            for (int i = 0; i < nu; i++) {
                const int32_t a = base + j * (nu + 1) + i, b = a + 1, c = a + (nu + 1), d = c + 1;
                tri(a, c, b, mat);
                tri(b, c, d, mat);
            }
        }
    }
    void box(D3 lo, D3 hi, int n, int32_t mat) {
        const D3 s = sub(hi, lo);
        // six faces, n x n quads each
        grid(n, n, mat, [&](double u, double v) { return d3(lo.x + s.x * u, lo.y + s.y * v, lo.z); });
        grid(n, n, mat, [&](double u, double v) { return d3(lo.x + s.x * v, lo.y + s.y * u, hi.z); });
        grid(n, n, mat, [&](double u, double v) { return d3(lo.x, lo.y + s.y * u, lo.z + s.z * v); });
        grid(n, n, mat, [&](double u, double v) { return d3(hi.x, lo.y + s.y * v, lo.z + s.z * u); });
        grid(n, n, mat, [&](double u, double v) { return d3(lo.x + s.x * v, lo.y, lo.z + s.z * u); });
        grid(n, n, mat, [&](double u, double v) { return d3(lo.x + s.x * u, hi.y, lo.z + s.z * v); });
    }
};

}  // namespace

extern "C" {

tt_status tt_synth_mesh_view(const tt_synth_mesh* m, tt_mesh_input* v) {
    if (!m || !v) return TT_ERR_INVALID_ARG;
    std::memset(v, 0, sizeof(*v));
    v->positions = m->pos.data();
    v->n_vertices = (uint32_t)(m->pos.size() / 3);
    v->normals = m->nrm.data();
    v->tangents = nullptr;
    v->uvs = m->uv.data();
    v->indices = m->idx.data();
    v->n_indices = (uint32_t)m->idx.size();
    v->matdat = m->mat.data();
    v->lossy_scale[0] = v->lossy_scale[1] = v->lossy_scale[2] = 1.0f;
    return TT_OK;
}

void tt_synth_mesh_free(tt_synth_mesh* m) { delete m; }

tt_synth_mesh* tt_synth_mesh_from_arrays(const float* pos, uint32_t n_vertices, const int32_t* idx,
                                         uint32_t n_indices, const int32_t* matdat) {
    tt_synth_mesh* m = new (std::nothrow) tt_synth_mesh();
    if (!m) return nullptr;
    m->pos.assign(pos, pos + 3 * (size_t)n_vertices);
    m->nrm.assign(3 * (size_t)n_vertices, 0.0f);
    for (uint32_t i = 0; i < n_vertices; i++) m->nrm[3 * i + 1] = 1.0f;
    m->uv.assign(2 * (size_t)n_vertices, 0.0f);
    m->idx.assign(idx, idx + n_indices);
    m->mat.assign(n_indices / 3, 0);
    if (matdat) m->mat.assign(matdat, matdat + n_indices / 3);
    return m;
}

// C1 Cornell box: room [-1,1]^3 with 5 walls (front open, 10 tris) and a
// ceiling light quad |x|,|z| <= 0.25 at y = 0.999 (2 tris).
tt_status tt_synth_cornell(tt_synth_mesh** out) {
    if (!out) return TT_ERR_INVALID_ARG;
    tt_synth_mesh* m = new (std::nothrow) tt_synth_mesh();
    if (!m) return TT_ERR_OOM;
    Builder b{m};
    auto quad = [&](D3 a, D3 bb, D3 c, D3 d, int32_t mat) {
        const D3 n = nrmz(crs(sub(bb, a), sub(d, a)));
        const int32_t i0 = b.vert(a, n, 0, 0), i1 = b.vert(bb, n, 1, 0), i2 = b.vert(c, n, 1, 1), i3 = b.vert(d, n, 0, 1);
        b.tri(i0, i1, i2, mat);
        b.tri(i0, i2, i3, mat);
    };
    quad(d3(-1, -1, -1), d3(1, -1, -1), d3(1, -1, 1), d3(-1, -1, 1), 0);   // floor
    quad(d3(-1, 1, -1), d3(-1, 1, 1), d3(1, 1, 1), d3(1, 1, -1), 0);       // ceiling
    quad(d3(-1, -1, -1), d3(-1, 1, -1), d3(1, 1, -1), d3(1, -1, -1), 0);   // back
    quad(d3(-1, -1, -1), d3(-1, -1, 1), d3(-1, 1, 1), d3(-1, 1, -1), 1);   // left (red)
    quad(d3(1, -1, -1), d3(1, 1, -1), d3(1, 1, 1), d3(1, -1, 1), 2);       // right (green)
    quad(d3(-0.25, 0.999, -0.25), d3(-0.25, 0.999, 0.25), d3(0.25, 0.999, 0.25), d3(0.25, 0.999, -0.25), 3);  // light
    *out = m;
    return TT_OK;
}

// Uniform triangle soup in a cube of half-size `extent`, edge ~ lognormal(tri_size, 0.5).
tt_status tt_synth_soup(uint64_t seed, uint32_t n_tris, float extent, float tri_size, tt_synth_mesh** out) {
    if (!out || !n_tris) return TT_ERR_INVALID_ARG;
    tt_synth_mesh* m = new (std::nothrow) tt_synth_mesh();
    if (!m) return TT_ERR_OOM;
    Builder b{m};
    Rng r(seed);
    for (uint32_t t = 0; t < n_tris; t++) {
        const D3 c = d3(r.uni(-extent, extent), r.uni(-extent, extent), r.uni(-extent, extent));
        const double s = r.lognormal(tri_size, 0.5);
        D3 p[3];
        for (int k = 0; k < 3; k++) p[k] = add(c, d3(r.uni(-s, s), r.uni(-s, s), r.uni(-s, s)));
        const D3 n = nrmz(crs(sub(p[1], p[0]), sub(p[2], p[0])));
        const int32_t a = b.vert(p[0], n, 0, 0), bb = b.vert(p[1], n, 1, 0), cc = b.vert(p[2], n, 0, 1);
        b.tri(a, bb, cc, (int32_t)(t % 4));
    }
    *out = m;
    return TT_OK;
}

// C2 Sponza-shaped hall: ~30 x 13 x 18 m, two colonnade floors of
// tessellated columns and arches, walls/floor grids, curtains and foliage clumps; padded with
// foliage to exactly n_tris triangles. Materials: 0 floor, 1 walls, 2 columns, 3 arches,
// 4 slabs, 5 curtains, 6 foliage.
tt_status tt_synth_sponza(uint64_t seed, uint32_t n_tris, tt_synth_mesh** out) {
    if (!out || n_tris < 200000) return TT_ERR_INVALID_ARG;
    tt_synth_mesh* m = new (std::nothrow) tt_synth_mesh();
    if (!m) return TT_ERR_OOM;
    Builder b{m};
    Rng r(seed);
    const double X0 = -15, X1 = 15, Z0 = -9, Z1 = 9, H = 13;
    const double PI = 3.141592653589793;
    // floor, slightly uneven tiles
    b.grid(96, 56, 0, [&](double u, double v) {
        return d3(X0 + (X1 - X0) * u, 0.002 * std::sin(40 * u) * std::sin(33 * v), Z0 + (Z1 - Z0) * v);
    });
    // walls with masonry relief
    auto wall = [&](D3 o, D3 du, D3 dv, D3 nrm, int nu, int nv) {
        b.grid(nu, nv, 1, [&](double u, double v) {
            const double relief = 0.01 * std::sin(u * 180.0) * std::sin(v * 70.0);
            return add(add(add(o, scl(du, u)), scl(dv, v)), scl(nrm, relief));
        });
    };
    wall(d3(X0, 0, Z0), d3(X1 - X0, 0, 0), d3(0, H, 0), d3(0, 0, 1), 110, 48);
    wall(d3(X0, 0, Z1), d3(0, H, 0), d3(X1 - X0, 0, 0), d3(0, 0, -1), 48, 110);
    wall(d3(X0, 0, Z0), d3(0, H, 0), d3(0, 0, Z1 - Z0), d3(1, 0, 0), 48, 66);
    wall(d3(X1, 0, Z0), d3(0, 0, Z1 - Z0), d3(0, H, 0), d3(-1, 0, 0), 66, 48);
    // balcony slabs and aisle roofs over z in [5,9] and [-9,-5]
    for (int side = -1; side <= 1; side += 2) {
        const double za = side > 0 ? 5.0 : -9.0, zb = side > 0 ? 9.0 : -5.0;
        b.box(d3(X0, 6.0, za), d3(X1, 6.4, zb), 12, 4);
        b.box(d3(X0, 12.6, za), d3(X1, 13.0, zb), 12, 4);
    }
    // colonnades: 2 sides x 2 floors x 9 columns, tessellated cylinders with bases/capitals
    const int nseg = 32, nring = 40;
    for (int side = -1; side <= 1; side += 2) {
        for (int fl = 0; fl < 2; fl++) {
            const double y0 = fl == 0 ? 0.0 : 6.4, y1 = fl == 0 ? 6.0 : 12.6;
            for (int c = 0; c < 9; c++) {
                const double cx = -12.0 + 3.0 * c, cz = 5.0 * side;
                const double rad = fl == 0 ? 0.38 : 0.30;
                b.grid(nseg, nring, 2, [&](double u, double v) {
                    const double a = 2 * PI * u, rr = rad * (1.0 + 0.04 * std::cos(16 * a));  // fluting
                    return d3(cx + rr * std::cos(a), y0 + (y1 - y0) * v, cz + rr * std::sin(a));
                });
                b.box(d3(cx - 0.5, y0, cz - 0.5), d3(cx + 0.5, y0 + 0.3, cz + 0.5), 4, 2);
                b.box(d3(cx - 0.55, y1 - 0.35, cz - 0.55), d3(cx + 0.55, y1, cz + 0.55), 4, 2);
            }
            // arches between adjacent columns: half-torus tubes in the x-y plane
            for (int c = 0; c < 8; c++) {
                const double ax = -12.0 + 3.0 * c + 1.5, az = 5.0 * side, ay = y1 - 1.5;
                b.grid(48, 16, 3, [&](double u, double v) {
                    const double th = PI * u, ph = 2 * PI * v, R = 1.5, rt = 0.22;
                    const double rr = R + rt * std::cos(ph);
                    return d3(ax - rr * std::cos(th), ay + rr * std::sin(th) * 0.9, az + rt * std::sin(ph));
                });
            }
        }
    }
    // curtains: wavy sheets hanging between ground-floor columns
    for (int k = 0; k < 6; k++) {
        const int side = (k % 2) ? 1 : -1;
        const double cx = -10.5 + 4.0 * k, cz = 5.0 * side + 0.6 * side;
        const double phase = r.uni(0, 6.28);
        b.grid(30, 60, 5, [&](double u, double v) {
            return d3(cx - 1.2 + 2.4 * u, 0.8 + 4.6 * v, cz + 0.12 * std::sin(18 * u + phase) * (0.3 + v));
        });
    }
    // foliage: clumps of small random leaves around plant pots, padding to exactly n_tris
    const size_t base = b.ntri();
    if (base >= n_tris) {
        delete m;
        return TT_ERR_INVALID_ARG;
    }
    const size_t leaves = n_tris - base;
    const int npots = 14;
    for (int pidx = 0; pidx < npots; pidx++) {
        const int side = (pidx % 2) ? 1 : -1;
        const double px = -13.0 + 2.0 * pidx, pz = (pidx % 3 == 0) ? 2.5 * side : 4.0 * side;
        b.box(d3(px - 0.35, 0.0, pz - 0.35), d3(px + 0.35, 0.6, pz + 0.35), 2, 6);
    }
    const size_t base2 = b.ntri();
    const size_t nleaf = n_tris - base2;
    (void)leaves;
    for (size_t t = 0; t < nleaf; t++) {
        const int pidx = (int)(t % npots);
        const int side = (pidx % 2) ? 1 : -1;
        const double px = -13.0 + 2.0 * pidx, pz = (pidx % 3 == 0) ? 2.5 * side : 4.0 * side;
        // leaf centre in an ellipsoidal bush above the pot
        double dx, dy, dz;
        do {
            dx = r.uni(-1, 1); dy = r.uni(-1, 1); dz = r.uni(-1, 1);
        } while (dx * dx + dy * dy + dz * dz > 1.0);
        const D3 c = d3(px + 0.9 * dx, 1.5 + 0.9 * dy, pz + 0.9 * dz);
        const double s = std::min(0.4, r.lognormal(0.08, 0.6));
        const D3 e1 = nrmz(d3(r.normal(), r.normal(), r.normal()));
        const D3 e2 = nrmz(crs(e1, nrmz(d3(r.normal(), r.normal(), r.normal()))));
        const D3 p0 = c, p1 = add(c, scl(e1, s)), p2 = add(c, scl(add(scl(e1, 0.5 * s), scl(e2, 0.6 * s)), 1.0));
        const D3 n = nrmz(crs(sub(p1, p0), sub(p2, p0)));
        const int32_t a = b.vert(p0, n, 0, 0), bb = b.vert(p1, n, 1, 0), cc = b.vert(p2, n, 0, 1);
        b.tri(a, bb, cc, 6);
    }
    *out = m;
    return TT_OK;
}

// Flat ground grid of nu x nv quads over [x0,x1] x [z0,z1] at y = 0 with a gentle camber
// (C4's street plane). Material 0.
tt_status tt_synth_ground(double x0, double x1, double z0, double z1, uint32_t nu, uint32_t nv,
                          tt_synth_mesh** out) {
    if (!out || !nu || !nv || !(x1 > x0) || !(z1 > z0)) return TT_ERR_INVALID_ARG;
    tt_synth_mesh* m = new (std::nothrow) tt_synth_mesh();
    if (!m) return TT_ERR_OOM;
    Builder b{m};
    b.grid((int)nu, (int)nv, 0, [&](double u, double v) {
        return d3(x0 + (x1 - x0) * u, 0.02 * std::sin(17.0 * u) * std::cos(13.0 * v), z0 + (z1 - z0) * v);
    });
    *out = m;
    return TT_OK;
}

// C5 San-Miguel-shaped courtyard: a ~44 x 14 x 32 m patio closed on three
// sides by two-storey arcades (walls, fluted columns, arches, balcony slabs), paved floor,
// tables and chairs, and ~60% foliage-like small triangles (tree crowns, potted plants, wall
// ivy), padded to exactly n_tris. Tessellation of the architecture scales with n_tris so the
// foliage share stays about the same. Materials: 0 floor, 1 walls, 2 columns, 3 arches,
// 4 slabs, 5 furniture, 6 trunks, 7 foliage.
tt_status tt_synth_san_miguel(uint64_t seed, uint32_t n_tris, tt_synth_mesh** out) {
    if (!out || n_tris < 1000000) return TT_ERR_INVALID_ARG;
    tt_synth_mesh* m = new (std::nothrow) tt_synth_mesh();
    if (!m) return TT_ERR_OOM;
    Builder b{m};
    Rng r(seed);
    const double PI = 3.141592653589793;
    const double X0 = -22, X1 = 22, Z0 = -16, Z1 = 16, H = 14;
    // ~730k architecture triangles at s = 1; aim for ~40% architecture
    const double s = std::sqrt(0.4 * (double)n_tris / 730000.0);
    auto res = [&](double base) { return std::max(2, (int)std::lround(base * s)); };
    // paved floor with slightly raised cobbles
    b.grid(res(400), res(300), 0, [&](double u, double v) {
        return d3(X0 + (X1 - X0) * u, 0.004 * std::sin(310 * u) * std::sin(233 * v), Z0 + (Z1 - Z0) * v);
    });
    auto wall = [&](D3 o, D3 du, D3 dv, D3 nrm, int nu, int nv) {
        b.grid(nu, nv, 1, [&](double u, double v) {
            const double relief = 0.015 * std::sin(u * 240.0) * std::sin(v * 90.0);
            return add(add(add(o, scl(du, u)), scl(dv, v)), scl(nrm, relief));
        });
    };
    wall(d3(X0, 0, Z1), d3(0, H, 0), d3(X1 - X0, 0, 0), d3(0, 0, -1), res(100), res(300));
    wall(d3(X0, 0, Z0), d3(0, H, 0), d3(0, 0, Z1 - Z0), d3(1, 0, 0), res(100), res(220));
    wall(d3(X1, 0, Z0), d3(0, 0, Z1 - Z0), d3(0, H, 0), d3(-1, 0, 0), res(220), res(100));
    // arcades 4 m deep along the back (z) and both sides (x): slabs, columns, arches
    b.box(d3(X0, 6.5, Z1 - 4), d3(X1, 6.9, Z1), res(10), 4);
    b.box(d3(X0, 6.5, Z0), d3(X0 + 4, 6.9, Z1 - 4), res(10), 4);
    b.box(d3(X1 - 4, 6.5, Z0), d3(X1, 6.9, Z1 - 4), res(10), 4);
    struct Col { double x, z; };
    std::vector<Col> cols;
    for (int c = 0; c < 12; c++) cols.push_back(Col{X0 + 2.0 + 3.636 * c, Z1 - 4});
    for (int c = 0; c < 8; c++) cols.push_back(Col{X0 + 4, Z0 + 2.0 + 3.5 * c});
    for (int c = 0; c < 8; c++) cols.push_back(Col{X1 - 4, Z0 + 2.0 + 3.5 * c});
    const int nseg = res(32), nring = res(40);
    for (int fl = 0; fl < 2; fl++) {
        const double y0 = fl == 0 ? 0.0 : 6.9, y1 = fl == 0 ? 6.5 : 13.2, rad = fl == 0 ? 0.34 : 0.27;
        for (const Col& c : cols) {
            b.grid(nseg, nring, 2, [&](double u, double v) {
                const double a = 2 * PI * u, rr = rad * (1.0 + 0.05 * std::cos(12 * a));
                return d3(c.x + rr * std::cos(a), y0 + (y1 - y0) * v, c.z + rr * std::sin(a));
            });
        }
        for (size_t k = 0; k + 1 < cols.size(); k++) {
            const Col a = cols[k], c = cols[k + 1];
            const double dx = c.x - a.x, dz = c.z - a.z, len = std::sqrt(dx * dx + dz * dz);
            if (len > 4.0) continue;  // no arch across the corner
            const double R = 0.5 * len, ay = y1 - R;
            b.grid(res(48), res(16), 3, [&](double u, double v) {
                const double th = PI * u, ph = 2 * PI * v, rt = 0.18, rr = R + rt * std::cos(ph);
                const double along = R - rr * std::cos(th);
                return d3(a.x + dx / len * along, ay + rr * std::sin(th) * 0.85, a.z + dz / len * along + rt * std::sin(ph));
            });
        }
    }
    // furniture: 30 tables (top + leg) with four chairs each
    for (int t = 0; t < 30; t++) {
        const double tx = r.uni(X0 + 6, X1 - 6), tz = r.uni(Z0 + 2, Z1 - 6);
        b.box(d3(tx - 0.45, 0.72, tz - 0.45), d3(tx + 0.45, 0.76, tz + 0.45), res(8), 5);
        b.box(d3(tx - 0.04, 0.0, tz - 0.04), d3(tx + 0.04, 0.72, tz + 0.04), res(4), 5);
        for (int c = 0; c < 4; c++) {
            const double a = PI / 2 * c + r.uni(-0.3, 0.3), cx = tx + 0.75 * std::cos(a), cz = tz + 0.75 * std::sin(a);
            b.box(d3(cx - 0.2, 0.42, cz - 0.2), d3(cx + 0.2, 0.46, cz + 0.2), res(5), 5);
            b.box(d3(cx - 0.2, 0.46, cz - 0.2), d3(cx + 0.2, 0.95, cz - 0.16), res(5), 5);
        }
    }
    // trees: trunks now, crowns later with the leaves
    struct Tree { double x, z, cy, rx, ry; };
    std::vector<Tree> trees;
    for (int t = 0; t < 10; t++) {
        Tree tr{r.uni(X0 + 7, X1 - 7), r.uni(Z0 + 3, Z1 - 7), r.uni(6.0, 8.5), r.uni(2.5, 4.0), r.uni(2.0, 3.0)};
        trees.push_back(tr);
        b.grid(res(24), res(24), 6, [&](double u, double v) {
            const double a = 2 * PI * u, rr = 0.25 * (1.2 - 0.4 * v);
            return d3(tr.x + rr * std::cos(a), (tr.cy - 0.5 * tr.ry) * v, tr.z + rr * std::sin(a));
        });
    }
    if (b.ntri() >= n_tris) {
        delete m;
        return TT_ERR_INVALID_ARG;
    }
    // foliage: 70% tree crowns, 15% potted plants along the arcades, 15% ivy on the walls
    const size_t nleaf = n_tris - b.ntri();
    auto leaf = [&](D3 c, double size) {
        const D3 e1 = nrmz(d3(r.normal(), r.normal(), r.normal()));
        const D3 e2 = nrmz(crs(e1, nrmz(d3(r.normal(), r.normal(), r.normal()))));
        const D3 p0 = c, p1 = add(c, scl(e1, size)), p2 = add(c, add(scl(e1, 0.5 * size), scl(e2, 0.6 * size)));
        const D3 n = nrmz(crs(sub(p1, p0), sub(p2, p0)));
        const int32_t a = b.vert(p0, n, 0, 0), bb = b.vert(p1, n, 1, 0), cc = b.vert(p2, n, 0, 1);
        b.tri(a, bb, cc, 7);
    };
    for (size_t t = 0; t < nleaf; t++) {
        const double kind = r.u01();
        const double size = std::min(0.25, r.lognormal(0.05, 0.5));
        double dx, dy, dz;
        do {
            dx = r.uni(-1, 1); dy = r.uni(-1, 1); dz = r.uni(-1, 1);
        } while (dx * dx + dy * dy + dz * dz > 1.0);
        if (kind < 0.70) {
            const Tree& tr = trees[t % trees.size()];
            leaf(d3(tr.x + tr.rx * dx, tr.cy + tr.ry * dy, tr.z + tr.rx * dz), size);
        } else if (kind < 0.85) {
            const int pot = (int)(t % cols.size());
            leaf(d3(cols[pot].x + 0.8 + 0.5 * dx, 0.9 + 0.5 * dy, cols[pot].z - 0.8 + 0.5 * dz), size);
        } else {
            const int w = (int)(t % 3);
            const double u = r.u01(), v = r.u01() * 0.85, off = 0.05 + 0.1 * r.u01();
            if (w == 0) leaf(d3(X0 + (X1 - X0) * u, H * v, Z1 - off), size);
            else if (w == 1) leaf(d3(X0 + off, H * v, Z0 + (Z1 - Z0) * u), size);
            else leaf(d3(X1 - off, H * v, Z0 + (Z1 - Z0) * u), size);
        }
    }
    *out = m;
    return TT_OK;
}

// C4 building block: one Bistro-shaped unique object (a facade/prop) with n_tris triangles in
// its own object space (about 1-12 m), for two-level instancing scenes.
tt_status tt_synth_prop(uint64_t seed, uint32_t n_tris, tt_synth_mesh** out) {
    if (!out || n_tris < 8) return TT_ERR_INVALID_ARG;
    tt_synth_mesh* m = new (std::nothrow) tt_synth_mesh();
    if (!m) return TT_ERR_OOM;
    Builder b{m};
    Rng r(seed);
    const int kind = (int)(r.g() % 3);
    const double sx = r.uni(1.0, 8.0), sy = r.uni(1.0, 12.0), sz = r.uni(1.0, 8.0);
    // main body: a relief grid wrapped as a box-ish shell until ~70% of the budget
    const uint32_t body = n_tris * 7 / 10;
    const int n = std::max(1, (int)std::sqrt((double)body / 12.0));
    if (kind == 0) {
        b.box(d3(-sx / 2, 0, -sz / 2), d3(sx / 2, sy, sz / 2), n, 0);
    } else {
        const int nu = std::max(3, n * 2), nv = std::max(2, n * 3 / 2);
        b.grid(nu, nv, 1, [&](double u, double v) {
            const double a = 6.283185307179586 * u, rr = 0.5 * sx * (1.0 + 0.1 * std::sin(7 * v + kind));
            return d3(rr * std::cos(a), sy * v, rr * std::sin(a) * sz / sx);
        });
    }
    while (b.ntri() < n_tris) {
        const D3 c = d3(r.uni(-sx / 2, sx / 2), r.uni(0, sy), r.uni(-sz / 2, sz / 2));
        const double s = std::min(1.0, r.lognormal(0.1, 0.7));
        D3 p[3];
        for (int k = 0; k < 3; k++) p[k] = add(c, d3(r.uni(-s, s), r.uni(-s, s), r.uni(-s, s)));
        const D3 nn = nrmz(crs(sub(p[1], p[0]), sub(p[2], p[0])));
        const int32_t a = b.vert(p[0], nn, 0, 0), bb = b.vert(p[1], nn, 1, 0), cc = b.vert(p[2], nn, 0, 1);
        b.tri(a, bb, cc, 2);
    }
    // trim to exactly n_tris
    m->idx.resize(3 * (size_t)n_tris);
    m->mat.resize(n_tris);
    *out = m;
    return TT_OK;
}

}  // extern "C"
