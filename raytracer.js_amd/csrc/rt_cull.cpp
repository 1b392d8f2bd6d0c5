// rt_cull.cpp — per-node cull hierarchies for rt_upload_scene.
//
// The reference tests a returned node's entities in EntitySet order and keeps the first one that
// reports a collision (src/raytracer.ts:186-195).  The GPU reaches the same entity with less work:
// each node's entity list gets a small binary BVH (SAH splits, one entity per leaf) whose boxes
// are the entities' AABBs widened by a margin `delta` and rounded outward to f32.  Only entities whose box the ray's half-line
// crosses run the exact binary64 test, and the hit with the smallest Set rank wins — the entity
// the reference's in-order loop stops at.  Entities whose exact test can be ill-conditioned
// (degenerate triangles, non-finite geometry) get an infinite box and are always tested.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "rt.h"
#include "rt_internal.h"

namespace {

struct Item {
    double lo[3], hi[3], c[3];
    int slot;           // index into the node's original (Set-order) prim records
};

float round_down(double x)
{
    float f = (float)x;
    if (isnan(x)) return -INFINITY;
    if ((double)f > x) f = nextafterf(f, -INFINITY);
    return f;
}

float round_up(double x)
{
    float f = (float)x;
    if (isnan(x)) return INFINITY;
    if ((double)f < x) f = nextafterf(f, INFINITY);
    return f;
}

// Conservative AABB of one primitive record (RtPrim layout), widened by delta.
void prim_bounds(const RtPrim &p, double delta, Item &it)
{
    const int type = p.meta & 3;
    const double *g = p.g;
    bool finite = true;
    if (type == RT_ENT_SPHERE) {
        // |2/d| recovers |d|: r = |d|/2 = 1/|k|
        const double r = 1.0 / fabs(g[6]);
        for (int i = 0; i < 3; i++) { it.lo[i] = g[i] - r; it.hi[i] = g[i] + r; }
        finite = isfinite(r);
    } else if (type == RT_ENT_BOX) {
        const double h = fabs(g[3]) * 0.5;
        for (int i = 0; i < 3; i++) { it.lo[i] = g[i] - h; it.hi[i] = g[i] + h; }
    } else {
        double l1 = 0, l2 = 0, l3 = 0;
        for (int i = 0; i < 3; i++) {
            const double v0 = g[i], v1 = g[i] + g[3 + i], v2 = g[i] + g[6 + i];
            it.lo[i] = std::min(v0, std::min(v1, v2));
            it.hi[i] = std::max(v0, std::max(v1, v2));
            l1 += g[3 + i] * g[3 + i];
            l2 += g[6 + i] * g[6 + i];
            l3 += (g[6 + i] - g[3 + i]) * (g[6 + i] - g[3 + i]);
        }
        const double L2 = std::max(l1, std::max(l2, l3));      // longest edge, squared
        // Moller-Trumbore divides by det = e1 . (d x e2).  Its rounding error, relative to the
        // barycentric margin a ray that misses the widened box has, is bounded by
        // ~6*sqrt(3)*eps*L^2*scale / (delta * |e1 x e2| * |cos(theta)|): negligible unless the
        // triangle is skinny (|e1 x e2| << L^2).  Skinny triangles (|e1 x e2| <= 1e-3 L^2) are
        // never culled; DESIGN.md §5.1 has the bound.
        const double cx = g[4] * g[8] - g[5] * g[7], cy = g[5] * g[6] - g[3] * g[8], cz = g[3] * g[7] - g[4] * g[6];
        const double area2 = cx * cx + cy * cy + cz * cz;
        if (!(area2 > 1e-6 * L2 * L2)) finite = false;
    }
    for (int i = 0; i < 3; i++) {
        finite = finite && isfinite(it.lo[i]) && isfinite(it.hi[i]) && isfinite(g[i]);
        it.c[i] = 0.5 * (it.lo[i] + it.hi[i]);
    }
    if (!finite) {
        for (int i = 0; i < 3; i++) {
            it.lo[i] = -INFINITY; it.hi[i] = INFINITY;
            it.c[i] = isfinite(g[i]) ? g[i] : 0.0;
        }
        return;
    }
    for (int i = 0; i < 3; i++) { it.lo[i] -= delta; it.hi[i] += delta; }
}

// Surface area of a box for the SAH cost, with infinite extents clamped to the scene scale.
double half_area(const double lo[3], const double hi[3], double clampv)
{
    double e[3];
    for (int i = 0; i < 3; i++) {
        const double l = std::max(lo[i], -clampv), h = std::min(hi[i], clampv);
        e[i] = h > l ? h - l : 0.0;
    }
    return e[0] * e[1] + e[1] * e[2] + e[2] * e[0];
}

struct Builder {
    std::vector<RtBvh> *bvh;
    std::vector<int> order;     // output slot order (indices into items)
    std::vector<Item> *items;
    bool sah;
    int leaf;                   // entities per leaf at most (RT_BVH_LEAF, 1..15)
    double clampv;              // SAH area clamp (scene scale)
    std::vector<double> right_area;

    // Full-sweep SAH over centroid-sorted items on every axis (sets are small: <= a few hundred
    // entities per node).  Returns the split index; items are left sorted on the chosen axis.
    int sah_split(int b, int e)
    {
        const int n = e - b;
        double best = INFINITY;
        int best_axis = -1, best_k = b + n / 2;
        right_area.resize(n + 1);
        for (int axis = 0; axis < 3; axis++) {
            std::sort(items->begin() + b, items->begin() + e, [axis](const Item &x, const Item &y) {
                return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.slot < y.slot);
            });
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int k = e - 1; k > b; k--) {
                const Item &it = (*items)[k];
                for (int i = 0; i < 3; i++) { lo[i] = std::min(lo[i], it.lo[i]); hi[i] = std::max(hi[i], it.hi[i]); }
                right_area[k - b] = half_area(lo, hi, clampv);
            }
            for (int i = 0; i < 3; i++) { lo[i] = INFINITY; hi[i] = -INFINITY; }
            for (int k = b + 1; k < e; k++) {
                const Item &it = (*items)[k - 1];
                for (int i = 0; i < 3; i++) { lo[i] = std::min(lo[i], it.lo[i]); hi[i] = std::max(hi[i], it.hi[i]); }
                const double cost = half_area(lo, hi, clampv) * (k - b) + right_area[k - b] * (e - k);
                if (cost < best) { best = cost; best_axis = axis; best_k = k; }
            }
        }
        if (best_axis != 2 && best_axis >= 0) {
            const int axis = best_axis;
            std::sort(items->begin() + b, items->begin() + e, [axis](const Item &x, const Item &y) {
                return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.slot < y.slot);
            });
        }
        return best_k;
    }

    void emit(int b, int e)     // items [b, e) of *items (already permuted in place)
    {
        const int me = (int)bvh->size();
        bvh->push_back(RtBvh());
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int k = b; k < e; k++) {
            const Item &it = (*items)[k];
            for (int i = 0; i < 3; i++) {
                lo[i] = std::min(lo[i], it.lo[i]); hi[i] = std::max(hi[i], it.hi[i]);
                clo[i] = std::min(clo[i], it.c[i]); chi[i] = std::max(chi[i], it.c[i]);
            }
        }
        RtBvh node;
        for (int i = 0; i < 3; i++) { node.lo[i] = round_down(lo[i]); node.hi[i] = round_up(hi[i]); }
        if (e - b <= leaf) {
            node.info = ((int)order.size() << 4) | (e - b);   // leaf: first prim slot << 4 | count
            for (int k = b; k < e; k++) order.push_back(k);
        } else {
            int mid;
            if (sah) {
                mid = sah_split(b, e);
            } else {
                int axis = 0;
                double ext = -1;
                for (int i = 0; i < 3; i++)
                    if (chi[i] - clo[i] > ext) { ext = chi[i] - clo[i]; axis = i; }
                mid = b + (e - b) / 2;
                std::nth_element(items->begin() + b, items->begin() + mid, items->begin() + e,
                                 [axis](const Item &x, const Item &y) {
                                     return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.slot < y.slot);
                                 });
            }
            node.info = -1;
            (*bvh)[me] = node;
            emit(b, mid);
            emit(mid, e);
        }
        node.skip = (int)bvh->size();
        (*bvh)[me] = node;
    }
};

}  // namespace

// Cull scale of a scene: delta (AABB widening) and the SAH area clamp, from the root cube only, so
// an incremental update rebuilds a node with the same constants as a full upload.
void rt_cull_scale(const double root_pos[3], double root_size, double *delta, double *clampv)
{
    double scale = fabs(root_size);
    for (int i = 0; i < 3; i++) scale = std::max(scale, std::max(fabs(root_pos[i]), fabs(root_pos[i] + root_size)));
    *delta = ldexp(scale, -13);          // ~1.2e-4 x scene scale
    *clampv = 4 * scale;
}

// One node's cull hierarchy (leaves of at most `leaf` entities).  `recs` are the node's c prim records in Set order (rank already
// set); prim_out[0..c) receives them in cull (leaf) order, bvh_out[0..2c-1) the hierarchy, with
// absolute prim slots (prim_base + k) in leaves and absolute skip pointers (bvh_base + i, -1 past
// the end).  prefix_out[4k..4k+2] = #sph/#box/#tri among Set positions 0..k (stats).
int rt_build_node_cull(const RtPrim *recs, int c, int prim_base, int bvh_base, double delta, double clampv,
                       bool sah, int leaf, RtPrim *prim_out, RtBvh *bvh_out, int32_t *prefix_out)
{
    leaf = leaf < 1 ? 1 : (leaf > 15 ? 15 : leaf);
    int cnt[3] = {0, 0, 0};
    for (int k = 0; k < c; k++) {
        cnt[recs[k].meta & 3]++;
        for (int t = 0; t < 3; t++) prefix_out[4 * (size_t)k + t] = cnt[t];
        prefix_out[4 * (size_t)k + 3] = 0;
    }
    if (c == 0) return -1;
    std::vector<Item> items(c);
    for (int k = 0; k < c; k++) {
        prim_bounds(recs[k], delta, items[k]);
        items[k].slot = k;
    }
    std::vector<RtBvh> bvh;
    bvh.reserve(2 * (size_t)c - 1);
    Builder B{&bvh, {}, &items, sah, leaf, clampv, {}};
    B.order.reserve(c);
    B.emit(0, c);
    const int end = (int)bvh.size();
    for (int i = 0; i < end; i++) {
        RtBvh n = bvh[i];
        n.skip = n.skip >= end ? -1 : n.skip + bvh_base;
        if (n.info >= 0) n.info = ((n.info >> 4) + prim_base) << 4 | (n.info & 15);
        bvh_out[i] = n;
    }
    for (int k = 0; k < c; k++) prim_out[k] = recs[items[B.order[k]].slot];
    return bvh_base;
}
