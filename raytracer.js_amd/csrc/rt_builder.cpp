// rt_builder.cpp — native scene construction behind rt_builder_* (include/rt.h).
//
// Implements the reference's add_entity_to_octree (src/octree_entity.ts:174-188) with
// get_covering_node_for_entity (:60-79), extend_tree_inside_to_fit_up_to_depth (:92-114),
// extend_tree_outside_to_fit_up_to_depth (:125-171) and Entity.set_octree (src/entity.ts:50-56)
// over an index-based node pool, then linearises the tree the way rt_upload_scene consumes it:
// DFS pre-order from the root (children 0..7), per-node entity lists in EntitySet insertion order.
// The JS host builds the same trees with the reference's own classes and serialises them to the
// identical layout (raytracer.js_amd/js/serialize.js).
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "rt.h"
#include "rt_internal.h"
#include "rt_jsnum.h"

namespace {

struct BNode {
    double pos[3];
    double size;
    int parent;
    int child[8];
    std::vector<int> set;   // EntitySet.set, insertion order
};

struct BEnt {
    int type;
    double g[9];
    int shade, substance;
    int max_in, max_out;    // AddEntityToOctreeFlags it was added with (reused by rt_builder_move)
    int owner;              // Entity._octree (-1 = none)
};

}  // namespace

struct rt_builder {
    std::vector<BNode> nodes;
    std::vector<BEnt> ents;
    int root = 0;           // the tree handed to add_entity_to_octree (the Raytracer's otree)
    // linearised output (kept alive for rt_builder_desc)
    std::vector<double> l_pos, l_size, l_geom;
    std::vector<int32_t> l_parent, l_child, l_begin, l_count, l_list, l_type, l_shade, l_sub;
    std::vector<rt_shade> l_shades;
    std::vector<double> l_ri;
    std::vector<int> l_order;          // builder node of each DFS id (the last rt_builder_desc)
    // rt_builder_sync: the store state this builder was last synced with, the device slot of every
    // node synced then, and the journal of edits since (nodes whose EntitySet or member entities
    // changed, parents that gained a child, entities whose data changed)
    const RtSceneStore *sync_store = nullptr;
    uint64_t sync_epoch = 0;
    std::vector<int32_t> slot;
    size_t synced_nodes = 0, synced_ents = 0;
    std::vector<int> j_nodes, j_child, j_ents;
    bool j_full = false;               // an edit the journal cannot express (replaced child, outward growth)
    std::vector<int32_t> sub;          // nodes in each node's subtree (DFS ids without a traversal)
    size_t unreached = 0;              // nodes the last full sync did not reach (replaced subtrees)
};

using namespace rtjs;

static int new_node(rt_builder *b, const double pos[3], double size, int parent)
{
    BNode n;
    n.pos[0] = pos[0]; n.pos[1] = pos[1]; n.pos[2] = pos[2];
    n.size = size;
    n.parent = parent;
    for (int i = 0; i < 8; i++) n.child[i] = -1;
    b->nodes.push_back(std::move(n));
    b->sub.push_back(1);
    for (int a = parent; a >= 0; a = b->nodes[a].parent) b->sub[a]++;
    return (int)b->nodes.size() - 1;
}

static int get_root(const rt_builder *b, int t)
{
    while (b->nodes[t].parent >= 0) t = b->nodes[t].parent;
    return t;
}

static int get_level(const rt_builder *b, int t)
{
    int l = 0;
    while ((t = b->nodes[t].parent) >= 0) l++;
    return l;
}

// point_in_space(..., CLOSE_OPEN) on a cube — src/space.ts:55-66
static bool point_in_cube(const double p[3], const double s[3], double size)
{
    for (int i = 0; i < 3; i++)
        if (!(p[i] >= s[i] && p[i] < s[i] + size)) return false;
    return true;
}

// aabb_in_space → space_in_space — src/space.ts:85-103
static bool aabb_in_cube(const double a[3], double asize, const double s[3], double ssize)
{
    for (int d = 0; d < 3; d++) {
        double ext_end = s[d] + ssize;
        double int_end = a[d] + asize;
        if (!(a[d] >= s[d] && int_end <= ext_end)) return false;
    }
    return true;
}

// node_at_pos — src/octree_space.ts:61-93.  1 found, 0 null, -1 Octree.get threw.
static int node_at_pos(const rt_builder *b, int octree, const double p[3], int *tree_out)
{
    const BNode &dim = b->nodes[octree];
    if (!point_in_cube(p, dim.pos, dim.size)) return 0;
    int cur = get_root(b, octree);
    double np[3] = {dim.pos[0], dim.pos[1], dim.pos[2]};
    double ns = dim.size;
    int next = cur;
    while (next >= 0) {
        double s = 2 / ns;
        int32_t ix = toint32((p[0] - np[0]) * s);
        int32_t iy = toint32((p[1] - np[1]) * s);
        int32_t iz = toint32((p[2] - np[2]) * s);
        cur = next;
        double idx = octant_sum(ix, iy, iz);
        if (!(idx >= 0 && idx <= 7)) return -1;
        next = b->nodes[cur].child[(int)idx];
        ns /= 2;
        np[0] += (double)ix * ns;
        np[1] += (double)iy * ns;
        np[2] += (double)iz * ns;
    }
    *tree_out = cur;
    return 1;
}

// Entity.get_aabb (sphere src/entities/entity_sphere.ts:90-96, box src/entities/entity_box.ts:75-82,
// face: min corner + max extent)
static void entity_aabb(const BEnt &e, double a[3], double *asize)
{
    const double *g = e.g;
    if (e.type == RT_ENT_SPHERE) {
        double d = g[3];
        for (int i = 0; i < 3; i++) a[i] = g[i] - d * 0.5;
        *asize = d;
    } else if (e.type == RT_ENT_BOX) {
        double h = g[3] / 2;
        for (int i = 0; i < 3; i++) a[i] = g[i] - h;
        *asize = g[3];
    } else {
        double ext[3];
        for (int i = 0; i < 3; i++) {
            double mn = jmin(jmin(g[i], g[3 + i]), g[6 + i]);
            double mx = jmax(jmax(g[i], g[3 + i]), g[6 + i]);
            a[i] = mn;
            ext[i] = mx - mn;
        }
        *asize = jmax(jmax(ext[0], ext[1]), ext[2]);
    }
}

static int extend_inside(rt_builder *b, int root, int node, const double a[3], double asize, int max_depth)
{
    int cur_depth = get_level(b, node) - get_level(b, root);
    int cur = node;
    while (cur_depth < max_depth) {
        const double cs = b->nodes[cur].size;
        double s = 2.0 / cs;
        int32_t xyz[3];
        double half = cs / 2;
        double sp[3];
        for (int i = 0; i < 3; i++) xyz[i] = toint32((a[i] - b->nodes[cur].pos[i]) * s);
        for (int i = 0; i < 3; i++) sp[i] = b->nodes[cur].pos[i] + (double)xyz[i] * half;
        if (!aabb_in_cube(a, asize, sp, half)) break;
        int idx = (int)(((uint32_t)xyz[2] << 2) | ((uint32_t)xyz[1] << 1) | ((uint32_t)xyz[0] << 0));
        if (!(idx >= 0 && idx <= 7)) return -1;
        int nt = new_node(b, sp, cs / 2, cur);
        if (b->nodes[cur].child[idx] >= 0) b->j_full = true;
        b->nodes[cur].child[idx] = nt;          // replaces an existing child, exactly like Octree.set
        b->j_child.push_back(cur);
        cur = nt;
        cur_depth++;
    }
    return cur;
}

static int extend_outside(rt_builder *b, int root, int node, const double a[3], double asize, int max_depth)
{
    if (b->nodes[node].parent >= 0) return -1;
    b->j_full = true;                           // a new root above the synced one
    int cur_depth = get_level(b, root) - get_level(b, node);
    int cur = node;
    while (cur_depth < max_depth) {
        const double cs = b->nodes[cur].size;
        double s = 1.0 / cs;
        double al[3], pp[3];
        for (int i = 0; i < 3; i++) {
            al[i] = (a[i] - b->nodes[cur].pos[i]) * s;
            al[i] = jmax(jmin(floor(al[i]), 0), -1);
        }
        for (int i = 0; i < 3; i++) pp[i] = b->nodes[cur].pos[i] + al[i] * cs;
        double psize = cs * 2;
        int idx = (toint32(-al[2]) << 2) | (toint32(-al[1]) << 1) | (toint32(-al[0]) << 0);
        if (!(idx >= 0 && idx <= 7)) return -1;
        int np = new_node(b, pp, psize, -1);
        b->nodes[np].child[idx] = cur;
        b->nodes[cur].parent = np;
        b->sub[np] += b->sub[cur];
        cur = np;
        if (aabb_in_cube(a, asize, pp, psize)) return cur;
        cur_depth++;
    }
    return -1;
}

// get_covering_node_for_entity + extend_tree_outside/inside (src/octree_entity.ts:60-188): the
// node add_entity_to_octree files `e` under (may grow the tree).
static int place(rt_builder *b, const BEnt &e, int *fit_out)
{
    double a[3], asize;
    entity_aabb(e, a, &asize);
    int fit = -1, deepest;
    int r = node_at_pos(b, b->root, a, &deepest);
    if (r < 0) return rt_set_error(RT_E_TREE, "add_entity_to_octree: Node index out of range (0..7)");
    if (r == 1) {
        int cur = deepest;
        do {
            if (aabb_in_cube(a, asize, b->nodes[cur].pos, b->nodes[cur].size)) break;
            cur = b->nodes[cur].parent;
        } while (cur >= 0);
        fit = cur;
    }
    if (fit < 0) {
        fit = extend_outside(b, b->root, get_root(b, b->root), a, asize, e.max_out);
        if (fit < 0) return rt_set_error(RT_E_TREE, "TreeOutsideGrowError: The tree outside-depth limit exceeded");
    }
    fit = extend_inside(b, b->root, fit, a, asize, e.max_in);
    if (fit < 0) return rt_set_error(RT_E_TREE, "add_entity_to_octree: Node index out of range (0..7)");
    *fit_out = fit;
    return RT_OK;
}

extern "C" int rt_builder_create(const double root_pos[3], double root_size, rt_builder **out)
{
    if (!root_pos || !out) return rt_set_error(RT_E_INVALID, "rt_builder_create: null argument");
    rt_builder *b = new (std::nothrow) rt_builder();
    if (!b) return rt_set_error(RT_E_INVALID, "rt_builder_create: out of memory");
    b->root = new_node(b, root_pos, root_size, -1);
    *out = b;
    return RT_OK;
}

extern "C" void rt_builder_destroy(rt_builder *b) { delete b; }

extern "C" int rt_builder_add(rt_builder *b, const rt_entity_in *in, int32_t *entity_id)
{
    if (!b || !in) return rt_set_error(RT_E_INVALID, "rt_builder_add: null argument");
    if (in->type < RT_ENT_SPHERE || in->type > RT_ENT_FACE)
        return rt_set_error(RT_E_INVALID, "rt_builder_add: bad entity type %d", in->type);
    BEnt e;
    e.type = in->type;
    for (int i = 0; i < 9; i++) e.g[i] = in->geom[i];
    if (e.type == RT_ENT_SPHERE) {
        // SphereEntity ctor (src/entities/entity_sphere.ts:34-39) + Sphere.update_cache
        // (src/math/intersection.ts:94-97)
        double d = in->geom[3];
        double radius = d / 2;
        e.g[4] = dot3(in->geom[0], in->geom[1], in->geom[2], in->geom[0], in->geom[1], in->geom[2]);
        e.g[5] = radius * radius;
        e.g[6] = d * d / 4;
        e.g[7] = 0;
        e.g[8] = 0;
    }
    e.shade = in->shade;
    e.substance = in->substance;
    e.owner = -1;

    e.max_in = in->max_in_depth;
    e.max_out = in->max_out_depth;
    int fit;
    int r = place(b, e, &fit);
    if (r != RT_OK) return r;
    int id = (int)b->ents.size();
    e.owner = fit;
    b->ents.push_back(e);
    b->nodes[fit].set.push_back(id);   // a fresh entity: Set.add appends
    b->j_nodes.push_back(fit);
    b->j_ents.push_back(id);
    if (entity_id) *entity_id = id;
    return RT_OK;
}

extern "C" int rt_builder_move(rt_builder *b, int32_t id, const double pos[3])
{
    if (!b || !pos) return rt_set_error(RT_E_INVALID, "rt_builder_move: null argument");
    if (id < 0 || id >= (int32_t)b->ents.size()) return rt_set_error(RT_E_INVALID, "rt_builder_move: entity %d", id);
    BEnt &e = b->ents[id];
    // Entity._set_pos
    if (e.type == RT_ENT_SPHERE) {
        // SphereEntity._set_pos (src/entities/entity_sphere.ts:55-61): sphere_math.pos = p runs
        // Sphere.update_cache (src/math/intersection.ts:94-97): _dot_pp anew, _radius_sq = r*r
        // (the same value as before); SphereEntity._radius_sq is untouched
        for (int i = 0; i < 3; i++) e.g[i] = pos[i];
        e.g[4] = dot3(pos[0], pos[1], pos[2], pos[0], pos[1], pos[2]);
    } else if (e.type == RT_ENT_BOX) {
        for (int i = 0; i < 3; i++) e.g[i] = pos[i];   // BasicEntity._set_pos (src/entities/entity_basic.ts:38-42)
    } else {
        // FaceEntity._set_pos (raytracer.js_amd/js/raytracer.js): translate so the centroid lands on pos
        double d[3];
        for (int i = 0; i < 3; i++) d[i] = pos[i] - (e.g[i] + e.g[3 + i] + e.g[6 + i]) / 3;
        for (int v = 0; v < 3; v++)
            for (int i = 0; i < 3; i++) e.g[3 * v + i] += d[i];
    }
    // add_entity_to_octree(root, entity, flags) -> Entity.set_octree(fitting): Set.delete + Set.add
    int fit;
    int r = place(b, e, &fit);
    if (r != RT_OK) return r;
    BEnt &m = b->ents[id];
    if (m.owner >= 0) {
        std::vector<int> &set = b->nodes[m.owner].set;
        set.erase(std::find(set.begin(), set.end(), id));
        b->j_nodes.push_back(m.owner);
    }
    m.owner = fit;
    b->nodes[fit].set.push_back(id);
    b->j_nodes.push_back(fit);
    b->j_ents.push_back(id);
    return RT_OK;
}

extern "C" int rt_builder_set_shade(rt_builder *b, int32_t id, int32_t shade, int32_t substance)
{
    if (!b) return rt_set_error(RT_E_INVALID, "rt_builder_set_shade: null argument");
    if (id < 0 || id >= (int32_t)b->ents.size()) return rt_set_error(RT_E_INVALID, "rt_builder_set_shade: entity %d", id);
    b->ents[id].shade = shade;
    b->ents[id].substance = substance;
    if (b->ents[id].owner >= 0) b->j_nodes.push_back(b->ents[id].owner);   // its prim record carries the shade
    b->j_ents.push_back(id);
    return RT_OK;
}

extern "C" int rt_builder_add_many(rt_builder *b, const rt_entity_in *in, int32_t n)
{
    for (int32_t i = 0; i < n; i++) {
        int r = rt_builder_add(b, in + i, nullptr);
        if (r != RT_OK) return r;
    }
    return RT_OK;
}

extern "C" int rt_builder_desc(rt_builder *b, const rt_shade *shades, int32_t n_shades,
                               const double *substance_ri, int32_t n_substances, rt_scene_desc *out)
{
    if (!b || !out) return rt_set_error(RT_E_INVALID, "rt_builder_desc: null argument");
    if (b->nodes[b->root].parent >= 0)
        return rt_set_error(RT_E_UNSUPPORTED,
                            "rt_builder_desc: the octree grew outward above the Raytracer's root");
    // DFS pre-order numbering with an explicit stack (children 0..7)
    std::vector<int> order;
    std::vector<int> id_of(b->nodes.size(), -1);
    std::vector<int> stack{b->root};
    while (!stack.empty()) {
        int t = stack.back();
        stack.pop_back();
        id_of[t] = (int)order.size();
        order.push_back(t);
        for (int c = 7; c >= 0; c--)
            if (b->nodes[t].child[c] >= 0) stack.push_back(b->nodes[t].child[c]);
    }
    const size_t n = order.size();
    b->l_order = order;
    b->l_pos.assign(3 * n, 0);
    b->l_size.assign(n, 0);
    b->l_parent.assign(n, -1);
    b->l_child.assign(8 * n, -1);
    b->l_begin.assign(n, 0);
    b->l_count.assign(n, 0);
    b->l_list.clear();
    for (size_t k = 0; k < n; k++) {
        const BNode &nd = b->nodes[order[k]];
        for (int i = 0; i < 3; i++) b->l_pos[3 * k + i] = nd.pos[i];
        b->l_size[k] = nd.size;
        b->l_parent[k] = nd.parent >= 0 && order[k] != b->root ? id_of[nd.parent] : -1;
        for (int c = 0; c < 8; c++) b->l_child[8 * k + c] = nd.child[c] >= 0 ? id_of[nd.child[c]] : -1;
        b->l_begin[k] = (int32_t)b->l_list.size();
        b->l_count[k] = (int32_t)nd.set.size();
        for (int e : nd.set) b->l_list.push_back(e);
    }
    const size_t ne = b->ents.size();
    b->l_type.resize(ne);
    b->l_shade.resize(ne);
    b->l_sub.resize(ne);
    b->l_geom.resize(9 * ne);
    for (size_t i = 0; i < ne; i++) {
        b->l_type[i] = b->ents[i].type;
        b->l_shade[i] = b->ents[i].shade;
        b->l_sub[i] = b->ents[i].substance;
        memcpy(&b->l_geom[9 * i], b->ents[i].g, 9 * sizeof(double));
    }
    b->l_shades.assign(shades, shades + (n_shades > 0 ? n_shades : 0));
    b->l_ri.assign(substance_ri, substance_ri + (n_substances > 0 ? n_substances : 0));
    memset(out, 0, sizeof(*out));
    out->n_nodes = (int32_t)n;
    out->n_list = (int32_t)b->l_list.size();
    out->n_entities = (int32_t)ne;
    out->n_shades = n_shades;
    out->n_substances = n_substances;
    out->node_pos = b->l_pos.data();
    out->node_size = b->l_size.data();
    out->node_parent = b->l_parent.data();
    out->node_child = b->l_child.data();
    out->node_ent_begin = b->l_begin.data();
    out->node_ent_count = b->l_count.data();
    out->list_entity = b->l_list.data();
    out->ent_type = b->l_type.data();
    out->ent_geom = b->l_geom.data();
    out->ent_shade = b->l_shade.data();
    out->ent_substance = b->l_sub.data();
    out->shades = b->l_shades.data();
    out->substance_ri = b->l_ri.data();
    return RT_OK;
}

// ---- rt_builder_sync (rt_api.hip) --------------------------------------------------------------------
// index_within_parent (src/octree_space.ts:113-125) of node n, as check_node computes it.
static int32_t octant_in_parent(const rt_builder *b, int n)
{
    const int p = b->nodes[n].parent;
    if (p < 0) return RT_OCT_UNDEF;
    const double sc = 2 / b->nodes[p].size;
    const int32_t ix = toint32((b->nodes[n].pos[0] - b->nodes[p].pos[0]) * sc);
    const int32_t iy = toint32((b->nodes[n].pos[1] - b->nodes[p].pos[1]) * sc);
    const int32_t iz = toint32((b->nodes[n].pos[2] - b->nodes[p].pos[2]) * sc);
    const double idx = octant_sum(ix, iy, iz);
    return (idx >= 0 && idx <= 7) ? (int32_t)idx : RT_OCT_BAD;
}

static bool rough_mirror(const rt_shade &sh)
{
    return !sh.light && sh.response == RT_RESP_REFLECTION && sh.mirror && sh.roughness > 0.0;
}

int rt_builder_edit(rt_builder *b, const RtSceneStore *st, uint64_t epoch, const rt_shade *shades, int32_t n_shades,
                    RtEdit &e)
{
    if (b->sync_store != st || b->sync_epoch != epoch || b->j_full || b->nodes[b->root].parent >= 0) return 1;
    const int N = (int)b->nodes.size();
    const int n_old = (int)b->synced_nodes;
    // new nodes take the next slots in creation order; every node is reachable (no child was replaced)
    if (b->unreached) return 1;                  // a node the last full sync did not reach
    b->slot.resize(N);
    for (int n = n_old; n < N; n++) b->slot[n] = n;
    e = RtEdit{};
    e.n_slots = N;
    e.n_entities = (int32_t)b->ents.size();
    // node records: new nodes and the old parents that gained a child
    std::vector<int> rec(b->j_child.begin(), b->j_child.end());
    for (int n = n_old; n < N; n++) rec.push_back(n);
    std::sort(rec.begin(), rec.end(), [&](int x, int y) { return b->slot[x] < b->slot[y]; });
    rec.erase(std::unique(rec.begin(), rec.end()), rec.end());
    for (int n : rec) {
        const BNode &nd = b->nodes[n];
        e.rec_slot.push_back(b->slot[n]);
        for (int i = 0; i < 3; i++) e.rec_cube.push_back(nd.pos[i]);
        e.rec_cube.push_back(nd.size);
        for (int c = 0; c < 8; c++) e.rec_child.push_back(nd.child[c] >= 0 ? b->slot[nd.child[c]] : -1);
        e.rec_up.push_back(n == b->root || nd.parent < 0 ? -1 : b->slot[nd.parent]);
        e.rec_up.push_back(n == b->root ? RT_OCT_UNDEF : octant_in_parent(b, n));
    }
    // dirty EntitySets: journaled nodes and every new node
    std::vector<int> dirty(b->j_nodes.begin(), b->j_nodes.end());
    for (int n = n_old; n < N; n++) dirty.push_back(n);
    std::sort(dirty.begin(), dirty.end(), [&](int x, int y) { return b->slot[x] < b->slot[y]; });
    dirty.erase(std::unique(dirty.begin(), dirty.end()), dirty.end());
    for (int n : dirty) {
        const std::vector<int> &set = b->nodes[n].set;
        e.set_slot.push_back(b->slot[n]);
        e.set_begin.push_back((int32_t)e.set_ent.size());
        e.set_count.push_back((int32_t)set.size());
        for (int id : set) {
            const BEnt &x = b->ents[id];
            if (x.shade < 0 || x.shade >= n_shades)
                return rt_set_error(RT_E_INVALID, "rt_builder_sync: entity %d shade %d (%d shades)", id, x.shade, n_shades);
            e.set_ent.push_back(id);
            e.set_type.push_back(x.type);
            e.set_shade.push_back(x.shade);
            e.set_geom.insert(e.set_geom.end(), x.g, x.g + 9);
        }
    }
    // substances of the edited and the new entities
    std::vector<int> ents(b->j_ents.begin(), b->j_ents.end());
    for (size_t i = b->synced_ents; i < b->ents.size(); i++) ents.push_back((int)i);
    std::sort(ents.begin(), ents.end());
    ents.erase(std::unique(ents.begin(), ents.end()), ents.end());
    for (int id : ents) {
        e.sub_ent.push_back(id);
        e.sub_val.push_back(b->ents[id].substance);
    }
    // DFS numbering (the node ids the outputs report) changes only when nodes were created: each new
    // node's id from the subtree sizes along its path (O(depth)), and for the existing nodes the
    // shift G (an old id a becomes a + #{j : G_j <= a}, G_j = F_j - j over the new ids F, ascending),
    // applied on the device
    if (N > n_old) {
        std::vector<int32_t> F;
        for (int n = n_old; n < N; n++) {
            int32_t id = 0;
            for (int x = n; x != b->root;) {
                const int p = b->nodes[x].parent;
                id += 1;
                for (int c = 0; c < 8 && b->nodes[p].child[c] != x; c++)
                    if (b->nodes[p].child[c] >= 0) id += b->sub[b->nodes[p].child[c]];
                x = p;
            }
            e.dfs_new_slot.push_back(b->slot[n]);
            e.dfs_new_val.push_back(id);
            F.push_back(id);
        }
        std::sort(F.begin(), F.end());
        for (size_t j = 0; j < F.size(); j++) e.dfs_shift.push_back(F[j] - (int32_t)j);
    }
    // a rough mirror is listed: only scenes whose shade table has one pay the entity scan
    bool any = false;
    for (int i = 0; i < n_shades; i++) any = any || rough_mirror(shades[i]);
    for (size_t i = 0; any && !e.scatter && i < b->ents.size(); i++)
        e.scatter = b->ents[i].owner >= 0 && b->ents[i].shade >= 0 && b->ents[i].shade < n_shades &&
                    rough_mirror(shades[b->ents[i].shade]);
    return 0;
}

void rt_builder_synced(rt_builder *b, const RtSceneStore *st, uint64_t epoch, bool full, const int32_t *order)
{
    if (full) {                                  // the full upload's slot of each DFS id (DFS order by default)
        b->slot.assign(b->nodes.size(), -1);
        for (size_t k = 0; k < b->l_order.size(); k++) b->slot[b->l_order[k]] = order ? order[k] : (int32_t)k;
        b->unreached = b->nodes.size() - b->l_order.size();
        // subtree sizes of the reachable tree (a replaced child leaves its old subtree counted)
        b->sub.assign(b->nodes.size(), 0);
        for (size_t k = b->l_order.size(); k-- > 0;) {
            const int n = b->l_order[k];
            b->sub[n] += 1;
            if (n != b->root && b->nodes[n].parent >= 0) b->sub[b->nodes[n].parent] += b->sub[n];
        }
    }
    b->synced_nodes = b->nodes.size();
    b->synced_ents = b->ents.size();
    b->j_nodes.clear();
    b->j_child.clear();
    b->j_ents.clear();
    b->j_full = false;
    b->sync_store = st;
    b->sync_epoch = epoch;
}
