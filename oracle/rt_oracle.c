/*
 * rt_oracle.c — CPU restatement of the raytracer.js render path (TEST INFRASTRUCTURE ONLY).
 *
 * See rt_oracle.h for scope and pinning.  This file deliberately mirrors the reference's own
 * object model (pointer octree with parent links, stateful OctreeWalker, insertion-ordered
 * EntitySet) so each function can be read side by side with the TypeScript it restates.
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math (oracle/Makefile).
 */
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ============================ JS number helpers ============================================ */

/* ToInt32 (ECMA-262 7.1.6), used by `x << k`, `x | y`, `x << 0` in the reference. */
static int32_t js_toint32(double x)
{
    if (!isfinite(x)) return 0;
    if (fabs(x) < 2147483648.0) return (int32_t)x;            /* truncation toward zero */
    double t = trunc(x);
    double m = fmod(t, 4294967296.0);
    if (m < 0) m += 4294967296.0;
    uint32_t u = (uint32_t)m;
    return (int32_t)u;
}

/* isNegative, src/math/mathutils.ts:45-47: x < 0 || Object.is(x, -0) */
static int js_is_negative(double x) { return x < 0 || (x == 0 && signbit(x)); }

/* Math.sign */
static double js_sign(double x)
{
    if (isnan(x)) return x;
    if (x > 0) return 1.0;
    if (x < 0) return -1.0;
    return x;                                                 /* keeps the sign of zero */
}

/* Math.min / Math.max (NaN-propagating, -0 < +0) */
static double js_min(double a, double b)
{
    if (isnan(a) || isnan(b)) return NAN;
    if (a < b) return a;
    if (b < a) return b;
    return signbit(a) ? a : b;
}
static double js_max(double a, double b)
{
    if (isnan(a) || isnan(b)) return NAN;
    if (a > b) return a;
    if (b > a) return b;
    return signbit(a) ? b : a;
}

/* vector.dot, src/math/vector.ts:78-86: sum starts at +0 and accumulates left to right */
static double vdot(const double *a, const double *b)
{
    double s = 0;
    s += a[0] * b[0];
    s += a[1] * b[1];
    s += a[2] * b[2];
    return s;
}

/* ============================ arena ========================================================= */

struct onode {
    double pos[3];
    double size;
    onode *parent;
    onode *child[8];
    int has_set;          /* value is an EntitySet (entity octree); KAT trees carry no value */
    int *set;             /* entity ids in Set insertion order */
    int set_n, set_cap;
    int dfs_id;
    onode *next_alloc;
    /* shadow rays (build extension): the geometry bounds of every entity at or below this node, and
     * their count (0: none); filled by shadow_bounds before a frame with lights */
    double sb_lo[3], sb_hi[3];
    int64_t sb_n;
};

typedef struct oentity {
    int type;
    double g[9];          /* rt.h rt_scene_desc.ent_geom layout (sphere caches derived) */
    int shade;
    int substance;
    onode *octree;        /* Entity._octree (src/entity.ts:43) */
} oentity;

struct owalker {
    onode *tree;          /* OctreeWalker.tree */
    int include_undefined;
    double pos[3];        /* this.pos */
    double dir[3];        /* this.direction */
    int has_pos;
    onode *cur_tree;      /* cur_node.tree (NULL: cur_node undefined) */
    int cur_oct;          /* cur_node.octant (ORC_OCT_UNDEF: undefined) */
    double np[3];         /* next_pos[0] */
    double nn[3];         /* next_pos[1] */
    int nn_valid;         /* next_pos[1] !== undefined */
    int cur_returned, stepped_in, depth, ahead;
    owalker *next_alloc;
    /* work counters of the owning trace (see rt_stats) */
    int64_t c_ret, c_slot, c_loc;
};

struct oworld {
    onode *nodes;
    owalker *walkers;
    oentity *ents;
    int n_ents, cap_ents;
    rt_shade *shades;
    int n_shades;
    double *ri;
    int n_ri;
    rt_image_desc *images;   /* ImageTextures (each rgb a private copy) */
    int n_images;
    int n_lights;            /* shadow rays (build extension, orc_set_lights): 0 = the reference */
    double ambient;
    rt_light lights[RT_MAX_LIGHTS];
    int shadow_brute;        /* orc_set_shadow_brute: test every entity (pins the bounded search) */
};

oworld *orc_world_new(void)
{
    return (oworld *)calloc(1, sizeof(oworld));
}

void orc_world_free(oworld *w)
{
    if (!w) return;
    for (onode *n = w->nodes; n;) { onode *nx = n->next_alloc; free(n->set); free(n); n = nx; }
    for (owalker *k = w->walkers; k;) { owalker *nx = k->next_alloc; free(k); k = nx; }
    free(w->ents);
    free(w->shades);
    free(w->ri);
    for (int i = 0; i < w->n_images; i++) free((void *)w->images[i].rgb);
    free(w->images);
    free(w);
}

/* new Octree(id, parent, value) — src/octree.ts:33-39 */
static onode *node_alloc(oworld *w, const double pos[3], double size, onode *parent, int with_set)
{
    onode *n = (onode *)calloc(1, sizeof(onode));
    n->pos[0] = pos[0]; n->pos[1] = pos[1]; n->pos[2] = pos[2];
    n->size = size;
    n->parent = parent;
    n->has_set = with_set;
    n->dfs_id = -1;
    n->next_alloc = w->nodes;
    w->nodes = n;
    return n;
}

onode *orc_tree_new(oworld *w, const double pos[3], double size, int with_entity_set)
{
    return node_alloc(w, pos, size, NULL, with_entity_set);
}

onode *orc_tree_parent(onode *t) { return t->parent; }

int orc_tree_id(onode *t) { return t ? t->dfs_id : -1; }   /* DFS id from the last linearisation */

void orc_tree_dims(onode *t, double pos[3], double *size)
{
    pos[0] = t->pos[0]; pos[1] = t->pos[1]; pos[2] = t->pos[2];
    *size = t->size;
}

/* Octree.get / check_bounds — src/octree.ts:41-54 */
int orc_tree_get(onode *t, int n, onode **out)
{
    if (!(n >= 0 && n <= 7)) return ORC_FAULT;                 /* "Node index out of range (0..7)" */
    *out = t->child[n];
    return 0;
}

/* Octree.get_root — src/octree.ts:101-110 */
static onode *get_root(onode *t)
{
    onode *cur = t;
    while (cur->parent) cur = cur->parent;
    return cur;
}

/* Octree.get_level — src/octree.ts:113-120 */
static int get_level(onode *t)
{
    int l = 0;
    while ((t = t->parent) != NULL) l++;
    return l;
}

/* ============================ space (src/space.ts) ========================================= */

/* point_in_space(point, {pos, size*[1,1,1]}, CLOSE_OPEN) — src/space.ts:55-66 */
static int point_in_cube_co(const double p[3], const double spos[3], double ssize)
{
    for (int i = 0; i < 3; i++)
        if (!(p[i] >= spos[i] && p[i] < spos[i] + ssize)) return 0;
    return 1;
}

/* aabb_in_space → space_in_space — src/space.ts:85-103.  The interior size vector is
 * scale([1,1,1], aabb.size) and the exterior one scale([1,1,1], size): 1*x == x exactly. */
static int aabb_in_cube(const double apos[3], double asize, const double spos[3], double ssize)
{
    for (int d = 0; d < 3; d++) {
        double ext_end = spos[d] + ssize;
        double int_end = apos[d] + asize;
        if (!(apos[d] >= spos[d] && int_end <= ext_end)) return 0;
    }
    return 1;
}

/* ============================ octree_space.ts ============================================== */

/* octant_adj_pos — src/octree_space.ts:41-50 */
static int octant_adj_pos(const onode *t, const double p[3])
{
    double h = t->size / 2;
    int px = p[0] >= t->pos[0] + h;
    int py = p[1] >= t->pos[1] + h;
    int pz = p[2] >= t->pos[2] + h;
    return (pz << 2) | (py << 1) | px;
}

/* node_at_pos(octree, pos, {}, CLOSE_OPEN) — src/octree_space.ts:61-93.
 * Returns 1 with (tree, octant), 0 for null, ORC_FAULT when Octree.get throws.
 * `levels` (nullable) counts loop iterations (descent levels). */
static int node_at_pos_c(onode *octree, const double p[3], onode **tree_out, int *oct_out, int64_t *levels)
{
    const onode *dim = octree;
    onode *cur = get_root(octree);
    if (!point_in_cube_co(p, dim->pos, dim->size)) return 0;
    int cur_index = 0;
    double npos[3] = {dim->pos[0], dim->pos[1], dim->pos[2]};
    double nsize = dim->size;
    onode *next = cur;
    while (next != NULL) {
        if (levels) (*levels)++;
        double s = 2 / nsize;
        double ind[3];
        for (int i = 0; i < 3; i++) ind[i] = (p[i] - npos[i]) * s;
        cur = next;
        int32_t i0 = js_toint32(ind[0]), i1 = js_toint32(ind[1]), i2 = js_toint32(ind[2]);
        /* (ind2 << 2) + (ind1 << 1) + (ind0 << 0): int32 shifts, then Number addition */
        double idx = (double)(int32_t)((uint32_t)i2 << 2) + (double)(int32_t)((uint32_t)i1 << 1) + (double)i0;
        if (!(idx >= 0 && idx <= 7)) return ORC_FAULT;
        cur_index = (int)idx;
        next = cur->child[cur_index];
        nsize /= 2;
        npos[0] += (double)i0 * nsize;
        npos[1] += (double)i1 * nsize;
        npos[2] += (double)i2 * nsize;
    }
    *tree_out = cur;
    *oct_out = cur_index;
    return 1;
}

int orc_node_at_pos(onode *t, const double p[3], onode **tree, int *octant)
{
    return node_at_pos_c(t, p, tree, octant, NULL);
}

/* new_subtree — src/octree_space.ts:95-108 (allow_replace false) */
int orc_new_subtree(oworld *w, onode *t, int n, onode **out)
{
    if (!(n >= 0 && n <= 7)) return ORC_FAULT;
    if (t->child[n] != NULL) return ORC_FAULT;                 /* "Child already defined" */
    double half = t->size / 2;
    double bits[3] = {(double)(n & 1), (double)((n >> 1) & 1), (double)((n >> 2) & 1)};
    double pos[3];
    for (int i = 0; i < 3; i++) pos[i] = t->pos[i] + bits[i] * half;
    onode *c = node_alloc(w, pos, half, t, t->has_set);
    t->child[n] = c;
    *out = c;
    return 0;
}

/* index_within_parent — src/octree_space.ts:113-125 (Octree.index_within_parent is never
 * assigned, src/octree.ts:27, so the geometric branch always runs).  *has = 0 for null. */
static double index_within_parent_d(const onode *c, int *has)
{
    const onode *p = c->parent;
    if (!p) { *has = 0; return 0; }
    *has = 1;
    double s = 2 / p->size;
    double ind[3];
    for (int i = 0; i < 3; i++) ind[i] = (c->pos[i] - p->pos[i]) * s;
    int32_t i0 = js_toint32(ind[0]), i1 = js_toint32(ind[1]), i2 = js_toint32(ind[2]);
    return (double)(int32_t)((uint32_t)i2 << 2) + (double)(int32_t)((uint32_t)i1 << 1) + (double)i0;
}

int orc_index_within_parent(onode *t, int *has)
{
    double v = index_within_parent_d(t, has);
    return (int)v;
}

/* ============================ math/intersection.ts ========================================= */

static const double FACE_NORMALS[6][3] = {      /* Box.FACE_NORMALS, src/math/intersection.ts:141-148 */
    {-1, 0, 0}, {1, 0, 0}, {0, -1, 0}, {0, 1, 0}, {0, 0, -1}, {0, 0, 1}};

/* Box.line_intersection — src/math/intersection.ts:150-204.
 * Returns 0 for [] (u1 > u2), else 1 with (u1, i1) entering and (u2, i2) exiting; i = -1 when
 * the face index stayed undefined. */
static int box_line_intersection(const double center[3], const double bsize[3], const double o[3],
                                 const double d[3], double *u1o, int *i1o, double *u2o, int *i2o)
{
    double tl[3];
    for (int i = 0; i < 3; i++) tl[i] = center[i] - bsize[i] * 0.5;
    double p[6] = {-d[0], d[0], -d[1], d[1], -d[2], d[2]};
    double q[6] = {o[0] - tl[0], tl[0] + bsize[0] - o[0],
                   o[1] - tl[1], tl[1] + bsize[1] - o[1],
                   o[2] - tl[2], tl[2] + bsize[2] - o[2]};
    double u1 = -INFINITY, u2 = INFINITY;
    int i1 = -1, i2 = -1;
    for (int i = 0; i < 6; i++) {
        double e = p[i];
        double u = q[i] / e;
        if (js_is_negative(e)) {
            if (u > u1) { u1 = u; i1 = i; }
        } else {
            if (u < u2) { u2 = u; i2 = i; }
        }
    }
    if (u1 > u2) return 0;
    *u1o = u1; *i1o = i1; *u2o = u2; *i2o = i2;
    return 1;
}

/* ============================ walker (src/octree_space.ts:159-408) ======================== */

owalker *orc_walker_new(oworld *w, onode *tree, int include_undefined)
{
    owalker *k = (owalker *)calloc(1, sizeof(owalker));
    k->tree = tree;
    k->include_undefined = include_undefined;
    k->cur_oct = ORC_OCT_UNDEF;
    k->next_alloc = w->walkers;
    w->walkers = k;
    return k;
}

/* reset_state — :240-246 */
static void walker_reset(owalker *k)
{
    k->np[0] = k->pos[0]; k->np[1] = k->pos[1]; k->np[2] = k->pos[2];
    k->nn_valid = 0;
    k->cur_returned = 0;
    k->stepped_in = 0;
    k->ahead = 0;
    k->depth = 0;
}

/* setup_cur_node — :251-278.  Returns 1 (true), 0 (false) or ORC_FAULT. */
static int walker_setup_cur_node(owalker *k)
{
    walker_reset(k);
    if (k->cur_tree != NULL) return 1;
    const onode *dim = k->tree;
    double center[3], bsize[3];
    for (int i = 0; i < 3; i++) {
        center[i] = dim->pos[i] + 0.5 * dim->size;
        bsize[i] = 1 * dim->size;
    }
    double u1, u2;
    int i1, i2;
    if (!box_line_intersection(center, bsize, k->pos, k->dir, &u1, &i1, &u2, &i2)) return 0;
    /* select_parameters(FORWARD): keep parameter >= 0, in order [u1, u2] */
    double t;
    int fi;
    if (u1 >= 0) { t = u1; fi = i1; }
    else if (u2 >= 0) { t = u2; fi = i2; }
    else return 0;
    double ip[3];
    for (int i = 0; i < 3; i++) ip[i] = k->pos[i] + k->dir[i] * t;
    if (fi < 0) return ORC_FAULT;                              /* vector.negate(undefined) throws */
    k->cur_tree = k->tree;
    k->cur_oct = ORC_OCT_UNDEF;
    for (int i = 0; i < 3; i++) { k->np[i] = ip[i]; k->nn[i] = -FACE_NORMALS[fi][i]; }
    k->nn_valid = 1;
    return 1;
}

/* set_position — :188-205 (pos always defined here); node_tree == NULL → node_at_pos. */
static int walker_set_position(owalker *k, const double pos[3], onode *node_tree, int node_oct)
{
    if (node_tree != NULL) {
        k->cur_tree = node_tree;
        k->cur_oct = node_oct;
    } else {
        onode *t = NULL;
        int oc = 0;
        int r = node_at_pos_c(k->tree, pos, &t, &oc, &k->c_loc);
        if (r < 0) return ORC_FAULT;
        if (r == 1) { k->cur_tree = t; k->cur_oct = oc; }
        else { k->cur_tree = NULL; k->cur_oct = ORC_OCT_UNDEF; }
    }
    k->pos[0] = pos[0]; k->pos[1] = pos[1]; k->pos[2] = pos[2];
    k->has_pos = 1;
    return walker_setup_cur_node(k);
}

/* set_pos_and_dir — :223-226 */
int orc_walker_set(owalker *k, const double pos[3], const double dir[3], onode *node_tree, int node_octant)
{
    k->dir[0] = dir[0]; k->dir[1] = dir[1]; k->dir[2] = dir[2];
    int r = walker_set_position(k, pos, node_tree, node_octant);
    return r < 0 ? r : 0;
}

/* step_back — :280-308 */
static void walker_step_back(owalker *k)
{
    k->stepped_in = 1;
    if (k->cur_oct == ORC_OCT_UNDEF) {
        k->cur_tree = NULL;
        k->cur_returned = 0;
        return;
    }
    if (k->depth > 0) { k->depth--; k->cur_returned = 1; }
    else k->cur_returned = 0;
    int has;
    double gp = index_within_parent_d(k->cur_tree, &has);
    if (has) {
        k->cur_tree = k->cur_tree->parent;
        /* a non-integral or out-of-range value throws at the next Octree.get */
        k->cur_oct = (gp >= 0 && gp <= 7) ? (int)gp : 1000;
    } else {
        k->cur_oct = ORC_OCT_UNDEF;
    }
}

/* update_next_pos — :369-384 (dim_relative_to_parent :127-136) */
static int walker_update_next_pos(owalker *k)
{
    k->c_slot++;
    const onode *pt = k->cur_tree;
    int n = k->cur_oct;
    double phsize = pt->size / 2;
    double bits[3] = {(double)((n >> 0) & 1), (double)((n >> 1) & 1), (double)((n >> 2) & 1)};
    double dpos[3], center[3], bsize[3];
    for (int i = 0; i < 3; i++) {
        dpos[i] = pt->pos[i] + bits[i] * phsize;
        center[i] = dpos[i] + 0.5 * phsize;
        bsize[i] = 1 * phsize;
    }
    double u1, u2;
    int i1, i2;
    if (!box_line_intersection(center, bsize, k->pos, k->dir, &u1, &i1, &u2, &i2))
        return ORC_FAULT;                                      /* [].pop() → undefined → throws */
    for (int i = 0; i < 3; i++) k->np[i] = k->pos[i] + k->dir[i] * u2;
    if (i2 < 0) { k->nn_valid = 0; }
    else { for (int i = 0; i < 3; i++) k->nn[i] = FACE_NORMALS[i2][i]; k->nn_valid = 1; }
    return 0;
}

/* next — :316-361 */
int orc_walker_next(owalker *k, onode **node, onode **pos_tree, int *pos_octant)
{
    while (k->cur_tree != NULL) {
        onode *ltree = k->cur_tree;
        int loct = k->cur_oct;
        onode *lnode;
        if (loct != ORC_OCT_UNDEF) {
            if (orc_tree_get(ltree, loct, &lnode) < 0) return ORC_FAULT;
        } else {
            lnode = ltree;
        }
        if (!k->cur_returned) {
            if (k->include_undefined || lnode != NULL) {
                k->cur_returned = 1;
                *node = lnode;
                *pos_tree = ltree;
                *pos_octant = loct;
                k->c_ret++;
                return 1;
            }
        }
        if (loct != ORC_OCT_UNDEF) {
            if (!k->ahead) {
                if (!k->stepped_in && lnode != NULL) {
                    int n = octant_adj_pos(lnode, k->np);
                    /* step_in — :310-314 */
                    k->depth++;
                    k->cur_tree = lnode;
                    k->cur_oct = n;
                    k->cur_returned = 0;
                    continue;
                }
                if (walker_update_next_pos(k) < 0) return ORC_FAULT;
            }
            if (!k->nn_valid) return ORC_FAULT;                /* vector.add(v, undefined) throws */
            double c[3] = {(double)(loct & 1), (double)((loct >> 1) & 1), (double)((loct >> 2) & 1)};
            double nx = c[0] + k->nn[0], ny = c[1] + k->nn[1], nz = c[2] + k->nn[2];
            if (!(nx < 0 || nx > 1 || ny < 0 || ny > 1 || nz < 0 || nz > 1)) {
                k->cur_oct = js_toint32(nx) | (js_toint32(ny) << 1) | (js_toint32(nz) << 2);
                k->cur_returned = 0;
                k->stepped_in = 0;
                k->ahead = 0;
                continue;
            } else {
                k->ahead = 1;
            }
        }
        walker_step_back(k);
    }
    return 0;
}

/* ============================ entities ===================================================== */

int orc_set_tables(oworld *w, const rt_shade *shades, int n_shades, const double *ri, int n_ri)
{
    free(w->shades);
    free(w->ri);
    w->shades = (rt_shade *)malloc(sizeof(rt_shade) * (size_t)(n_shades > 0 ? n_shades : 1));
    w->ri = (double *)malloc(sizeof(double) * (size_t)(n_ri > 0 ? n_ri : 1));
    if (n_shades) memcpy(w->shades, shades, sizeof(rt_shade) * (size_t)n_shades);
    if (n_ri) memcpy(w->ri, ri, sizeof(double) * (size_t)n_ri);
    w->n_shades = n_shades;
    w->n_ri = n_ri;
    return 0;
}

/* Loaded ImageTextures (rt_image_desc: the canvas bytes behind image_data, which holds them / 255.0) */
int orc_set_images(oworld *w, const rt_image_desc *images, int n)
{
    for (int i = 0; i < w->n_images; i++) free((void *)w->images[i].rgb);
    free(w->images);
    w->images = (rt_image_desc *)calloc((size_t)(n > 0 ? n : 1), sizeof(rt_image_desc));
    for (int i = 0; i < n; i++) {
        size_t b = (size_t)images[i].width * (size_t)images[i].height * 3;
        uint8_t *px = (uint8_t *)malloc(b ? b : 1);
        memcpy(px, images[i].rgb, b);
        w->images[i].width = images[i].width;
        w->images[i].height = images[i].height;
        w->images[i].rgb = px;
    }
    w->n_images = n;
    return 0;
}

/* ---- Math.atan / Math.atan2 (V8 = fdlibm s_atan.c / e_atan2.c), needed bit-exact by
 * uv_map_sphere (src/math/uv_mapping.ts:19-25).  Pinned against node (tests/golden). */
static uint32_t orc_hi(double x) { uint64_t b; memcpy(&b, &x, 8); return (uint32_t)(b >> 32); }
static uint32_t orc_lo(double x) { uint64_t b; memcpy(&b, &x, 8); return (uint32_t)b; }

static const double ATANHI[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                 9.82793723247329054082e-01, 1.57079632679489655800e+00};
static const double ATANLO[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                 1.39033110312309984516e-17, 6.12323399573676603587e-17};
static const double AT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                              1.42857142725034663711e-01, -1.11111104054623557880e-01,
                              9.09088713343650656196e-02, -7.69187620504482999495e-02,
                              6.66107313738753120669e-02, -5.83357013379057348645e-02,
                              4.97687799461593236017e-02, -3.65315727442169155270e-02,
                              1.62858201153657823623e-02};

double orc_atan(double x)
{
    int32_t hx = (int32_t)orc_hi(x);
    uint32_t ix = (uint32_t)hx & 0x7fffffffu;
    int id;
    if (ix >= 0x44100000u) {
        if (ix > 0x7ff00000u || (ix == 0x7ff00000u && orc_lo(x) != 0)) return x + x;
        return hx > 0 ? ATANHI[3] + ATANLO[3] : -ATANHI[3] - ATANLO[3];
    }
    if (ix < 0x3fdc0000u) {
        if (ix < 0x3e400000u) return x;
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000u) {
            if (ix < 0x3fe60000u) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
            else { id = 1; x = (x - 1.0) / (x + 1.0); }
        } else if (ix < 0x40038000u) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
        else { id = 3; x = -1.0 / x; }
    }
    double z = x * x, w = z * z;
    double s1 = z * (AT[0] + w * (AT[2] + w * (AT[4] + w * (AT[6] + w * (AT[8] + w * AT[10])))));
    double s2 = w * (AT[1] + w * (AT[3] + w * (AT[5] + w * (AT[7] + w * AT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = ATANHI[id] - ((x * (s1 + s2) - ATANLO[id]) - x);
    return hx < 0 ? -z : z;
}

double orc_atan2(double y, double x)
{
    const double tiny = 1.0e-300, pi_o_4 = 7.8539816339744827900e-01, pi_o_2 = 1.5707963267948965580e+00;
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    int32_t hx = (int32_t)orc_hi(x), hy = (int32_t)orc_hi(y);
    uint32_t ix = (uint32_t)hx & 0x7fffffffu, iy = (uint32_t)hy & 0x7fffffffu;
    uint32_t lx = orc_lo(x), ly = orc_lo(y);
    if ((ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u || (iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u) return x + y;
    if ((((uint32_t)hx - 0x3ff00000u) | lx) == 0) return orc_atan(y);
    int m = (int)(((uint32_t)hy >> 31) & 1u) | (int)(((uint32_t)hx >> 30) & 2u);
    if ((iy | ly) == 0) {
        if (m < 2) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if ((ix | lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7ff00000u) {
        if (iy == 0x7ff00000u) {
            if (m == 0) return pi_o_4 + tiny;
            if (m == 1) return -pi_o_4 - tiny;
            if (m == 2) return 3.0 * pi_o_4 + tiny;
            return -3.0 * pi_o_4 - tiny;
        }
        if (m == 0) return 0.0;
        if (m == 1) return -0.0;
        if (m == 2) return pi + tiny;
        return -pi - tiny;
    }
    if (iy == 0x7ff00000u) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    int k = ((int32_t)iy - (int32_t)ix) >> 20;
    double z;
    if (k > 60) { z = pi_o_2 + 0.5 * pi_lo; m &= 1; }
    else if (hx < 0 && k < -60) z = 0.0;
    else z = orc_atan(fabs(y / x));
    if (m == 0) return z;
    if (m == 1) return -z;
    if (m == 2) return pi - (z - pi_lo);
    return (z - pi_lo) - pi;
}

/* uv_map_sphere (src/math/uv_mapping.ts:19-25) */
void orc_uv_map_sphere(const double d[3], double uv[2])
{
    const double PI = 3.141592653589793, EPS = 2.220446049250313e-16;
    uv[0] = orc_atan2(d[1], d[0]) / PI / 2.0 + 0.5 - EPS;
    double len = sqrt((0.0 + d[0] * d[0]) + d[1] * d[1]);     /* vector.length(vector.reduce(dir, 2)) */
    uv[1] = orc_atan2(d[2], len) / PI + 0.5 - EPS;
}

/* ToInt32 of a finite double below 2^31 in magnitude (u*width, v*height): truncation */
static int32_t orc_toint32_small(double x)
{
    if (!(fabs(x) < 2147483648.0)) {
        if (!isfinite(x)) return 0;
        double m = fmod(trunc(x), 4294967296.0);
        if (m < 0) m += 4294967296.0;
        return (int32_t)(uint32_t)m;
    }
    return (int32_t)x;
}

/* ImageTexture.get_color (src/texture/texture_image.ts:40-63) of image k (1-based): 0 ok, -1 throw */
static int orc_image_color(const oworld *w, int k, double u, double v, double rgb[3])
{
    const double EPS = 2.220446049250313e-16;
    const rt_image_desc *im = &w->images[k - 1];
    if (u < 0 - EPS || u > 1 - EPS || v < 0 - EPS || v > 1 - EPS) return -1;  /* 'Texture coordinates out of bounds' */
    int32_t ui = orc_toint32_small(u * im->width), vi = orc_toint32_small(v * im->height);
    int64_t px_idx = ((int64_t)vi * im->width + ui) * 3;
    for (int c = 0; c < 3; c++) rgb[c] = (double)im->rgb[px_idx + c] / 255.0;   /* image_data[i] = byte / 255.0 */
    return 0;
}

/* Entity.get_aabb: sphere src/entities/entity_sphere.ts:90-96, box src/entities/entity_box.ts:75-82,
 * face DESIGN.md §Triangle (min corner, max extent). */
static void entity_aabb(const oentity *e, double apos[3], double *asize)
{
    const double *g = e->g;
    if (e->type == RT_ENT_SPHERE) {
        double d = g[3];
        for (int i = 0; i < 3; i++) apos[i] = g[i] - d * 0.5;
        *asize = d;
    } else if (e->type == RT_ENT_BOX) {
        double size = g[3];
        double h = size / 2;
        for (int i = 0; i < 3; i++) apos[i] = g[i] - h;
        *asize = size;
    } else {
        double ext[3];
        for (int i = 0; i < 3; i++) {
            double mn = js_min(js_min(g[i], g[3 + i]), g[6 + i]);
            double mx = js_max(js_max(g[i], g[3 + i]), g[6 + i]);
            apos[i] = mn;
            ext[i] = mx - mn;
        }
        *asize = js_max(js_max(ext[0], ext[1]), ext[2]);
    }
}

static void set_add(onode *t, int id)
{
    for (int i = 0; i < t->set_n; i++)
        if (t->set[i] == id) return;                            /* Set.add of a member: no-op */
    if (t->set_n == t->set_cap) {
        t->set_cap = t->set_cap ? 2 * t->set_cap : 4;
        t->set = (int *)realloc(t->set, sizeof(int) * (size_t)t->set_cap);
    }
    t->set[t->set_n++] = id;
}

static void set_delete(onode *t, int id)
{
    for (int i = 0; i < t->set_n; i++)
        if (t->set[i] == id) {
            memmove(t->set + i, t->set + i + 1, sizeof(int) * (size_t)(t->set_n - i - 1));
            t->set_n--;
            return;
        }
}

int orc_entity_in_set(onode *t, int id)
{
    for (int i = 0; i < t->set_n; i++)
        if (t->set[i] == id) return 1;
    return 0;
}

/* get_covering_node_for_entity — src/octree_entity.ts:60-79 */
static int covering_node(onode *tree, const double apos[3], double asize, onode **out)
{
    onode *t = NULL;
    int oc;
    int r = node_at_pos_c(tree, apos, &t, &oc, NULL);
    if (r < 0) return r;
    if (r == 0) { *out = NULL; return 0; }
    onode *cur = t;
    do {
        if (aabb_in_cube(apos, asize, cur->pos, cur->size)) break;
        cur = cur->parent;
    } while (cur != NULL);
    *out = cur;
    return 0;
}

/* extend_tree_inside_to_fit_up_to_depth — src/octree_entity.ts:92-114 */
static onode *extend_inside(oworld *w, onode *root, onode *node, const double apos[3], double asize, int max_depth)
{
    int cur_depth = get_level(node) - get_level(root);
    onode *cur = node;
    while (cur_depth < max_depth) {
        double s = 2.0 / cur->size;
        int32_t xyz[3];
        for (int i = 0; i < 3; i++) xyz[i] = js_toint32((apos[i] - cur->pos[i]) * s);
        double half = cur->size / 2;
        double spos[3];
        for (int i = 0; i < 3; i++) spos[i] = cur->pos[i] + (double)xyz[i] * half;
        if (!aabb_in_cube(apos, asize, spos, half)) break;
        onode *nt = node_alloc(w, spos, cur->size / 2, cur, 1);
        int idx = (int)(((uint32_t)xyz[2] << 2) | ((uint32_t)xyz[1] << 1) | ((uint32_t)xyz[0] << 0));
        if (!(idx >= 0 && idx <= 7)) return NULL;              /* Octree.set throws */
        cur->child[idx] = nt;                                   /* replaces an existing child, as the reference does */
        cur = nt;
        cur_depth++;
    }
    return cur;
}

/* extend_tree_outside_to_fit_up_to_depth — src/octree_entity.ts:125-171 */
static onode *extend_outside(oworld *w, onode *root, onode *node, const double apos[3], double asize, int max_depth)
{
    if (node->parent != NULL) return NULL;
    int cur_depth = get_level(root) - get_level(node);
    onode *cur = node;
    while (cur_depth < max_depth) {
        double s = 1.0 / cur->size;
        double a[3];
        for (int i = 0; i < 3; i++) {
            a[i] = (apos[i] - cur->pos[i]) * s;
            a[i] = js_max(js_min(floor(a[i]), 0), -1);          /* clamp(Math.floor(x), -1, 0) */
        }
        double ppos[3];
        for (int i = 0; i < 3; i++) ppos[i] = cur->pos[i] + a[i] * cur->size;
        double psize = cur->size * 2;
        int idx = (js_toint32(-a[2]) << 2) | (js_toint32(-a[1]) << 1) | (js_toint32(-a[0]) << 0);
        onode *np = node_alloc(w, ppos, psize, NULL, 1);
        if (!(idx >= 0 && idx <= 7)) return NULL;
        np->child[idx] = cur;
        cur->parent = np;
        cur = np;
        if (aabb_in_cube(apos, asize, ppos, psize)) return cur;
        cur_depth++;
    }
    return NULL;                                               /* TreeOutsideGrowError */
}

/* add_entity_to_octree — src/octree_entity.ts:174-188 (+ Entity.set_octree, src/entity.ts:50-56) */
int orc_add_entity(oworld *w, onode *tree, int type, const double geom[9], int shade, int substance,
                   int max_in_depth, int max_out_depth, onode **fitting_out)
{
    if (w->n_ents == w->cap_ents) {
        w->cap_ents = w->cap_ents ? 2 * w->cap_ents : 64;
        w->ents = (oentity *)realloc(w->ents, sizeof(oentity) * (size_t)w->cap_ents);
    }
    oentity *e = &w->ents[w->n_ents];
    memset(e, 0, sizeof(*e));
    e->type = type;
    for (int i = 0; i < 9; i++) e->g[i] = geom[i];
    if (type == RT_ENT_SPHERE) {
        /* SphereEntity ctor (src/entities/entity_sphere.ts:34-39) + Sphere.update_cache
         * (src/math/intersection.ts:94-97) */
        double d = geom[3];
        double radius = d / 2;
        e->g[4] = vdot(geom, geom);        /* _dot_pp    */
        e->g[5] = radius * radius;         /* _radius_sq (Sphere) */
        e->g[6] = d * d / 4;               /* _radius_sq (SphereEntity) */
        e->g[7] = 0; e->g[8] = 0;
    }
    e->shade = shade;
    e->substance = substance;
    e->octree = NULL;
    int id = w->n_ents++;

    double apos[3], asize;
    entity_aabb(e, apos, &asize);
    onode *fit = NULL;
    if (covering_node(tree, apos, asize, &fit) < 0) { w->n_ents--; return RT_E_TREE; }
    if (fit == NULL) {
        onode *abs_root = get_root(tree);
        fit = extend_outside(w, tree, abs_root, apos, asize, max_out_depth);
        if (!fit) { w->n_ents--; return RT_E_TREE; }
    }
    fit = extend_inside(w, tree, fit, apos, asize, max_in_depth);
    if (!fit) { w->n_ents--; return RT_E_TREE; }
    e = &w->ents[id];
    if (e->octree != NULL) set_delete(e->octree, id);
    e->octree = fit;
    set_add(fit, id);
    if (fitting_out) *fitting_out = fit;
    return id;
}

/* Entity._set_pos(pos) then add_entity_to_octree(tree, entity, flags) — the edit a host makes to
 * move an entity.  _set_pos: SphereEntity (src/entities/entity_sphere.ts:55-61; sphere_math.pos
 * runs Sphere.update_cache, src/math/intersection.ts:94-97, recomputing _dot_pp and, to the same
 * value, _radius_sq), BasicEntity (src/entities/entity_basic.ts:38-42), the build's FaceEntity
 * (translate so the centroid lands on pos).  Then Entity.set_octree (src/entity.ts:50-56):
 * Set.delete from the old node, Set.add to the fitting one — to the END of its Set order, even
 * when it is the same node. */
int orc_move_entity(oworld *w, onode *tree, int id, const double pos[3], int max_in_depth, int max_out_depth)
{
    if (id < 0 || id >= w->n_ents) return RT_E_INVALID;
    oentity *e = &w->ents[id];
    if (e->type == RT_ENT_SPHERE) {
        for (int i = 0; i < 3; i++) e->g[i] = pos[i];
        e->g[4] = vdot(pos, pos);
    } else if (e->type == RT_ENT_BOX) {
        for (int i = 0; i < 3; i++) e->g[i] = pos[i];
    } else {
        double d[3];
        for (int i = 0; i < 3; i++) d[i] = pos[i] - (e->g[i] + e->g[3 + i] + e->g[6 + i]) / 3;
        for (int v = 0; v < 3; v++)
            for (int i = 0; i < 3; i++) e->g[3 * v + i] += d[i];
    }
    double apos[3], asize;
    entity_aabb(e, apos, &asize);
    onode *fit = NULL;
    if (covering_node(tree, apos, asize, &fit) < 0) return RT_E_TREE;
    if (fit == NULL) {
        onode *abs_root = get_root(tree);
        fit = extend_outside(w, tree, abs_root, apos, asize, max_out_depth);
        if (!fit) return RT_E_TREE;
    }
    fit = extend_inside(w, tree, fit, apos, asize, max_in_depth);
    if (!fit) return RT_E_TREE;
    e = &w->ents[id];
    if (e->octree != NULL) set_delete(e->octree, id);
    e->octree = fit;
    set_add(fit, id);
    return 0;
}

/* Entity.set_material / set_texture / set_substance */
int orc_set_shade(oworld *w, int id, int shade, int substance)
{
    if (id < 0 || id >= w->n_ents) return RT_E_INVALID;
    w->ents[id].shade = shade;
    w->ents[id].substance = substance;
    return 0;
}

/* is_within: sphere src/entities/entity_sphere.ts:63-66, box src/entities/entity_box.ts:47-52
 * (pos as MIN corner), face: false. */
static int entity_is_within(const oentity *e, const double p[3])
{
    const double *g = e->g;
    if (e->type == RT_ENT_SPHERE) {
        double dist[3] = {p[0] - g[0], p[1] - g[1], p[2] - g[2]};
        return vdot(dist, dist) <= g[6];
    }
    if (e->type == RT_ENT_BOX) return point_in_cube_co(p, g, 1 * g[3]);
    return 0;
}

/* entity_at_pos — src/octree_entity.ts:191-202 */
static int entity_at_pos_c(oworld *w, onode *tree, const double p[3], int64_t *levels, int *fault)
{
    onode *t = NULL;
    int oc;
    int r = node_at_pos_c(tree, p, &t, &oc, levels);
    if (r < 0) { *fault = 1; return -1; }
    onode *cur = (r == 1) ? t : NULL;
    while (cur != NULL) {
        for (int i = 0; i < cur->set_n; i++) {
            int id = cur->set[i];
            if (entity_is_within(&w->ents[id], p)) return id;
        }
        cur = cur->parent;
    }
    return -1;
}

int orc_entity_at_pos(oworld *w, onode *tree, const double p[3])
{
    int fault = 0;
    int r = entity_at_pos_c(w, tree, p, NULL, &fault);
    return fault ? ORC_FAULT : r;
}

/* collision results */
typedef struct ohit {
    double point[3];
    double normal[3];
    int fault;
} ohit;

/* SphereEntity.collision_info — src/entities/entity_sphere.ts:68-88 with
 * Sphere.line_intersection src/math/intersection.ts:109-128 */
static int sphere_collision(const oentity *e, const double o[3], const double d[3], ohit *h)
{
    const double *g = e->g;
    double dist[3] = {o[0] - g[0], o[1] - g[1], o[2] - g[2]};
    double a = vdot(d, d);
    double b = vdot(dist, d) * 2;
    double c = vdot(o, o) + g[4] - vdot(o, g) * 2 - g[5];
    double delta = b * b - a * c * 4;
    if (delta < 0) return 0;
    double s = sqrt(delta);
    double tmp1 = -b / (a * 2);
    double tmp2 = s / (a * 2);
    double t1 = tmp1 - tmp2;
    double t2 = tmp1 + tmp2;
    double t;
    if (t1 >= 0) t = t1;
    else if (t2 >= 0) t = t2;
    else return 0;
    for (int i = 0; i < 3; i++) h->point[i] = o[i] + d[i] * t;
    double k = 2 / g[3];
    for (int i = 0; i < 3; i++) h->normal[i] = (h->point[i] - g[i]) * k;
    double sg = -js_sign(vdot(d, h->normal));
    for (int i = 0; i < 3; i++) h->normal[i] *= sg;
    return 1;
}

/* BoxEntity.collision_info — src/entities/entity_box.ts:54-73 */
static int box_collision(const oentity *e, const double o[3], const double d[3], ohit *h)
{
    const double *g = e->g;
    double bsize[3] = {1 * g[3], 1 * g[3], 1 * g[3]};
    double u1, u2;
    int i1, i2;
    if (!box_line_intersection(g, bsize, o, d, &u1, &i1, &u2, &i2)) return 0;
    double t;
    int fi;
    if (u1 >= 0) { t = u1; fi = i1; }
    else if (u2 >= 0) { t = u2; fi = i2; }
    else return 0;
    for (int i = 0; i < 3; i++) h->point[i] = o[i] + d[i] * t;
    if (fi < 0) { h->fault = 1; return 1; }                   /* vector.dot(dir, undefined) throws */
    const double *N = FACE_NORMALS[fi];
    double sg = -js_sign(vdot(d, N));
    for (int i = 0; i < 3; i++) h->normal[i] = N[i] * sg;
    return 1;
}

/* FaceEntity.collision_info — the build's triangle entity: fixed-order
 * f64 Moller-Trumbore on (v0, e1 = v1 - v0, e2 = v2 - v0), FORWARD t >= 0, normal =
 * normalize(cross(e1, e2)) * -sign(dot(d, n)), following the sphere/box conventions above. */
static void vcross(const double *a, const double *b, double *r)
{
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
}

static int face_collision(const oentity *e, const double o[3], const double d[3], ohit *h)
{
    const double *g = e->g;
    double e1[3], e2[3];
    for (int i = 0; i < 3; i++) { e1[i] = g[3 + i] - g[i]; e2[i] = g[6 + i] - g[i]; }
    double pv[3];
    vcross(d, e2, pv);
    double det = vdot(e1, pv);
    if (!(det != 0)) return 0;                                 /* parallel (or NaN) */
    double inv = 1 / det;
    double tv[3] = {o[0] - g[0], o[1] - g[1], o[2] - g[2]};
    double u = vdot(tv, pv) * inv;
    if (!(u >= 0 && u <= 1)) return 0;
    double qv[3];
    vcross(tv, e1, qv);
    double v = vdot(d, qv) * inv;
    if (!(v >= 0 && u + v <= 1)) return 0;
    double t = vdot(e2, qv) * inv;
    if (!(t >= 0)) return 0;
    for (int i = 0; i < 3; i++) h->point[i] = o[i] + d[i] * t;
    double n[3];
    vcross(e1, e2, n);
    double il = 1.0 / sqrt(vdot(n, n));
    for (int i = 0; i < 3; i++) n[i] = n[i] * il;
    double sg = -js_sign(vdot(d, n));
    for (int i = 0; i < 3; i++) h->normal[i] = n[i] * sg;
    return 1;
}

/* ============================ linearisation ================================================ */

static void dfs_number(onode *t, int *counter, int *n_list)
{
    t->dfs_id = (*counter)++;
    *n_list += t->set_n;
    for (int c = 0; c < 8; c++)
        if (t->child[c]) dfs_number(t->child[c], counter, n_list);
}

int orc_linear_size(onode *root, int *n_nodes, int *n_list)
{
    int cnt = 0, nl = 0;
    dfs_number(root, &cnt, &nl);
    *n_nodes = cnt;
    *n_list = nl;
    return 0;
}

static void dfs_fill(onode *t, int parent_id, double *node_pos, double *node_size, int32_t *node_parent,
                     int32_t *node_child, int32_t *ent_begin, int32_t *ent_count, int32_t *list, int *lpos)
{
    int id = t->dfs_id;
    for (int i = 0; i < 3; i++) node_pos[3 * id + i] = t->pos[i];
    node_size[id] = t->size;
    node_parent[id] = parent_id;
    ent_begin[id] = *lpos;
    ent_count[id] = t->set_n;
    for (int i = 0; i < t->set_n; i++) list[(*lpos)++] = t->set[i];
    for (int c = 0; c < 8; c++) node_child[8 * id + c] = t->child[c] ? t->child[c]->dfs_id : -1;
    for (int c = 0; c < 8; c++)
        if (t->child[c])
            dfs_fill(t->child[c], id, node_pos, node_size, node_parent, node_child, ent_begin, ent_count, list, lpos);
}

int orc_linearize(onode *root, double *node_pos, double *node_size, int32_t *node_parent,
                  int32_t *node_child, int32_t *ent_begin, int32_t *ent_count, int32_t *list)
{
    int n, nl;
    orc_linear_size(root, &n, &nl);
    int lpos = 0;
    dfs_fill(root, -1, node_pos, node_size, node_parent, node_child, ent_begin, ent_count, list, &lpos);
    return 0;
}

/* ============================ camera (src/view/camera.ts:207-250) ========================== */

/* vector.rotate_vectors — src/math/vector.ts:318-323 */
static void rotate_pair(double bx[3], double by[3], const double rot[2])
{
    double nx[3], ny[3];
    for (int i = 0; i < 3; i++) {
        nx[i] = bx[i] * rot[0] + by[i] * rot[1];
        ny[i] = bx[i] * -rot[1] + by[i] * rot[0];
    }
    memcpy(bx, nx, sizeof nx);
    memcpy(by, ny, sizeof ny);
}

typedef void (*emit_fn)(void *ud, int x, int y, const double dir[3]);

/* get_dir_for_each_pixel with the outer loop over n_outer (rows) and inner over n_inner. */
static void camera_scan(const rt_camera_desc *cam, int n_outer, int n_inner, emit_fn emit, void *ud)
{
    const double ch[2] = {cam->scan_h[0], -cam->scan_h[1]};   /* rot_scan_h_counter_v */
    const double cv[2] = {cam->scan_v[0], -cam->scan_v[1]};   /* rot_scan_v_counter_v */
    for (int half = 0; half < 2; half++) {
        /* iter_v(screen>>1, screen, rot_scan_v_v, 1, false) / iter_v((screen>>1)-1, -1, counter, -1, true) */
        int from_y = half == 0 ? (n_outer >> 1) : (n_outer >> 1) - 1;
        int to_y = half == 0 ? n_outer : -1;
        int inc_y = half == 0 ? 1 : -1;
        const double *rv = half == 0 ? cam->scan_v : cv;
        double fr[3], up[3];
        memcpy(fr, cam->fr, sizeof fr);
        memcpy(up, cam->up, sizeof up);
        if (half == 1) rotate_pair(fr, up, rv);
        for (int y = from_y; y != to_y; y += inc_y) {
            for (int hh = 0; hh < 2; hh++) {
                /* iter_h(inner>>1, inner, y, rot_scan_h_v, fr_v, 1, false) and
                 * iter_h((inner>>1)-1, -1, y, counter, fr_v, -1, true) */
                int from_x = hh == 0 ? (n_inner >> 1) : (n_inner >> 1) - 1;
                int to_x = hh == 0 ? n_inner : -1;
                int inc_x = hh == 0 ? 1 : -1;
                const double *rh = hh == 0 ? cam->scan_h : ch;
                double f[3], l[3];
                memcpy(f, fr, sizeof f);
                memcpy(l, cam->lf, sizeof l);
                if (hh == 1) rotate_pair(f, l, rh);
                for (int x = from_x; x != to_x; x += inc_x) {
                    emit(ud, x, y, f);
                    rotate_pair(f, l, rh);
                }
            }
            rotate_pair(fr, up, rv);
        }
    }
}

typedef struct { double *dirs; int w; } dirs_ud;
static void emit_rowmajor(void *ud, int x, int y, const double dir[3])
{
    dirs_ud *u = (dirs_ud *)ud;
    double *p = u->dirs + 3 * ((size_t)y * (size_t)u->w + (size_t)x);
    p[0] = dir[0]; p[1] = dir[1]; p[2] = dir[2];
}

int orc_camera_dirs(const rt_camera_desc *cam, double *dirs)
{
    if (cam->width <= 0 || cam->height <= 0) return RT_E_INVALID;
    dirs_ud u = {dirs, cam->width};
    camera_scan(cam, cam->height, cam->width, emit_rowmajor, &u);
    return 0;
}

typedef struct { int32_t *xs, *ys; double *dirs; size_t k; } lit_ud;
static void emit_literal(void *ud, int x, int y, const double dir[3])
{
    lit_ud *u = (lit_ud *)ud;
    u->xs[u->k] = x;
    u->ys[u->k] = y;
    memcpy(u->dirs + 3 * u->k, dir, 3 * sizeof(double));
    u->k++;
}

int orc_camera_scan_literal(const rt_camera_desc *cam, int32_t *xs, int32_t *ys, double *dirs)
{
    lit_ud u = {xs, ys, dirs, 0};
    /* reference: outer over screen_w (y), inner over screen_h (x) */
    camera_scan(cam, cam->width, cam->height, emit_literal, &u);
    return 0;
}

/* ============================ Ray.trace (src/raytracer.ts:168-277) ======================== */

enum { ST_OK = 0, ST_WARN = 1, ST_FAULT = 2, ST_CAP = 3 };

typedef struct trace_ctx {
    oworld *w;
    onode *root;
    const rt_config_desc *cfg;
    onode *start_tree;
    int start_oct;
    int start_sub;
    const double *start_pos;
} trace_ctx;

typedef struct ray_out {
    double rgb[3];
    int hit_ent, hit_node, segments, status;
    int64_t n_sph, n_box, n_tri, n_hit;
} ray_out;

/* RT_SCATTER_COUNTER (include/rt.h): draw n of pixel p is a pure function of (seed, p, n) —
 * the splitmix64 finaliser, top 53 bits scaled by 2^-53 — replacing the reference's shared
 * sequential `this.tracer.rng` stream, whose draw order depends on the pixel visiting order. */
static uint64_t orc_mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static double orc_counter_draw(uint64_t seed, uint64_t pixel, uint32_t n)
{
    uint64_t x = orc_mix64(seed + pixel * 0x9E3779B97F4A7C15ULL + ((uint64_t)n + 1) * 0xD1B54A32D192ED03ULL);
    return (double)(x >> 11) * (1.0 / 9007199254740992.0);
}

/* Ray.scatter_ray (src/raytracer.ts:121-133) after reflect_ray: isotropic_sphere_sample
 * (src/math/vector_utils.ts:8-14, rejection sampling, x/y/z drawn in argument order; capped at 64
 * attempts so a counter stream always terminates — P(64 rejections) = (1-pi/6)^64 ~ 1e-21), the
 * sample flipped into the normal's hemisphere, blended with the mirror direction by
 * roughness_index and normalised (vector.normalize_self = scale_self(v, 1.0/length(v))). */
static void orc_scatter(uint64_t seed, uint64_t pixel, uint32_t *draws, const double n[3], double rough,
                        double d[3])
{
    double v[3];
    for (int attempt = 0;; attempt++) {
        for (int i = 0; i < 3; i++) v[i] = orc_counter_draw(seed, pixel, (*draws)++) * 2 - 1;
        if (!(vdot(v, v) > 1) || attempt == 63) break;
    }
    if (vdot(v, n) < 0)
        for (int i = 0; i < 3; i++) v[i] *= -1;
    double keep = 1 - rough;
    double ref[3];
    for (int i = 0; i < 3; i++) ref[i] = d[i] * keep + v[i] * rough;
    double inv = 1.0 / sqrt(vdot(ref, ref));
    for (int i = 0; i < 3; i++) d[i] = ref[i] * inv;
}

/* test hook: one scatter_ray with the counter stream; returns the draw counter after it */
uint32_t orc_scatter_dir(uint64_t seed, uint64_t pixel, uint32_t draws, const double normal[3], double roughness,
                         double dir_inout[3])
{
    orc_scatter(seed, pixel, &draws, normal, roughness, dir_inout);
    return draws;
}

double orc_counter_draw_at(uint64_t seed, uint64_t pixel, uint32_t n) { return orc_counter_draw(seed, pixel, n); }

/* ---- shadow rays: a BUILD EXTENSION (the reference samples no lights, src/raytracer.ts:168-277).
 * The frozen definition is include/rt.h's rt_set_lights comment; this is its CPU
 * statement, the GPU's parity target.  Not pinned by any reference output: parity is against this. */
int orc_set_lights(oworld *w, const rt_light *lights, int n, double ambient)
{
    if (n < 0 || n > RT_MAX_LIGHTS || (n && !lights)) return RT_E_INVALID;
    w->n_lights = n;
    w->ambient = n ? ambient : 0;
    for (int k = 0; k < n; k++) w->lights[k] = lights[k];
    return 0;
}

void orc_set_shadow_brute(oworld *w, int on) { w->shadow_brute = on != 0; }

/* The bounds of an entity's collision geometry (not Entity.get_aabb): sphere centre +- |d|/2, box
 * centre +- |size|/2 (intersection.Box is centred, src/entities/entity_box.ts:54-56), triangle the
 * vertices' min / max.  Non-finite geometry gets an unbounded box. */
static void geom_bounds(const oentity *e, double lo[3], double hi[3])
{
    const double *g = e->g;
    int finite = 1;
    for (int i = 0; i < 3; i++) {
        if (e->type == RT_ENT_FACE) {
            lo[i] = g[i]; hi[i] = g[i];
            for (int v = 1; v < 3; v++) {
                if (g[3 * v + i] < lo[i]) lo[i] = g[3 * v + i];
                if (g[3 * v + i] > hi[i]) hi[i] = g[3 * v + i];
            }
            for (int v = 0; v < 3; v++) finite = finite && isfinite(g[3 * v + i]);
        } else {
            double h = fabs(g[3]) * 0.5;
            lo[i] = g[i] - h; hi[i] = g[i] + h;
            finite = finite && isfinite(lo[i]) && isfinite(hi[i]);
        }
    }
    if (!finite)
        for (int i = 0; i < 3; i++) { lo[i] = -INFINITY; hi[i] = INFINITY; }
}

/* Post-order: every node's sb_lo / sb_hi / sb_n over its own set and its subtrees. */
static void shadow_bounds(oworld *w, onode *t)
{
    for (int i = 0; i < 3; i++) { t->sb_lo[i] = INFINITY; t->sb_hi[i] = -INFINITY; }
    t->sb_n = t->set_n;
    for (int k = 0; k < t->set_n; k++) {
        double lo[3], hi[3];
        geom_bounds(&w->ents[t->set[k]], lo, hi);
        for (int i = 0; i < 3; i++) {
            if (lo[i] < t->sb_lo[i]) t->sb_lo[i] = lo[i];
            if (hi[i] > t->sb_hi[i]) t->sb_hi[i] = hi[i];
        }
    }
    for (int c = 0; c < 8; c++) {
        onode *ch = t->child[c];
        if (!ch) continue;
        shadow_bounds(w, ch);
        if (!ch->sb_n) continue;
        t->sb_n += ch->sb_n;
        for (int i = 0; i < 3; i++) {
            if (ch->sb_lo[i] < t->sb_lo[i]) t->sb_lo[i] = ch->sb_lo[i];
            if (ch->sb_hi[i] > t->sb_hi[i]) t->sb_hi[i] = ch->sb_hi[i];
        }
    }
}

/* Whether the segment q + u t, t in [0, dist], may meet the box [lo, hi]: a slab test on the box
 * widened by 2^-20 of the largest magnitude involved (and by as much on the parameter), so that a
 * hit point computed in binary64 on the segment's part before dist is never pruned.  Conservative
 * only: the decision itself is the exact test of each entity that passes. */
static int seg_may_meet(const double q[3], const double u[3], double dist, const double lo[3], const double hi[3])
{
    double S = 1 + fabs(dist);
    for (int i = 0; i < 3; i++) {
        if (fabs(q[i]) > S) S = fabs(q[i]);
        if (isfinite(lo[i]) && fabs(lo[i]) > S) S = fabs(lo[i]);
        if (isfinite(hi[i]) && fabs(hi[i]) > S) S = fabs(hi[i]);
    }
    const double m = S * 0x1p-20;
    double t0 = -m, t1 = dist + m;
    for (int i = 0; i < 3; i++) {
        const double l = lo[i] - m, h = hi[i] + m;
        if (u[i] == 0) {
            if (q[i] < l || q[i] > h) return 0;
            continue;
        }
        double a = (l - q[i]) / u[i], b = (h - q[i]) / u[i];
        if (a > b) { double x = a; a = b; b = x; }
        if (a > t0) t0 = a;                                   /* a NaN bound never prunes */
        if (b < t1) t1 = b;
        if (t0 > t1) return 0;
    }
    return 1;
}

/* Whether entity e blocks the shadow ray: not a light, and its collision_info(q, u) hits (or throws,
 * with the hit point it computed) at h with |h - q| < lim. */
static int entity_blocks(const oworld *w, const oentity *e, const double q[3], const double u[3], double lim)
{
    ohit h;
    memset(&h, 0, sizeof h);
    int got;
    if (e->type == RT_ENT_SPHERE) got = sphere_collision(e, q, u, &h);
    else if (e->type == RT_ENT_BOX) got = box_collision(e, q, u, &h);
    else got = face_collision(e, q, u, &h);
    if (!got || w->shades[e->shade].light) return 0;
    double diff[3] = {h.point[0] - q[0], h.point[1] - q[1], h.point[2] - q[2]};
    return sqrt(vdot(diff, diff)) < lim;
}

static int subtree_blocks(const oworld *w, const onode *t, const double q[3], const double u[3], double dist,
                          double lim)
{
    const int brute = w->shadow_brute;
    if (!t->sb_n || (!brute && !seg_may_meet(q, u, dist, t->sb_lo, t->sb_hi))) return 0;
    for (int k = 0; k < t->set_n; k++) {
        const oentity *e = &w->ents[t->set[k]];
        if (!brute) {
            double lo[3], hi[3];
            geom_bounds(e, lo, hi);
            if (!seg_may_meet(q, u, dist, lo, hi)) continue;
        }
        if (entity_blocks(w, e, q, u, lim)) return 1;
    }
    for (int c = 0; c < 8; c++)
        if (t->child[c] && subtree_blocks(w, t->child[c], q, u, dist, lim)) return 1;
    return 0;
}

/* 1 when the shadow ray (q, u) toward a light at distance dist (from the hit point) is blocked: some
 * entity of the tree that is not a light has a forward hit, or a throwing test, nearer than
 * dist - 1e-3 (include/rt.h rt_set_lights).  An existence question: the order entities are visited in
 * does not matter, and the bounds only skip entities whose test cannot report such a hit
 * (shadow_brute tests them all).  Needs shadow_bounds(root) first. */
static int shadow_blocked(oworld *w, onode *root, const double q[3], const double u[3], double dist)
{
    return subtree_blocks(w, root, q, u, dist, dist - 1e-3);
}

/* test hook: one shadow ray's answer on the tree as it is now (bounds recomputed) */
int orc_shadow_blocked(oworld *w, onode *root, const double q[3], const double u[3], double dist)
{
    shadow_bounds(w, root);
    return shadow_blocked(w, root, q, u, dist);
}

/* the matte hit's light factor: ambient + the unblocked lights' rgb * (cosine * isl) */
static void shadow_factor(oworld *w, onode *root, const rt_config_desc *cfg, const double p[3],
                          const double nrm[3], double path, double s[3])
{
    s[0] = s[1] = s[2] = w->ambient;
    for (int l = 0; l < w->n_lights; l++) {
        const rt_light *lt = &w->lights[l];
        double v[3] = {lt->pos[0] - p[0], lt->pos[1] - p[1], lt->pos[2] - p[2]};
        double dist = sqrt(vdot(v, v));
        if (!(dist > 0)) continue;
        double inv = 1.0 / dist;
        double u[3] = {v[0] * inv, v[1] * inv, v[2] * inv};
        double cosine = vdot(nrm, u);
        if (!(cosine > 0)) continue;
        double q[3] = {p[0] + u[0] * 1e-3, p[1] + u[1] * 1e-3, p[2] + u[2] * 1e-3};
        if (shadow_blocked(w, root, q, u, dist)) continue;
        double t = (path + dist) * cfg->distance_attenuation_factor;
        double isl = 1.0 / (2.220446049250313e-16 + t * t);
        double k = cosine * isl;
        for (int i = 0; i < 3; i++) s[i] += lt->rgb[i] * k;
    }
}

static void trace_ray(const trace_ctx *tc, owalker *wk, const double dir0[3], uint64_t pixel, ray_out *ro)
{
    int matte = 0;                                                           /* shadow rays */
    double mnrm[3] = {0, 0, 0};
    uint32_t draws = 0;
    oworld *w = tc->w;
    const rt_config_desc *cfg = tc->cfg;
    double o[3] = {tc->start_pos[0], tc->start_pos[1], tc->start_pos[2]};   /* refpoint = clone(start) */
    double d[3] = {dir0[0], dir0[1], dir0[2]};                               /* keep_dir_unnormalized */
    double col[3] = {1, 1, 1};                                               /* COLOR_WHITE */
    int refcount = 0, light_hit = 0, cur_sub = tc->start_sub;
    double path = 0;
    ro->hit_ent = -1; ro->hit_node = -1; ro->segments = 1; ro->status = ST_OK;

    if (orc_walker_set(wk, o, d, tc->start_tree, tc->start_oct) < 0) { ro->status = ST_FAULT; goto out; }
    for (;;) {
        onode *node, *pt;
        int po;
        int r = orc_walker_next(wk, &node, &pt, &po);
        if (r < 0) { ro->status = ST_FAULT; goto out; }
        if (r == 0) break;
        /* for (entity of search_array.set) — first entity with a collision wins */
        int hit_id = -1;
        ohit h;
        for (int i = 0; i < node->set_n; i++) {
            int id = node->set[i];
            const oentity *e = &w->ents[id];
            memset(&h, 0, sizeof h);
            int got;
            if (e->type == RT_ENT_SPHERE) { ro->n_sph++; got = sphere_collision(e, o, d, &h); }
            else if (e->type == RT_ENT_BOX) { ro->n_box++; got = box_collision(e, o, d, &h); }
            else { ro->n_tri++; got = face_collision(e, o, d, &h); }
            if (got) { hit_id = id; break; }
        }
        if (hit_id < 0) continue;
        if (h.fault) { ro->status = ST_FAULT; goto out; }
        if (ro->hit_ent < 0 && ro->segments == 1) { ro->hit_ent = hit_id; ro->hit_node = node->dfs_id; }
        /* acute-normal guard :200-203 */
        if (vdot(d, h.normal) >= 0) { ro->status = ST_WARN; goto out; }
        refcount++;
        ro->n_hit++;
        const oentity *e = &w->ents[hit_id];
        const rt_shade *sh = &w->shades[e->shade];
        /* SolidMaterial.alter_ray → mul_color (src/materials/material_solid.ts:30-36, src/physics/color.ts:50-52) */
        if (sh->image) {
            /* texture.get_color(entity.map_uv(point)): sphere uv_map_sphere(vector.sub(p, pos))
             * (src/entities/entity_sphere.ts:98-101); box (src/entities/entity_box.ts:104-107) and
             * face: [0, 0] */
            double uv[2] = {0, 0}, tc[3];
            if (e->type == RT_ENT_SPHERE) {
                double dist[3] = {h.point[0] - e->g[0], h.point[1] - e->g[1], h.point[2] - e->g[2]};
                orc_uv_map_sphere(dist, uv);
            }
            if (orc_image_color(w, sh->image, uv[0], uv[1], tc) < 0) { ro->status = ST_FAULT; goto out; }
            for (int i = 0; i < 3; i++) col[i] = col[i] * tc[i];
        } else {
            for (int i = 0; i < 3; i++) col[i] = col[i] * sh->rgb[i];
        }
        double diff[3] = {h.point[0] - o[0], h.point[1] - o[1], h.point[2] - o[2]};
        path += sqrt(vdot(diff, diff));
        o[0] = h.point[0]; o[1] = h.point[1]; o[2] = h.point[2];
        if (sh->light) { light_hit = 1; break; }
        if (sh->response == RT_RESP_REFLECTION) {
            if (!sh->mirror) {                                  /* matte: terminal */
                if (w->n_lights) { matte = 1; mnrm[0] = h.normal[0]; mnrm[1] = h.normal[1]; mnrm[2] = h.normal[2]; }
                goto out;
            }
            /* reflect_ray → vector.reflection (src/math/vector.ts:263-268) */
            double ns = -vdot(d, h.normal);
            double k = ns * 2;
            for (int i = 0; i < 3; i++) d[i] = d[i] + h.normal[i] * k;
            if (sh->roughness > 0.0) {                          /* :233-235 */
                if (cfg->scatter_mode != RT_SCATTER_COUNTER) { ro->status = ST_FAULT; goto out; }
                orc_scatter(cfg->scatter_seed, pixel, &draws, h.normal, sh->roughness, d);
            }
            for (int i = 0; i < 3; i++) o[i] += d[i] * 1e-3;    /* move_slightly_forward :158-164 */
        } else if (sh->response == RT_RESP_TRANSMISSION) {
            for (int i = 0; i < 3; i++) o[i] += d[i] * 1e-3;
            int fault = 0;
            int rf = entity_at_pos_c(w, tc->root, o, &wk->c_loc, &fault);
            if (fault) { ro->status = ST_FAULT; goto out; }
            int sub = rf >= 0 ? w->ents[rf].substance : cfg->default_substance;
            if (sub >= 0) {
                if (cur_sub < 0) { ro->status = ST_FAULT; goto out; }   /* undefined.refractive_index */
                /* refract_ray :135-150 */
                double r_ratio = w->ri[cur_sub] / w->ri[sub];
                double r_ratio_sq = r_ratio * r_ratio;
                double cosine = vdot(d, h.normal);
                double cosine_sq = cosine * cosine;
                double ref_sine_sq = (1 - cosine_sq) * r_ratio_sq;
                if (ref_sine_sq <= 1) {
                    double ref_cosine = sqrt(1 - ref_sine_sq);
                    double adj[3];
                    for (int i = 0; i < 3; i++) adj[i] = h.normal[i] * (ref_cosine - cosine);
                    for (int i = 0; i < 3; i++) d[i] *= r_ratio;
                    for (int i = 0; i < 3; i++) d[i] -= adj[i];
                } else {
                    double ns = -vdot(d, h.normal);
                    double k = ns * 2;
                    for (int i = 0; i < 3; i++) d[i] = d[i] + h.normal[i] * k;
                }
                cur_sub = sub;
            }
        } else {
            goto out;                                           /* default: return */
        }
        if (orc_walker_set(wk, o, d, NULL, 0) < 0) { ro->status = ST_FAULT; goto out; }
        if (refcount >= cfg->refmax) { col[0] = col[1] = col[2] = 0; goto out; }   /* COLOR_BLACK */
        ro->segments++;
    }
    if (!light_hit) {
        if (cfg->sky_image) {
            /* SkySphere.get_color(this.dir) — src/sky/sky_sphere.ts:23-26 */
            double uv[2], tc[3];
            orc_uv_map_sphere(d, uv);
            if (orc_image_color(w, cfg->sky_image, uv[0], uv[1], tc) < 0) { ro->status = ST_FAULT; goto out; }
            for (int i = 0; i < 3; i++) col[i] = col[i] * tc[i];
        } else {
            for (int i = 0; i < 3; i++) col[i] = col[i] * cfg->sky_rgb[i];   /* sky.get_color(dir) */
        }
    } else {
        double t = path * cfg->distance_attenuation_factor;
        double isl = 1.0 / (2.220446049250313e-16 + t * t);   /* (x)**2 == x*x (fdlibm pow special case) */
        for (int i = 0; i < 3; i++) col[i] = col[i] * isl;
        /* walker.set_pos_and_dir(this.refpoint, this.dir) — :276.  The colour is final, but the re-seat
         * runs node_at_pos / setup_cur_node, which throw like the seat at :254: the frame aborts */
        if (orc_walker_set(wk, o, d, NULL, 0) < 0) ro->status = ST_FAULT;
    }
out:
    if (matte) {
        double sf[3];
        shadow_factor(w, tc->root, cfg, o, mnrm, path, sf);
        for (int i = 0; i < 3; i++) col[i] = col[i] * sf[i];
    }
    ro->rgb[0] = col[0]; ro->rgb[1] = col[1]; ro->rgb[2] = col[2];
}

/* ============================ trace_frame (src/raytracer.ts:308-330) ====================== */

typedef struct frame_job {
    const trace_ctx *tc;
    const rt_camera_desc *cam;
    const double *dirs;
    int npix;
    const int32_t *pix;
    float *rgb;
    int32_t *hit_entity, *hit_node, *segs;
    uint8_t *status;
    int tid, nthreads;
    owalker *wk;
    int64_t counters[11];
} frame_job;

static void *frame_worker(void *arg)
{
    frame_job *j = (frame_job *)arg;
    const rt_config_desc *cfg = j->tc->cfg;
    double wgt = cfg->col_weight;
    for (int k = j->tid; k < j->npix; k += j->nthreads) {
        int p = j->pix ? j->pix[k] : k;
        ray_out ro;
        memset(&ro, 0, sizeof ro);
        trace_ray(j->tc, j->wk, j->dirs + 3 * (size_t)p, (uint64_t)p, &ro);
        /* ExposureBuffer.set_color_i — src/view/exposure_buffer.ts:77-91 */
        float *px = j->rgb + 3 * (size_t)p;
        for (int c = 0; c < 3; c++) {
            double v = ro.rgb[c] * wgt;
            v += (double)px[c] * (1 - wgt);
            px[c] = (float)v;
        }
        if (j->hit_entity) j->hit_entity[p] = ro.hit_ent;
        if (j->hit_node) j->hit_node[p] = ro.hit_node;
        if (j->segs) j->segs[p] = ro.segments;
        if (j->status) j->status[p] = (uint8_t)ro.status;
        j->counters[0] += ro.segments;
        j->counters[4] += ro.n_sph;
        j->counters[5] += ro.n_box;
        j->counters[6] += ro.n_tri;
        j->counters[7] += ro.n_hit;
        j->counters[8] += 1;
        j->counters[9] += ro.status == ST_WARN;
        j->counters[10] += ro.status == ST_FAULT || ro.status == ST_CAP;
    }
    j->counters[1] = j->wk->c_ret;
    j->counters[2] = j->wk->c_slot;
    j->counters[3] = j->wk->c_loc;
    return NULL;
}

int orc_trace_frame(oworld *w, onode *root, const rt_camera_desc *cam, const rt_config_desc *cfg,
                    int npix, const int32_t *pix, float *rgb_inout, int32_t *hit_entity,
                    int32_t *hit_node, int32_t *segments, uint8_t *status, int64_t *counters,
                    int nthreads)
{
    if (cam->width <= 0 || cam->height <= 0 || nthreads < 1) return RT_E_INVALID;
    size_t P = (size_t)cam->width * (size_t)cam->height;
    if (!pix) npix = (int)P;
    int nn, nl;
    orc_linear_size(root, &nn, &nl);                            /* assigns dfs ids */
    double *dirs = (double *)malloc(sizeof(double) * 3 * P);
    orc_camera_dirs(cam, dirs);

    trace_ctx tc;
    tc.w = w;
    tc.root = root;
    tc.cfg = cfg;
    tc.start_pos = cam->pos;
    /* start_node = node_at_pos(otree, start_pos); start substance from entity_at_pos (:309-313) */
    onode *st = NULL;
    int so = 0;
    int r = node_at_pos_c(root, cam->pos, &st, &so, NULL);
    int fault = 0;
    int se = entity_at_pos_c(w, root, cam->pos, NULL, &fault);
    if (r < 0 || fault) { free(dirs); return ORC_FAULT; }
    tc.start_tree = r == 1 ? st : NULL;
    tc.start_oct = so;
    tc.start_sub = se >= 0 ? w->ents[se].substance : cfg->default_substance;
    if (w->n_lights) shadow_bounds(w, root);                    /* shadow rays: the tree's bounds */

    frame_job *jobs = (frame_job *)calloc((size_t)nthreads, sizeof(frame_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        frame_job *j = &jobs[t];
        j->tc = &tc; j->cam = cam; j->dirs = dirs; j->npix = npix; j->pix = pix;
        j->rgb = rgb_inout; j->hit_entity = hit_entity; j->hit_node = hit_node; j->segs = segments;
        j->status = status; j->tid = t; j->nthreads = nthreads;
        j->wk = orc_walker_new(w, root, 0);
    }
    if (nthreads == 1) frame_worker(&jobs[0]);
    else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, frame_worker, &jobs[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    int64_t tot[11] = {0};
    for (int t = 0; t < nthreads; t++)
        for (int c = 0; c < 11; c++) tot[c] += jobs[t].counters[c];
    if (counters) memcpy(counters, tot, sizeof tot);
    free(jobs);
    free(th);
    free(dirs);
    return tot[10] ? ORC_FAULT : 0;
}

/* ============================ ExposureBuffer consumers ===================================== */

/* rgb_to_y, src/view/exposure_buffer.ts:161-172: W_R*r + W_G*g + W_B*b, left to right */
static double orc_rgb_to_y(const float *px)
{
    const double W_R = 0.299, W_G = 0.587, W_B = 0.114;
    return W_R * (double)px[0] + W_G * (double)px[1] + W_B * (double)px[2];
}

/* get_mean :90-104, get_variance(mean) :106-120, get_absolute_dev(mean) :122-136 — sequential
 * sums, each divided by n_pixels (the _mean/_variance caches are never filled). */
void orc_exposure_stats(const float *rgb, int64_t n_pixels, double out[3])
{
    double mean = 0;
    for (int64_t i = 0; i < n_pixels * 3; i += 3) mean += orc_rgb_to_y(rgb + i);
    mean /= (double)n_pixels;
    double variance = 0;
    for (int64_t i = 0; i < n_pixels * 3; i += 3) {
        const double delta = orc_rgb_to_y(rgb + i) - mean;
        variance += delta * delta;
    }
    variance /= (double)n_pixels;
    double dev = 0;
    for (int64_t i = 0; i < n_pixels * 3; i += 3) dev += fabs(orc_rgb_to_y(rgb + i) - mean);
    dev /= (double)n_pixels;
    out[0] = mean;
    out[1] = variance;
    out[2] = dev;
}

/* clamp, src/math/mathutils.ts:18-20 */
static double js_clamp(double x, double lo, double hi) { return js_max(js_min(x, hi), lo); }

/* ToneMapper_Identity :26-34; ToneMapper_DRLimited constructor :39-44 (dynamic_coef = 1 << dr);
 * _StdDevAroundMean :48-63; _AbsDevAroundMean :65-80 */
int orc_tonemap_range(int mode, const double stats[3], int dynamic_range, double min_dynamic, double max_dynamic,
                      double out[2])
{
    if (mode == 0) { out[0] = 0; out[1] = 1; return 0; }
    if (mode != 1 && mode != 2) return -1;
    const double coef = (double)(int32_t)((uint32_t)1 << ((uint32_t)dynamic_range & 31));
    const double mean_br = stats[0];
    const double dev_br = mode == 1 ? sqrt(stats[1]) : stats[2];
    double drange_max = js_min(mean_br + dev_br, max_dynamic);
    double drange_min = drange_max / coef;
    if (drange_min < min_dynamic) {
        drange_min = min_dynamic;
        drange_max = drange_min * coef;
    }
    out[0] = drange_min;
    out[1] = drange_max;
    return 0;
}

/* discretize_to_screen :145-158 with CanvasScreen.set_pixel_i / convert_color
 * (src/view/screen_canvas.ts:45-55,92-94).  `this.pixels.slice(i, i+2)` is a two-element
 * Float32Array; its .map() stores each clamp(c * scale_coef, 0, 1) rounded to f32, and
 * convert_color maps those through (clamp(x,0,1)*255) << 0.  col_conv[2] is undefined, which the
 * Uint8ClampedArray stores as 0; alpha is 0xff. */
void orc_tonemap(const float *rgb, int64_t n_pixels, double low, double high, uint8_t *rgba)
{
    const double drange = high - low;
    const double EPS = 2.220446049250313e-16;          /* Number.EPSILON */
    for (int64_t px_i = 0, i = 0; px_i < n_pixels; ++px_i, i += 3) {
        const double px_brightness = orc_rgb_to_y(rgb + i);
        const double cmpr_brightness = (px_brightness - low) / drange;
        const double scale_coef = cmpr_brightness / (px_brightness + EPS);
        float compressed[2];
        for (int k = 0; k < 2; k++) compressed[k] = (float)js_clamp((double)rgb[i + k] * scale_coef, 0.0, 1.0);
        for (int k = 0; k < 2; k++) rgba[4 * px_i + k] = (uint8_t)js_toint32(js_clamp((double)compressed[k], 0.0, 1.0) * 255);
        rgba[4 * px_i + 2] = 0;
        rgba[4 * px_i + 3] = 0xff;
    }
}
