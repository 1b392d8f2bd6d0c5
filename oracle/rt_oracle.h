/*
 * rt_oracle.h — CPU restatement of the raytracer.js render path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the HIP path is compared against; nothing in the
 * product (raytracer.js_amd/, include/) links, loads or calls it.  Only tests/, the smoke() check
 * in __graft_entry__.py and bench.py's cpu_baseline leg may use it.
 *
 * Pinning: the reference is TypeScript and its toolchain (tsc / esbuild / jest) is absent from
 * this image, so it cannot be executed here.  This restatement is pinned by
 * the reference's own known-answer tests (test/octree-space-walker.test.ts:29-35,57-70,
 * test/octree-space.test.ts:36-46, test/octree-entity.test.ts:52-63, test/octree.test.ts:3-7,
 * test/view-camera.test.ts:17-49) — see tests/golden/reference_kats.json.  Pixel colours are not
 * covered by any reference test: for them parity is UNPINNED beyond this line-by-line restatement.
 *
 * Every function cites the reference file:line it restates.  Arithmetic follows JS `number`
 * semantics: IEEE-754 binary64, one rounding per operation, evaluation order as written in the
 * reference, no fused multiply-add (built with -ffp-contract=off), ToInt32 for `<<`/`|`.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include "../include/rt.h"   /* plain-data descriptor layouts only (rt_camera_desc, rt_config_desc, rt_shade) */

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_OCT_UNDEF (-2147483647 - 1)   /* JS `undefined` octant (the tree itself)          */
#define ORC_FAULT     (-5)                /* the reference would throw here                      */

typedef struct onode onode;
typedef struct oworld oworld;
typedef struct owalker owalker;

/* world = arena owning every node, entity and walker */
oworld *orc_world_new(void);
void    orc_world_free(oworld *w);

/* --- octree (src/octree.ts, src/octree_space.ts) --- */
onode  *orc_tree_new(oworld *w, const double pos[3], double size, int with_entity_set);
int     orc_new_subtree(oworld *w, onode *t, int n, onode **out);       /* new_subtree, :95-108 */
int     orc_tree_get(onode *t, int n, onode **out);                      /* Octree.get, :51-54 (-1 = throw) */
onode  *orc_tree_parent(onode *t);
int     orc_tree_id(onode *t);
void    orc_tree_dims(onode *t, double pos[3], double *size);
int     orc_node_at_pos(onode *t, const double p[3], onode **tree, int *octant);  /* 1 found, 0 null, <0 throw */
int     orc_index_within_parent(onode *t, int *has);                     /* :113-125 */

/* --- walker (src/octree_space.ts:159-408) --- */
owalker *orc_walker_new(oworld *w, onode *tree, int include_undefined);
/* node_tree == NULL: let set_position locate the node (node_at_pos) */
int      orc_walker_set(owalker *wk, const double pos[3], const double dir[3], onode *node_tree, int node_octant);
/* 1 = output (node may be NULL with include_undefined; pos_octant ORC_OCT_UNDEF for the root),
 * 0 = undefined (end), ORC_FAULT = throw */
int      orc_walker_next(owalker *wk, onode **node, onode **pos_tree, int *pos_octant);

/* --- scene (src/octree_entity.ts, src/entity.ts, src/entities/) --- */
int  orc_set_tables(oworld *w, const rt_shade *shades, int n_shades, const double *ri, int n_ri);
int  orc_set_images(oworld *w, const rt_image_desc *images, int n);      /* ImageTextures (copied) */
/* shadow rays, a build extension (include/rt.h rt_set_lights): n = 0 is the reference */
int  orc_set_lights(oworld *w, const rt_light *lights, int n, double ambient);
/* shadow rays: test every entity instead of the bounded search (tests pin the two equal) */
void orc_set_shadow_brute(oworld *w, int on);
/* test hook: whether the shadow ray from q along u toward a light at distance dist is blocked */
int  orc_shadow_blocked(oworld *w, onode *root, const double q[3], const double u[3], double dist);
double orc_atan(double x);                                                 /* Math.atan (V8 / fdlibm) */
double orc_atan2(double y, double x);                                      /* Math.atan2 (V8 / fdlibm) */
void orc_uv_map_sphere(const double d[3], double uv[2]);                  /* src/math/uv_mapping.ts:19-25 */
/* add_entity_to_octree(tree, entity, {max_in_depth, max_out_depth}) (:174-188); returns entity id
 * (creation order) or <0; *fitting receives the node holding the entity. */
int  orc_add_entity(oworld *w, onode *tree, int type, const double geom[9], int shade, int substance,
                    int max_in_depth, int max_out_depth, onode **fitting);
/* Entity._set_pos + add_entity_to_octree (re-filed at the end of the fitting node's Set order) */
int  orc_move_entity(oworld *w, onode *tree, int entity_id, const double pos[3], int max_in_depth, int max_out_depth);
int  orc_set_shade(oworld *w, int entity_id, int shade, int substance);
int  orc_entity_in_set(onode *t, int entity_id);                          /* EntitySet.set.has */
int  orc_entity_at_pos(oworld *w, onode *tree, const double p[3]);       /* :191-202, -1 = undefined */

/* DFS pre-order linearisation (children 0..7) of the tree below `root` */
int  orc_linear_size(onode *root, int *n_nodes, int *n_list);
int  orc_linearize(onode *root, double *node_pos, double *node_size, int32_t *node_parent,
                   int32_t *node_child, int32_t *ent_begin, int32_t *ent_count, int32_t *list);

/* --- frame (src/raytracer.ts:308-330 with src/view/camera.ts:207-250) --- */
/* Primary directions in row-major pixel order (corrected axes). */
int  orc_camera_dirs(const rt_camera_desc *cam, double *dirs);
/* Reference-literal scan order (x over screen_h, y over screen_w; src/view/camera.ts:242-249),
 * emitted as (x, y, dir) triples in generator order; square screens only in the reference. */
int  orc_camera_scan_literal(const rt_camera_desc *cam, int32_t *xs, int32_t *ys, double *dirs);

/* Trace selected pixels (pix == NULL: all W*H) of one frame.  Outputs are indexed by pixel
 * (y*W+x).  rgb_inout: ExposureBuffer pixels (read when col_weight != 1).  counters[11] receive
 * the rt_stats counter fields in order (segments .. n_fault). nthreads >= 1.  Returns 0, or
 * ORC_FAULT when any traced pixel faulted (outputs are still written; status[] == 2 there). */
int  orc_trace_frame(oworld *w, onode *root, const rt_camera_desc *cam, const rt_config_desc *cfg,
                     int npix, const int32_t *pix, float *rgb_inout, int32_t *hit_entity,
                     int32_t *hit_node, int32_t *segments, uint8_t *status, int64_t *counters,
                     int nthreads);

/* ExposureBuffer consumers (src/view/exposure_buffer.ts, src/view/tone_mapping.ts,
 * src/view/screen_canvas.ts): sequential luminance statistics {mean, variance, absdev}, the
 * ToneMapper dynamic range (mode 0 identity, 1 std-dev, 2 abs-dev), and the RGBA8 image
 * discretize_to_screen hands a CanvasScreen. */
void orc_exposure_stats(const float *rgb, int64_t n_pixels, double out[3]);
int  orc_tonemap_range(int mode, const double stats[3], int dynamic_range, double min_dynamic,
                       double max_dynamic, double out[2]);
void orc_tonemap(const float *rgb, int64_t n_pixels, double low, double high, uint8_t *rgba);

/* RT_SCATTER_COUNTER (include/rt.h): draw n of pixel p, and one Ray.scatter_ray
 * (src/raytracer.ts:121-133) on dir_inout starting at draw `draws`; returns the next draw index. */
double orc_counter_draw_at(uint64_t seed, uint64_t pixel, uint32_t n);
uint32_t orc_scatter_dir(uint64_t seed, uint64_t pixel, uint32_t draws, const double normal[3], double roughness,
                         double dir_inout[3]);

#ifdef __cplusplus
}
#endif
#endif
