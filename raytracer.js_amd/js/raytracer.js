/*
 * raytracer.js — drop-in replacement for the reference's `Raytracer` class
 * (Dark565/raytracer.js src/raytracer.ts:281-339) whose trace_frame() runs on an MI355X.
 *
 * The scene objects stay the reference's own: the Octree/EntitySet tree built with
 * add_entity_to_octree (src/octree_entity.ts:174-188), SphereEntity / BoxEntity (and the
 * FaceEntity below), SolidMaterial, SolidTexture, SkySphere, Camera and ExposureBuffer.  This
 * module reads them (duck-typed: no reference code is imported), flattens the octree once
 * (`invalidate_scene()` re-flattens after the tree changed), and calls the N-API addon, which
 * calls librt_amd.so (include/rt.h).  There is no CPU fallback: a missing addon or GPU throws.
 *
 * Node >= 12, CommonJS, no `??` / `?.` (the image's Node is v12).
 */
'use strict';

const path = require('path');

let addon = null;
function load_addon() {
	if (addon) return addon;
	const p = process.env.RT_NAPI_PATH || path.join(__dirname, 'build', 'rt_napi.node');
	try {
		addon = require(p);
	} catch (e) {
		const err = new Error('raytracer.js_amd: N-API addon not loadable (' + p + '): ' + e.message +
			' — build it with `make -C raytracer.js_amd/js`');
		err.code = 'RT_E_NOADDON';
		throw err;
	}
	return addon;
}

const RT_ENT_SPHERE = 0, RT_ENT_BOX = 1, RT_ENT_FACE = 2;

function vec(v) {                       // math/vector.ts Vector {v: number[]} or a plain array
	return Array.isArray(v) ? v : v.v;
}

/* ---- entity / material / texture introspection (duck-typed on the reference classes) ---------- */

function entity_kind(e) {
	if (e && e.is_face_entity === true) return RT_ENT_FACE;
	if (e && typeof e.get_diameter === 'function') return RT_ENT_SPHERE;          // SphereEntity
	if (e && typeof e.get_size === 'function' && typeof e.get_faces === 'function') return RT_ENT_BOX;  // BoxEntity
	const err = new Error('raytracer.js_amd: unsupported entity type for the GPU path: ' +
		(e && e.constructor ? e.constructor.name : String(e)));
	err.code = 'RT_E_UNSUPPORTED';
	throw err;
}

function solid_color(tex, what) {
	// SolidTexture.get_size() is undefined (src/texture/texture_solid.ts:37-39), as is an
	// ImageTexture's (loaded ones are handled by loaded_image; an unloaded one shows its fallback
	// colour through get_color).
	if (!tex || typeof tex.get_color !== 'function' || (typeof tex.get_size === 'function' && tex.get_size() !== undefined)) {
		const err = new Error('raytracer.js_amd: only SolidTexture is supported on the GPU path (' + what + ')');
		err.code = 'RT_E_UNSUPPORTED';
		throw err;
	}
	const c = tex.get_color(0, 0);
	return [c.r, c.g, c.b];
}

/* ImageTexture after loading (src/texture/texture_image.ts:75-124): image_data holds the canvas
 * bytes / 255.0, width x height texels of 3 values.  Before loading get_color returns the fallback
 * colour, which the solid path handles. */
function loaded_image(tex) {
	return !!tex && tex.image_data != undefined && typeof tex.width === 'number' && typeof tex.height === 'number';
}

const image_bytes_cache = new WeakMap();
function image_bytes(tex) {                     // the bytes back from image_data (exact: round(b / 255 * 255) = b)
	const c = image_bytes_cache.get(tex);
	if (c && c.data === tex.image_data) return c.bytes;
	const n = tex.width * tex.height * 3;
	if (tex.image_data.length < n) {
		const err = new Error('raytracer.js_amd: ImageTexture image_data shorter than width*height*3');
		err.code = 'RT_E_INVALID';
		throw err;
	}
	const bytes = new Uint8Array(n);
	for (let i = 0; i < n; i++) bytes[i] = Math.round(tex.image_data[i] * 255);
	image_bytes_cache.set(tex, { data: tex.image_data, bytes });
	return bytes;
}

function material_fields(m) {
	// StaticMaterial (src/material.ts:67-103): point-independent response / mirror / light.
	const ORIGIN = { v: [0, 0, 0] };
	const resp = typeof m.response_type === 'function' ? m.response_type(ORIGIN) : m.response;
	return {
		response: resp | 0,
		light: (typeof m.is_light_source === 'function' ? m.is_light_source() : m.light_source) ? 1 : 0,
		mirror: (typeof m.is_mirror === 'function' ? m.is_mirror(ORIGIN) : m.mirror) ? 1 : 0,
		roughness: +m.roughness_index
	};
}

/* ---- scene flattening ------------------------------------------------------------------------- */

/**
 * Flatten an EntityOtree (the root the Raytracer holds) into the rt_scene_desc arrays: nodes in DFS
 * pre-order with children 0..7 (Octree.get, src/octree.ts:51-54), each node's EntitySet in
 * insertion order (src/octree_entity.ts:32-49).  Returns {arrays..., entities, substances}.
 * With `prev` (an earlier result for the same Raytracer), entity, shade and substance indices stay
 * stable — known objects keep their index, new ones are appended — which rt_update_scene needs to
 * send only what changed.
 */
function serialize_scene(otree, default_substance, prev, sky_texture) {
	if (otree.parent != undefined) {
		const err = new Error('raytracer.js_amd: the Raytracer octree has a parent (it grew outward); not supported');
		err.code = 'RT_E_UNSUPPORTED';
		throw err;
	}
	const nodes = [];
	const stack = [otree];
	while (stack.length) {                           // iterative DFS pre-order
		const t = stack.pop();
		t.__rt_id = nodes.length;
		nodes.push(t);
		for (let c = 7; c >= 0; c--) {
			const ch = t.get(c);
			if (ch != undefined) stack.push(ch);
		}
	}
	const n = nodes.length;
	const node_pos = new Float64Array(3 * n), node_size = new Float64Array(n);
	const node_parent = new Int32Array(n), node_child = new Int32Array(8 * n).fill(-1);
	const node_ent_begin = new Int32Array(n), node_ent_count = new Int32Array(n);
	const entities = prev ? prev.entities.slice() : [], list = [];
	const ent_index = prev ? new Map(prev._maps.ent_index) : new Map();
	const substances = prev ? prev.substances.slice() : [];
	const images = prev ? prev._maps.images.slice() : [];
	const image_index = prev ? new Map(prev._maps.image_index) : new Map();
	const image_of = (tex) => {                  // rt_shade.image / sky_image: 1-based, 0 = solid
		if (!loaded_image(tex)) return 0;
		if (!image_index.has(tex)) { images.push(tex); image_index.set(tex, images.length); }
		return image_index.get(tex);
	};
	const sub_index = prev ? new Map(prev._maps.sub_index) : new Map();
	const sub_of = (s) => {
		if (s == undefined) return -1;
		if (!sub_index.has(s)) { sub_index.set(s, substances.length); substances.push(s); }
		return sub_index.get(s);
	};
	for (let k = 0; k < n; k++) {
		const t = nodes[k];
		const p = vec(t.id.pos);
		node_pos[3 * k] = p[0]; node_pos[3 * k + 1] = p[1]; node_pos[3 * k + 2] = p[2];
		node_size[k] = t.id.size;
		node_parent[k] = k === 0 ? -1 : t.parent.__rt_id;
		for (let c = 0; c < 8; c++) {
			const ch = t.get(c);
			if (ch != undefined) node_child[8 * k + c] = ch.__rt_id;
		}
		node_ent_begin[k] = list.length;
		const set = t.value ? t.value.set : undefined;
		let cnt = 0;
		if (set) {
			for (const e of set) {
				if (!ent_index.has(e)) { ent_index.set(e, entities.length); entities.push(e); }
				list.push(ent_index.get(e));
				cnt++;
			}
		}
		node_ent_count[k] = cnt;
	}
	for (const t of nodes) delete t.__rt_id;

	const ne = entities.length;
	const ent_type = new Int32Array(ne), ent_geom = new Float64Array(9 * ne);
	const ent_shade = new Int32Array(ne), ent_substance = new Int32Array(ne);
	const shades = prev ? prev._maps.shades.slice() : [];
	const shade_index = new Map();
	if (prev) for (const [m, per] of prev._maps.shade_index) shade_index.set(m, new Map(per));
	for (let i = 0; i < ne; i++) {
		const e = entities[i];
		const kind = entity_kind(e);
		ent_type[i] = kind;
		const g = ent_geom.subarray(9 * i, 9 * i + 9);
		if (kind === RT_ENT_SPHERE) {
			const pos = vec(e.get_pos());
			const d = e.get_diameter();
			const sm = e.sphere_math || {};
			g[0] = pos[0]; g[1] = pos[1]; g[2] = pos[2]; g[3] = d;
			// caches exactly as the reference holds them (src/entities/entity_sphere.ts:34-39,
			// src/math/intersection.ts:94-97)
			g[4] = sm._dot_pp !== undefined ? sm._dot_pp : ((0 + pos[0] * pos[0]) + pos[1] * pos[1]) + pos[2] * pos[2];
			g[5] = sm._radius_sq !== undefined ? sm._radius_sq : (d / 2) * (d / 2);
			g[6] = e._radius_sq !== undefined ? e._radius_sq : d * d / 4;
		} else if (kind === RT_ENT_BOX) {
			const pos = vec(e.get_pos());
			g[0] = pos[0]; g[1] = pos[1]; g[2] = pos[2]; g[3] = e.get_size();
		} else {
			const vs = e.get_vertices();
			for (let j = 0; j < 3; j++) {
				const v = vec(vs[j]);
				g[3 * j] = v[0]; g[3 * j + 1] = v[1]; g[3 * j + 2] = v[2];
			}
		}
		const m = e.get_material(), tex = e.get_texture();
		let per_mat = shade_index.get(m);
		if (!per_mat) { per_mat = new Map(); shade_index.set(m, per_mat); }
		if (!per_mat.has(tex)) {
			per_mat.set(tex, shades.length);
			shades.push(null);
		}
		ent_shade[i] = per_mat.get(tex);
		ent_substance[i] = sub_of(e.get_substance());
	}
	// every (material, texture) row is re-read: a host may have edited a material in place
	for (const [m, per] of shade_index)
		for (const [tex, i] of per) {
			const image = image_of(tex);
			shades[i] = Object.assign(material_fields(m), { image, rgb: image ? [0, 0, 0] : solid_color(tex, 'entity texture') });
		}
	const sky_image = image_of(sky_texture);
	const def_sub = sub_of(default_substance);
	const ns = shades.length;
	const shade_response = new Int32Array(ns), shade_light = new Int32Array(ns), shade_mirror = new Int32Array(ns);
	const shade_roughness = new Float64Array(ns), shade_rgb = new Float64Array(3 * ns), shade_image = new Int32Array(ns);
	shades.forEach((s, i) => {
		shade_response[i] = s.response; shade_light[i] = s.light; shade_mirror[i] = s.mirror;
		shade_image[i] = s.image;
		shade_roughness[i] = s.roughness;
		shade_rgb[3 * i] = s.rgb[0]; shade_rgb[3 * i + 1] = s.rgb[1]; shade_rgb[3 * i + 2] = s.rgb[2];
	});
	const substance_ri = new Float64Array(substances.map((s) => s.refractive_index));
	return {
		node_pos, node_size, node_parent, node_child, node_ent_begin, node_ent_count,
		list_entity: new Int32Array(list), ent_type, ent_geom, ent_shade, ent_substance,
		shade_response, shade_light, shade_mirror, shade_roughness, shade_rgb, shade_image, substance_ri,
		images: images.map((t) => ({ width: t.width, height: t.height, rgb: image_bytes(t) })),
		entities, substances, default_substance_index: def_sub, sky_image,
		_maps: { ent_index, sub_index, shades, shade_index, images, image_index }
	};
}

/* ---- camera / config ---------------------------------------------------------------------------- */

/** rt_camera_desc from a reference Camera (src/view/camera.ts:50-59): the host's own cos/sin bits. */
function camera_desc(camera) {
	const conf = camera.conf;
	return {
		width: conf.screen_w, height: conf.screen_h,
		pos: vec(camera.get_pos()).slice(0, 3),
		fr: vec(camera.norm_fr).slice(0, 3), lf: vec(camera.norm_lf).slice(0, 3), up: vec(camera.norm_up).slice(0, 3),
		scan_h: vec(camera.rot_scan_h_v).slice(0, 2), scan_v: vec(camera.rot_scan_v_v).slice(0, 2)
	};
}

/* ---- the drop-in ------------------------------------------------------------------------------- */

class Raytracer {
	/** Same signature as the reference (src/raytracer.ts:291-298); `options.device` picks the GPU, or
	 * `options.devices` (e.g. [0,1,2,3,4,5,6,7]) splits every frame over several GPUs of the node:
	 * 8-row stripes dealt round-robin (`options.stripe_rows`), each GPU holding a replica of the
	 * scene, the parts gathered on devices[0] over RCCL and copied into the ebuffer once.
	 * `options.scatter === 'counter'` renders rough mirrors with the counter-based RNG (include/rt.h
	 * RT_SCATTER_COUNTER), keyed each frame by one draw of this Raytracer's rng; otherwise they are
	 * rejected (RT_E_UNSUPPORTED), as scatter_ray's sequential PRNG cannot be reproduced in parallel.
	 * `options.stats` fills `last_stats` with the frame's work counters (segments, walker steps,
	 * entity tests); counting runs the slower fused kernel, so without it `last_stats` holds only
	 * `frame_ms`. */
	constructor(config, otree, camera, ebuffer, rng, options) {
		this.camera = camera;
		this.ebuffer = ebuffer;
		this.otree = otree;
		this._rng = rng;
		this.config = Object.assign({}, config);
		this.options = Object.assign({ device: 0 }, options || {});
		this._ctx = null;
		this._scene = null;
		this.last_stats = null;
		this.last_hit_entity = null;
		this.last_hit_node = null;
		this.last_status = null;
	}

	set_camera(camera) { this.camera = camera; }
	set_ebuffer(ebuffer) { this.ebuffer = ebuffer; }
	get tree() { return this.otree; }
	get rng() { return this._rng; }

	/** Re-flatten the octree before the next frame (call after adding / moving entities or changing
	 * materials).  The GPU copy is then updated incrementally (rt_update_scene): only the nodes
	 * whose EntitySet or member entities changed are rebuilt and sent; `last_update` reports it. */
	invalidate_scene() { this._dirty = true; }

	/** Release the GPU context now instead of at garbage collection. */
	close() {
		if (this._ctx) { load_addon().destroy(this._ctx); this._ctx = null; }
	}

	_sync_scene() {
		const a = load_addon();
		if (!this._ctx) {
			const o = this.options;
			this._ctx = Array.isArray(o.devices) ? a.create(o.devices.map((x) => x | 0), (o.stripe_rows | 0))
				: a.create(o.device | 0);
		}
		const sky = this.config.sky.texture;
		if (this._scene && loaded_image(sky) && !this._scene._maps.image_index.has(sky)) this._dirty = true;
		if (!this._scene) {
			this._scene = serialize_scene(this.otree, this.config.default_substance, undefined, sky);
			a.uploadScene(this._ctx, this._scene);
		} else if (this._dirty) {
			this._scene = serialize_scene(this.otree, this.config.default_substance, this._scene, sky);
			this.last_update = a.updateScene(this._ctx, this._scene);
		}
		this._dirty = false;
		return this._scene;
	}

	/** Render one frame into the ExposureBuffer (src/raytracer.ts:308-330). */
	trace_frame() {
		const a = load_addon();
		const scene = this._sync_scene();
		const cam = camera_desc(this.camera);
		const eb = this.ebuffer;
		if (eb.width !== cam.width || eb.height !== cam.height) {
			throw Error('x or y out of bounds');                       // ExposureBuffer.check_bounds
		}
		const cfg = {
			refmax: this.config.refmax,
			default_substance: scene.default_substance_index,
			sky_image: loaded_image(this.config.sky.texture) ? scene._maps.image_index.get(this.config.sky.texture) : 0,
			sky_rgb: loaded_image(this.config.sky.texture) ? [0, 0, 0] : solid_color(this.config.sky.texture, 'sky'),
			distance_attenuation_factor: this.config.distance_attenuation_factor,
			col_weight: eb.col_weight
		};
		if (this.options.scatter === 'counter') {
			cfg.scatter_mode = 1;
			cfg.scatter_seed = Math.floor(this._rng.next() * 9007199254740992);   // one draw per frame
		}
		const P = cam.width * cam.height;
		if (this.options.keep_ids) {
			if (!this.last_hit_entity || this.last_hit_entity.length !== P) {
				this.last_hit_entity = new Int32Array(P);
				this.last_hit_node = new Int32Array(P);
				this.last_status = new Uint8Array(P);
			}
			this.last_stats = a.traceFrame(this._ctx, cam, cfg, eb.pixels, this.last_hit_entity,
				this.last_hit_node, this.last_status, !!this.options.stats);
		} else {
			this.last_stats = a.traceFrame(this._ctx, cam, cfg, eb.pixels, null, null, null, !!this.options.stats);
		}
		if (typeof eb.clean_cache === 'function') eb.clean_cache();  // set_color_i invalidates the stats cache
	}
}

/* ---- FaceEntity: the triangle entity (fills src/entities/entity_face.ts, DESIGN.md §Triangle) ---- */

function v3(x, y, z) { return { v: [x, y, z] }; }
function dot(a, b) { let s = 0; s += a[0] * b[0]; s += a[1] * b[1]; s += a[2] * b[2]; return s; }
function cross(a, b) {
	return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]];
}

class FaceEntity {
	/** (entity_otree, material, texture, substance, v0, v1, v2) — the BasicEntity argument order
	 * (src/entities/entity_basic.ts:30-36) with three vertices in place of one position. */
	constructor(entity_otree, material, texture, substance, v0, v1, v2) {
		this._octree = entity_otree;             // Entity ctor (src/entity.ts:45-48): not added to the set
		this.substance = substance;
		this.material = material;
		this.texture = texture;
		this.v0 = vec(v0).slice(0, 3); this.v1 = vec(v1).slice(0, 3); this.v2 = vec(v2).slice(0, 3);
		this.is_face_entity = true;
	}
	set_octree(tree, flags) {                    // Entity.set_octree (src/entity.ts:50-56)
		flags = flags || {};
		if (!flags.keep_in_current && this._octree != undefined) this._octree.value.set.delete(this);
		this._octree = tree;
		tree.value.set.add(this);
	}
	get octree() { return this._octree; }
	get_substance() { return this.substance; }
	set_substance(s) { const o = this.substance; this.substance = s; return o; }
	get_vertices() { return [v3.apply(null, this.v0), v3.apply(null, this.v1), v3.apply(null, this.v2)]; }
	get_pos() {                                  // centroid
		const c = [0, 1, 2].map((i) => (this.v0[i] + this.v1[i] + this.v2[i]) / 3);
		return v3(c[0], c[1], c[2]);
	}
	_set_pos(p) {                                // translate so the centroid lands on p
		const old = this.get_pos();
		const d = [0, 1, 2].map((i) => vec(p)[i] - old.v[i]);
		for (const v of [this.v0, this.v1, this.v2]) for (let i = 0; i < 3; i++) v[i] += d[i];
		return old;
	}
	get_material() { return this.material; }
	set_material(m) { const o = this.material; this.material = m; return o; }
	get_texture() { return this.texture; }
	set_texture(t) { const o = this.texture; this.texture = t; return o; }
	is_within(_p) { return false; }
	/** [min corner, max extent] — a cube, as Entity.get_aabb requires (src/entity.ts:94-96). */
	get_aabb() {
		const mn = [0, 1, 2].map((i) => Math.min(Math.min(this.v0[i], this.v1[i]), this.v2[i]));
		const mx = [0, 1, 2].map((i) => Math.max(Math.max(this.v0[i], this.v1[i]), this.v2[i]));
		const ext = [0, 1, 2].map((i) => mx[i] - mn[i]);
		return [v3(mn[0], mn[1], mn[2]), Math.max(Math.max(ext[0], ext[1]), ext[2])];
	}
	map_uv(_p) { return [0, 0]; }
	/** Fixed-order binary64 Moller-Trumbore; FORWARD t >= 0; normal faces the incoming ray. */
	collision_info(ray) {
		const o = vec(ray.get_pos()), d = vec(ray.get_dir());
		const g0 = this.v0;
		const e1 = [0, 1, 2].map((i) => this.v1[i] - g0[i]);
		const e2 = [0, 1, 2].map((i) => this.v2[i] - g0[i]);
		const pv = cross(d, e2);
		const det = dot(e1, pv);
		if (!(det != 0)) return null;
		const inv = 1 / det;
		const tv = [o[0] - g0[0], o[1] - g0[1], o[2] - g0[2]];
		const u = dot(tv, pv) * inv;
		if (!(u >= 0 && u <= 1)) return null;
		const qv = cross(tv, e1);
		const v = dot(d, qv) * inv;
		if (!(v >= 0 && u + v <= 1)) return null;
		const t = dot(e2, qv) * inv;
		if (!(t >= 0)) return null;
		const point = v3(o[0] + d[0] * t, o[1] + d[1] * t, o[2] + d[2] * t);
		const n = cross(e1, e2);
		const il = 1.0 / Math.sqrt(dot(n, n));
		const nn = [n[0] * il, n[1] * il, n[2] * il];
		const sg = -Math.sign(dot(d, nn));
		return { point, material: this.material, texture: this.texture, normal: v3(nn[0] * sg, nn[1] * sg, nn[2] * sg) };
	}
}

module.exports = {
	Raytracer, FaceEntity, serialize_scene, camera_desc, load_addon,
	RT_ENT_SPHERE, RT_ENT_BOX, RT_ENT_FACE
};
