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

	const ne = entities.length;
	const ent_type = new Int32Array(ne), ent_geom = new Float64Array(9 * ne);
	const ent_shade = new Int32Array(ne), ent_substance = new Int32Array(ne);
	const shades = prev ? prev._maps.shades.slice() : [];
	const shade_index = new Map();
	if (prev) for (const [m, per] of prev._maps.shade_index) shade_index.set(m, new Map(per));
	for (const t of nodes) delete t.__rt_id;
	for (let i = 0; i < ne; i++) {
		const e = entities[i];
		ent_type[i] = entity_geom(e, ent_geom.subarray(9 * i, 9 * i + 9));
		ent_shade[i] = shade_row(shade_index, shades, e);
		ent_substance[i] = sub_of(e.get_substance());
	}
	const tables = shade_tables(shades, shade_index, image_of);
	const sky_image = image_of(sky_texture);
	const def_sub = sub_of(default_substance);
	const substance_ri = new Float64Array(substances.map((s) => s.refractive_index));
	return Object.assign({
		node_pos, node_size, node_parent, node_child, node_ent_begin, node_ent_count,
		list_entity: new Int32Array(list), ent_type, ent_geom, ent_shade, ent_substance, substance_ri,
		images: images.map((t) => ({ width: t.width, height: t.height, rgb: image_bytes(t) })),
		entities, substances, default_substance_index: def_sub, sky_image,
		_maps: { ent_index, sub_index, shades, shade_index, images, image_index, sub_of },
		_nodes: nodes
	}, tables);
}

/** rt_scene_desc's ent_type / ent_geom record of entity e: its RT_ENT_* kind, geometry into g[0..8]. */
function entity_geom(e, g) {
	const kind = entity_kind(e);
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
	return kind;
}

/** The shade row of e's (material, texture) pair; a new pair gets the next row (filled by shade_tables). */
function shade_row(shade_index, shades, e) {
	const m = e.get_material(), tex = e.get_texture();
	let per_mat = shade_index.get(m);
	if (!per_mat) { per_mat = new Map(); shade_index.set(m, per_mat); }
	if (!per_mat.has(tex)) {
		per_mat.set(tex, shades.length);
		shades.push(null);
	}
	return per_mat.get(tex);
}

/** Every (material, texture) row re-read (a host may have edited a material in place), as the
 * shade_* arrays of rt_scene_desc. */
function shade_tables(shades, shade_index, image_of) {
	for (const [m, per] of shade_index)
		for (const [tex, i] of per) {
			const image = image_of(tex);
			shades[i] = Object.assign(material_fields(m), { image, rgb: image ? [0, 0, 0] : solid_color(tex, 'entity texture') });
		}
	const ns = shades.length;
	const t = {
		shade_response: new Int32Array(ns), shade_light: new Int32Array(ns), shade_mirror: new Int32Array(ns),
		shade_roughness: new Float64Array(ns), shade_rgb: new Float64Array(3 * ns), shade_image: new Int32Array(ns)
	};
	shades.forEach((s, i) => {
		t.shade_response[i] = s.response; t.shade_light[i] = s.light; t.shade_mirror[i] = s.mirror;
		t.shade_image[i] = s.image;
		t.shade_roughness[i] = s.roughness;
		t.shade_rgb[3 * i] = s.rgb[0]; t.shade_rgb[3 * i + 1] = s.rgb[1]; t.shade_rgb[3 * i + 2] = s.rgb[2];
	});
	return t;
}

/* ---- O(edit) scene updates: a journal over the reference's own mutators ---------------------------- */
// The reference edits a scene through a handful of methods: Entity.set_octree (EntitySet delete /
// add, src/entity.ts:50-56; add_entity_to_octree calls it, src/octree_entity.ts:174-188), Octree.set
// (new nodes, src/octree.ts:56-70; add_entity_to_octree's tree extension) and the entity setters
// (_set_pos, set_material, set_texture: src/entities/entity_basic.ts:38-57; set_substance:
// src/entity.ts:67-71; set_diameter: entity_sphere.ts:45-60; set_size: entity_box.ts:37).  Each is
// wrapped once, on the prototype that defines it (the reference's code is not changed, and no
// per-object state is added to entities); the wrapper notes the object in every live Raytracer's
// journal before the original runs.  invalidate_scene() then sends only the noted nodes and the sets
// holding noted entities (rt_apply_edit), not the whole scene.
// A Raytracer that is dropped without close() cannot be seen going away on Node 12 (no WeakRef), so a
// journal bounds itself: past `cap` noted objects it forgets them and marks itself `over`, which
// makes its Raytracer's next sync a full re-read, and every later mutator call skips it.  Where
// FinalizationRegistry exists, a collected Raytracer's journal also leaves JOURNALS.
const JOURNALS = new Set();
const JOURNAL_GC = typeof FinalizationRegistry === 'function' ? new FinalizationRegistry((j) => JOURNALS.delete(j)) : null;
const WRAPPED = Symbol('rt_journal_wrapped');
const ENTITY_MUTATORS = ['_set_pos', 'set_material', 'set_texture', 'set_substance', 'set_diameter', 'set_size'];

function entity_node(e) { return e._octree !== undefined ? e._octree : e.octree; }

function wrap_method(obj, name, note) {
	let p = Object.getPrototypeOf(obj);
	while (p && p !== Object.prototype && !Object.prototype.hasOwnProperty.call(p, name)) p = Object.getPrototypeOf(p);
	if (!p || p === Object.prototype || typeof p[name] !== 'function' || p[name][WRAPPED]) return;
	const orig = p[name];
	const w = function () {
		if (JOURNALS.size) for (const j of JOURNALS) if (!j.over) {
			note(j, this, arguments);
			if (j.nodes.size + j.ents.size + j.struct.size > j.cap) {
				j.over = true;
				j.nodes.clear(); j.ents.clear(); j.struct.clear();
			}
		}
		return orig.apply(this, arguments);
	};
	w[WRAPPED] = true;
	Object.defineProperty(p, name, { value: w, writable: true, configurable: true, enumerable: false });
}

function journal_classes(node, entity) {
	if (node) wrap_method(node, 'set', (j, t) => j.struct.add(t));
	if (entity) {
		wrap_method(entity, 'set_octree', (j, e, args) => {
			const old = entity_node(e);
			if (old) j.nodes.add(old);
			if (args[0]) j.nodes.add(args[0]);
		});
		for (const m of ENTITY_MUTATORS) wrap_method(entity, m, (j, e) => j.ents.add(e));
	}
}

// The mutators of every entity class in `ents` (once per prototype; wrap_method skips wrapped ones)
function wrap_entity_classes(ents) {
	const seen = new Set();
	for (const e of ents) {
		const p = Object.getPrototypeOf(e);
		if (!seen.has(p)) { seen.add(p); journal_classes(null, e); }
	}
}

function grow_i32(a, n, fill) {
	if (a.length >= n) return a;
	const b = new Int32Array(Math.max(n, 2 * a.length));
	if (fill !== undefined) b.fill(fill);
	b.set(a);
	return b;
}

// index_within_parent (src/octree_space.ts:113-125), as rt_upload_scene computes it: RT_OCT_BAD (1000)
// when the geometric index is not 0..7
function octant_in_parent(t) {
	const p = t.parent, c = vec(t.id.pos), q = vec(p.id.pos), sc = 2 / p.id.size;
	const idx = (((c[2] - q[2]) * sc) << 2) + (((c[1] - q[1]) * sc) << 1) + (((c[0] - q[0]) * sc) << 0);
	return idx >= 0 && idx <= 7 ? idx : 1000;
}

/**
 * The edit since the last sync as an rt_edit_desc (include/rt.h) in resident slots, from journal j
 * and the slot state st (built at the last full sync), or null when the edit cannot be expressed
 * (a child replaced or removed, a node re-parented, a new ImageTexture, an entity whose node is
 * unknown): the caller then re-reads the whole scene.  New nodes take the next slots in DFS
 * pre-order of their subtrees; their DFS ids come from subtree sizes along their paths (O(depth)),
 * the existing nodes' ids shift on the device.  Updates st and scene._maps in place.
 */
function build_edit(scene, st, j, default_substance, sky_texture) {
	const sym = st.sym, maps = scene._maps;
	const slot = (t) => t[sym];
	// 1. structure: new subtrees under existing nodes
	const new_nodes = [], rec = new Set(), base = st.n_slots;
	for (const t of j.struct) {
		const sl = slot(t);
		if (sl === undefined || sl >= base) continue;    // a node outside the scene, or a new one (below)
		for (let c = 0; c < 8; c++) {
			const ch = t.get(c), old = st.child[8 * sl + c];
			if (ch == undefined) { if (old >= 0) return null; continue; }
			const cs = slot(ch);
			if (cs !== undefined) { if (cs !== old) return null; continue; }
			if (old >= 0 || ch.parent !== t) return null;
			const stack = [ch];
			while (stack.length) {
				const x = stack.pop();
				if (slot(x) !== undefined) return null;
				x[sym] = st.n_slots;
				st.nodes[st.n_slots++] = x;
				new_nodes.push(x);
				for (let k = 7; k >= 0; k--) {
					const y = x.get(k);
					if (y != undefined) { if (y.parent !== x) return null; stack.push(y); }
				}
			}
			rec.add(sl);
		}
	}
	st.child = grow_i32(st.child, 8 * st.n_slots, -1);
	st.sub = grow_i32(st.sub, st.n_slots);
	for (const x of new_nodes) {
		const sx = slot(x);
		for (let c = 0; c < 8; c++) {
			const y = x.get(c);
			st.child[8 * sx + c] = y != undefined ? slot(y) : -1;
		}
		rec.add(sx);
	}
	for (const t of rec) {                              // parents that gained a child
		const x = st.nodes[t];
		for (let c = 0; c < 8; c++) {
			const y = x.get(c);
			st.child[8 * t + c] = y != undefined ? slot(y) : -1;
		}
	}
	// DFS ids of the new nodes: subtree sizes first (every new node counts on its whole path)
	for (const x of new_nodes) {
		st.sub[slot(x)] = 0;
	}
	for (const x of new_nodes)
		for (let y = x; y != undefined; y = y.parent) st.sub[slot(y)] += 1;
	const dfs_new_slot = new Int32Array(new_nodes.length), dfs_new_val = new Int32Array(new_nodes.length);
	new_nodes.forEach((x, i) => {
		let id = 0;
		for (let y = x; y.parent != undefined; y = y.parent) {
			const p = y.parent;
			id += 1;
			for (let c = 0; c < 8; c++) {
				const z = p.get(c);
				if (z === y) break;
				if (z != undefined) id += st.sub[slot(z)];
			}
		}
		dfs_new_slot[i] = slot(x);
		dfs_new_val[i] = id;
	});
	const F = Array.from(dfs_new_val).sort((a, b) => a - b);
	const dfs_shift = Int32Array.from(F, (f, k) => f - k);
	// 2. node records, ascending slots
	const rec_slot = Int32Array.from(Array.from(rec).sort((a, b) => a - b));
	const nr = rec_slot.length;
	const rec_cube = new Float64Array(4 * nr), rec_child = new Int32Array(8 * nr), rec_up = new Int32Array(2 * nr);
	for (let k = 0; k < nr; k++) {
		const sl = rec_slot[k], x = st.nodes[sl], p = vec(x.id.pos);
		rec_cube[4 * k] = p[0]; rec_cube[4 * k + 1] = p[1]; rec_cube[4 * k + 2] = p[2]; rec_cube[4 * k + 3] = x.id.size;
		for (let c = 0; c < 8; c++) rec_child[8 * k + c] = st.child[8 * sl + c];
		const root = sl === 0;
		rec_up[2 * k] = root ? -1 : slot(x.parent);
		rec_up[2 * k + 1] = root ? -1 : octant_in_parent(x);
	}
	// 3. dirty EntitySets: noted nodes, the nodes of noted entities, every new node
	const dirty = new Set(new_nodes.map(slot));
	for (const t of j.nodes) { const sl = slot(t); if (sl !== undefined) dirty.add(sl); }
	for (const e of j.ents) {
		const t = entity_node(e);
		if (t == undefined) { if (maps.ent_index.has(e)) return null; continue; }
		const sl = slot(t);
		if (sl !== undefined) dirty.add(sl);
	}
	const set_slot = Int32Array.from(Array.from(dirty).sort((a, b) => a - b));
	const members = [];
	const set_begin = new Int32Array(set_slot.length), set_count = new Int32Array(set_slot.length);
	const new_ents = [];
	for (let k = 0; k < set_slot.length; k++) {
		const t = st.nodes[set_slot[k]];
		set_begin[k] = members.length;
		const set = t.value ? t.value.set : undefined;
		if (set) for (const e of set) {
			if (!maps.ent_index.has(e)) { maps.ent_index.set(e, scene.entities.length); scene.entities.push(e); new_ents.push(e); }
			members.push(e);
		}
		set_count[k] = members.length - set_begin[k];
	}
	const nm = members.length;
	const set_ent = new Int32Array(nm), set_type = new Int32Array(nm), set_shade = new Int32Array(nm);
	const set_geom = new Float64Array(9 * nm);
	members.forEach((e, i) => {
		set_ent[i] = maps.ent_index.get(e);
		set_type[i] = entity_geom(e, set_geom.subarray(9 * i, 9 * i + 9));
		set_shade[i] = shade_row(maps.shade_index, maps.shades, e);
	});
	// 4. substances of the noted and the new entities
	const subs = new Set();
	for (const e of j.ents) if (maps.ent_index.has(e)) subs.add(maps.ent_index.get(e));
	for (const e of new_ents) subs.add(maps.ent_index.get(e));
	const sub_ent = Int32Array.from(Array.from(subs).sort((a, b) => a - b));
	const sub_val = Int32Array.from(sub_ent, (i) => maps.sub_of(scene.entities[i].get_substance()));
	// 5. tables: every shade row re-read; a new ImageTexture needs the image table (full upload)
	const no_new_image = (tex) => {
		if (!loaded_image(tex)) return 0;
		if (!maps.image_index.has(tex)) throw NEW_IMAGE;
		return maps.image_index.get(tex);
	};
	let tables;
	try {
		tables = shade_tables(maps.shades, maps.shade_index, no_new_image);
		no_new_image(sky_texture);
	} catch (err) {
		if (err !== NEW_IMAGE) throw err;
		return null;                                     // (rows added above are filled by the full path)
	}
	maps.sub_of(default_substance);
	// rough mirrors listed (rt_create's scatter gate): a row in use by a member of any set
	st.ent_shade = grow_i32(st.ent_shade, scene.entities.length, -1);
	for (let i = 0; i < nm; i++) st.ent_shade[set_ent[i]] = set_shade[i];
	let scatter = 0;
	const rough = maps.shades.map((r) => !r.light && r.response === 0 && r.mirror && r.roughness > 0);
	if (rough.some((x) => x))
		for (let i = 0; i < scene.entities.length && !scatter; i++)
			if (st.ent_shade[i] >= 0 && rough[st.ent_shade[i]] && entity_node(scene.entities[i]) != undefined) scatter = 1;
	return Object.assign({
		new_ents,                                        // (not read by the addon) their classes get journaled
		n_slots: st.n_slots, n_entities: scene.entities.length,
		rec_slot, rec_cube, rec_child, rec_up, set_slot, set_begin, set_count, set_ent, set_type, set_shade, set_geom,
		sub_ent, sub_val, dfs_new_slot, dfs_new_val, dfs_shift, scatter,
		substance_ri: new Float64Array(scene.substances.map((x) => x.refractive_index))
	}, tables);
}
const NEW_IMAGE = { rt_new_image: true };

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
	 * `frame_ms`.
	 * `options.lights` ([{pos, rgb}], pos a vector3 or [x, y, z]) and `options.ambient` turn on shadow
	 * rays, a BUILD EXTENSION the reference does not have (include/rt.h rt_set_lights, DESIGN.md §3.6);
	 * `set_lights()` changes them between frames, and no lights (the default) is the reference. */
	constructor(config, otree, camera, ebuffer, rng, options) {
		this.camera = camera;
		this.ebuffer = ebuffer;
		this.otree = otree;
		this._rng = rng;
		this.config = Object.assign({}, config);
		this.options = Object.assign({ device: 0 }, options || {});
		this._ctx = null;
		this._scene = null;
		this._journal = null;           // edits noted since the last sync (JOURNALS)
		this._st = null;                // resident slots of the scene's nodes (build_edit)
		this._sym = Symbol('rt_slot');  // this Raytracer's slot property on the octree's nodes
		this._full = false;
		this.last_stats = null;
		this.last_hit_entity = null;
		this.last_hit_node = null;
		this.last_status = null;
		this._lights = null;            // shadow rays: the last light list (null: none set)
		this._lights_sent = null;       // the context _lights went to (a new context gets them again)
		if (this.options.lights) this.set_lights(this.options.lights, this.options.ambient);
	}

	/** Shadow rays (build extension): point lights [{pos, rgb}] and the ambient term; [] turns them off. */
	set_lights(lights, ambient) {
		const vec = (p) => (p && p.v ? p.v : p);
		this._lights = { list: (lights || []).map((l) => ({ pos: Array.from(vec(l.pos)), rgb: Array.from(vec(l.rgb)) })),
			ambient: +(ambient || 0) };
		this._lights_sent = null;
	}

	set_camera(camera) { this.camera = camera; }
	set_ebuffer(ebuffer) { this.ebuffer = ebuffer; }
	get tree() { return this.otree; }
	get rng() { return this._rng; }

	/** Bring the GPU copy of the scene up to date before the next frame (call after adding / moving
	 * entities or changing materials).  Edits made through the reference's own mutators
	 * (add_entity_to_octree, Entity.set_octree / _set_pos / set_material / set_texture /
	 * set_substance / set_diameter / set_size, Octree.set) are journaled as they happen, and only
	 * the nodes and EntitySets they touched are read and sent (rt_apply_edit, O(edit)).
	 * `invalidate_scene({ full: true })` re-reads the whole octree instead (after direct field writes
	 * that bypass those methods); the GPU copy is then diffed and patched (rt_update_scene).
	 * `last_update` reports what was sent. */
	invalidate_scene(opts) {
		this._dirty = true;
		if (opts && opts.full) this._full = true;
	}

	/** Release the GPU context now instead of at garbage collection. */
	close() {
		if (this._journal) { JOURNALS.delete(this._journal); this._journal = null; }
		this._st = null;
		if (this._ctx) { load_addon().destroy(this._ctx); this._ctx = null; }
		this._lights_sent = null;
	}

	// After a full read of the scene: the resident slot of every node (slots: sceneSlots' map; null =
	// DFS order), subtree sizes, child slots, and a fresh journal.
	_begin_journal(slots, n_slots) {
		const sc = this._scene, n = sc.node_size.length, sym = this._sym;
		if (this._st) for (const x of this._st.nodes) if (x) delete x[sym];
		const slot = (k) => (slots ? slots[k] : k);
		// mirrors with headroom, so that the edits of many frames never copy them
		const cap = n_slots + (n_slots >> 3) + 1024, ecap = sc.ent_shade.length + (sc.ent_shade.length >> 3) + 1024;
		const st = { sym, n_slots, nodes: new Array(n_slots).fill(null), child: new Int32Array(8 * cap).fill(-1),
			sub: new Int32Array(cap), ent_shade: new Int32Array(ecap).fill(-1) };
		st.ent_shade.set(sc.ent_shade);
		for (let k = 0; k < n; k++) {
			const x = sc._nodes[k], sl = slot(k);
			x[sym] = sl;
			st.nodes[sl] = x;
			for (let c = 0; c < 8; c++) {
				const ch = sc.node_child[8 * k + c];
				st.child[8 * sl + c] = ch >= 0 ? slot(ch) : -1;
			}
		}
		for (let k = n - 1; k >= 0; k--) {             // DFS pre-order: children after their parent
			st.sub[slot(k)] += 1;
			if (k > 0) st.sub[slot(sc.node_parent[k])] += st.sub[slot(k)];
		}
		this._st = st;
		if (!this._journal) {
			this._journal = { nodes: new Set(), ents: new Set(), struct: new Set(), over: false, cap: 0 };
			JOURNALS.add(this._journal);
			if (JOURNAL_GC) JOURNAL_GC.register(this, this._journal);
		}
		const j = this._journal;
		j.nodes.clear(); j.ents.clear(); j.struct.clear();
		j.over = false;
		j.cap = Math.max(1 << 16, n_slots + sc.entities.length);
		journal_classes(this.otree, null);
		wrap_entity_classes(sc.entities);
	}

	// After rt_apply_edit took `edit`: a fresh journal, and the mutators of entity classes the last full
	// read did not see (a sphere added to a box-only scene: SphereEntity._set_pos, set_diameter) wrapped
	_edit_applied(edit) {
		wrap_entity_classes(edit.new_ents);
		const j = this._journal;
		j.nodes.clear(); j.ents.clear(); j.struct.clear();
	}

	_sync_scene() {
		const a = load_addon();
		let fresh = false;
		if (!this._ctx) {
			const o = this.options;
			this._ctx = Array.isArray(o.devices) ? a.create(o.devices.map((x) => x | 0), (o.stripe_rows | 0))
				: a.create(o.device | 0);
			fresh = true;                   // a new context (first frame, or after close()) holds no scene
		}
		const sky = this.config.sky.texture;
		if (this._scene && loaded_image(sky) && !this._scene._maps.image_index.has(sky)) this._dirty = true;
		if (!this._scene || fresh) {
			this._scene = serialize_scene(this.otree, this.config.default_substance, undefined, sky);
			a.uploadScene(this._ctx, this._scene);
			const sl = a.sceneSlots(this._ctx, this._scene.node_size.length);
			this._begin_journal(sl.slots, sl.n_slots);
		} else if (this._dirty) {
			let u = null;
			if (!this._full && this._st && !this._journal.over) {
				const t0 = process.hrtime();
				const edit = build_edit(this._scene, this._st, this._journal, this.config.default_substance, sky);
				const t1 = process.hrtime(t0);
				if (edit) u = a.applyEdit(this._ctx, edit);     // null: the store asks for a full upload
				if (u) {
					this._edit_applied(edit);
					const dt = process.hrtime(t0);
					u.build_ms = t1[0] * 1e3 + t1[1] / 1e6;        // journal -> rt_edit_desc (JS)
					u.js_ms = dt[0] * 1e3 + dt[1] / 1e6;          // ... -> applied (JS + addon + librt)
					u.via = 'edit';
				}
			}
			if (!u) {
				this._scene = serialize_scene(this.otree, this.config.default_substance, this._scene, sky);
				u = a.updateScene(this._ctx, this._scene);
				u.via = 'scene';
				const sl = a.sceneSlots(this._ctx, this._scene.node_size.length);
				if (sl) this._begin_journal(sl.slots, sl.n_slots);
				else this._st = null;
			}
			this._full = false;
			this.last_update = u;
		}
		this._dirty = false;
		return this._scene;
	}

	/** Render one frame into the ExposureBuffer (src/raytracer.ts:308-330). */
	trace_frame() {
		const a = load_addon();
		const scene = this._sync_scene();
		if (this._lights && this._lights_sent !== this._ctx) {
			// kept after sending: a context created after close() (or any new one) gets them too
			a.setLights(this._ctx, this._lights.list, this._lights.ambient);
			this._lights_sent = this._ctx;
		}
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
	RT_ENT_SPHERE, RT_ENT_BOX, RT_ENT_FACE,
	_internal: { build_edit }                 // tests/js/check_edit.js
};
