/*
 * refshape.js — TEST FIXTURE: plain objects laid out like the reference's scene classes
 * (Octree src/octree.ts:25-126, EntitySet src/octree_entity.ts:32-49, SphereEntity
 * src/entities/entity_sphere.ts:29-102, BoxEntity src/entities/entity_box.ts:29-108,
 * StaticMaterial src/material.ts:67-103, SolidTexture src/texture/texture_solid.ts:21-44,
 * Substance src/substance.ts, Camera src/view/camera.ts:50-59, ExposureBuffer
 * src/view/exposure_buffer.ts:26-66), with the reference's mutators (Entity.set_octree, _set_pos,
 * set_material, set_texture, set_substance, Octree.set) and a restatement of add_entity_to_octree
 * for max_out_depth 0, so tests edit a live scene the way a host does.  Used because the reference
 * itself is not importable here (no TypeScript toolchain) nor present on the GPU box.
 */
'use strict';
const { FaceEntity } = require('../../raytracer.js_amd/js/raytracer.js');

class Octree {
	constructor(id, parent, value) { this.id = id; this.parent = parent; this.value = value; this.nodes = Array(8).fill(undefined); }
	get(n) { if (!(n >= 0 && n <= 7)) throw Error('Node index out of range (0..7)'); return this.nodes[n]; }
	set(n, value) {                                            // src/octree.ts:56-70 (no invalidation flags)
		if (!(n >= 0 && n <= 7)) throw Error('Node index out of range (0..7)');
		const old = this.nodes[n];
		this.nodes[n] = value;
		return old;
	}
	get_level() { let l = 0; for (let t = this.parent; t != undefined; t = t.parent) l++; return l; }
}
class EntitySet { constructor() { this._set = new Set(); } get set() { return this._set; } }
class Substance { constructor(ri) { this.refractive_index = ri; } }
class SolidTexture {
	constructor(c) { this.color = c; }
	get_color(_u, _v) { return this.color; }
	get_size() { return undefined; }
}
class ImageTexture {                       // a loaded ImageTexture: image_data = bytes / 255.0
	constructor(width, height, bytes) {
		this.width = width; this.height = height;
		this.image_data = Array.from(bytes, (b) => b / 255.0);
		this.fallback_color = { r: 1, g: 0, b: 1, a: 1 };
	}
	get_color(u, v) {
		if (u < 0 - Number.EPSILON || u > 1 - Number.EPSILON || v < 0 - Number.EPSILON || v > 1 - Number.EPSILON)
			throw Error('Texture coordinates out of bounds');
		const i = (((v * this.height) << 0) * this.width + ((u * this.width) << 0)) * 3;
		return { r: this.image_data[i], g: this.image_data[i + 1], b: this.image_data[i + 2], a: 1.0 };
	}
	get_size() { return undefined; }
}
class SolidMaterial {
	constructor(response, light, mirror, roughness) { this.response = response; this.light_source = light; this.mirror = mirror; this.roughness_index = roughness; }
	response_type(_) { return this.response; }
	is_mirror(_) { return this.mirror; }
	is_light_source() { return this.light_source; }
}
class Entity {                                               // src/entity.ts:38-71: the octree link
	set_octree(tree, flags) {
		if (!(flags && flags.keep_in_current) && this._octree != undefined) this._octree.value.set.delete(this);
		this._octree = tree;
		tree.value.set.add(this);
	}
	get octree() { return this._octree; }
	set_substance(s) { const old = this.substance; this.substance = s; return old; }
}
class BasicShape extends Entity {                           // src/entities/entity_basic.ts:25-57
	constructor(material, texture, substance, pos) { super(); this.material = material; this.texture = texture; this.substance = substance; this.pos = { v: pos }; this._octree = undefined; }
	get_pos() { return this.pos; }
	_set_pos(p) { const old = this.pos; this.pos = p; return old; }
	get_material() { return this.material; }
	set_material(m) { const old = this.material; this.material = m; return old; }
	get_texture() { return this.texture; }
	set_texture(t) { const old = this.texture; this.texture = t; return old; }
	get_substance() { return this.substance; }
}
class SphereEntity extends BasicShape {
	constructor(m, t, s, pos, d) {
		super(m, t, s, pos);
		this.diameter = d;
		const r = d / 2;
		this.sphere_math = { _pos: this.pos, _radius: r, _dot_pp: ((0 + pos[0] * pos[0]) + pos[1] * pos[1]) + pos[2] * pos[2], _radius_sq: r * r };
		this._radius_sq = d * d / 4;
	}
	get_diameter() { return this.diameter; }
	_set_pos(p) {                                           // entity_sphere.ts:55-60 + Sphere's pos setter (intersection.ts:94-97)
		const old = this.pos;
		this.pos = p;
		this.sphere_math._pos = p;
		this.sphere_math._dot_pp = ((0 + p.v[0] * p.v[0]) + p.v[1] * p.v[1]) + p.v[2] * p.v[2];
		return old;
	}
	get_aabb() {                                            // entity_sphere.ts:90-96
		const d = this.diameter, p = this.pos.v;
		return [{ v: [p[0] - d * 0.5, p[1] - d * 0.5, p[2] - d * 0.5] }, d];
	}
}
class BoxEntity extends BasicShape {
	constructor(m, t, s, pos, size) { super(m, t, s, pos); this.size = size; }
	get_size() { return this.size; }
	get_faces() { return []; }
	get_aabb() { const h = this.size / 2, p = this.pos.v; return [{ v: [p[0] - h, p[1] - h, p[2] - h] }, this.size]; }
}

/* add_entity_to_octree (src/octree_entity.ts:56-113, 174-188) for a tree that never grows outward
 * (max_out_depth 0): the deepest node covering the entity's AABB (node_at_pos of its corner,
 * src/octree_space.ts:61-93, then up until the AABB fits, src/space.ts:82-103), extended inward
 * while a child octant still covers it, then Entity.set_octree. */
function aabb_fits(pos, size, t) {
	const q = t.id.pos.v, s = t.id.size;
	for (let i = 0; i < 3; i++) if (!(pos[i] >= q[i] && pos[i] + size <= q[i] + s)) return false;
	return true;
}
function add_entity_to_octree(root, e, flags) {
	const [corner, size] = e.get_aabb();
	const a = corner.v, rp = root.id.pos.v, rs = root.id.size;
	let t;
	if (a[0] >= rp[0] && a[0] < rp[0] + rs && a[1] >= rp[1] && a[1] < rp[1] + rs && a[2] >= rp[2] && a[2] < rp[2] + rs) {
		let pos = rp.slice(), sz = rs, next = root;
		while (next != undefined) {                           // node_at_pos
			t = next;
			const ix = ((a[0] - pos[0]) * (2 / sz)), iy = ((a[1] - pos[1]) * (2 / sz)), iz = ((a[2] - pos[2]) * (2 / sz));
			next = t.get((iz << 2) + (iy << 1) + (ix << 0));
			sz /= 2;
			pos = [pos[0] + (ix << 0) * sz, pos[1] + (iy << 0) * sz, pos[2] + (iz << 0) * sz];
		}
		while (t != undefined && !aabb_fits(a, size, t)) t = t.parent;
	}
	if (t == undefined) throw Error('the entity does not fit the tree (max_out_depth 0)');
	for (let depth = t.get_level() - root.get_level(); depth < flags.max_in_depth; depth++) {
		const q = t.id.pos.v, s = t.id.size;
		const x = ((a[0] - q[0]) * (2.0 / s)) << 0, y = ((a[1] - q[1]) * (2.0 / s)) << 0, z = ((a[2] - q[2]) * (2.0 / s)) << 0;
		const sp = [q[0] + x * (s / 2), q[1] + y * (s / 2), q[2] + z * (s / 2)];
		const child = { id: { pos: { v: sp }, size: s / 2 } };
		if (!aabb_fits(a, size, child)) break;
		const n = new Octree({ pos: { v: sp }, size: s / 2 }, t, new EntitySet());
		t.set((z << 2) | (y << 1) | (x << 0), n);
		t = n;
	}
	e.set_octree(t);
	return t;
}

/** Inflate a linearised scene (tests write it as JSON) into reference-shaped objects. */
function inflate(sc) {
	const n = sc.node_size.length;
	const nodes = [];
	for (let k = 0; k < n; k++) {
		const p = sc.node_pos.slice(3 * k, 3 * k + 3);
		nodes.push(new Octree({ pos: { v: p }, size: sc.node_size[k] }, undefined, new EntitySet()));
	}
	for (let k = 0; k < n; k++) {
		for (let c = 0; c < 8; c++) {
			const ch = sc.node_child[8 * k + c];
			if (ch >= 0) { nodes[k].nodes[c] = nodes[ch]; nodes[ch].parent = nodes[k]; }
		}
	}
	const subs = sc.substance_ri.map((ri) => new Substance(ri));
	const images = (sc.images || []).map((im) => new ImageTexture(im.width, im.height, im.rgb));
	const mats = new Map();
	const ents = [];
	for (let i = 0; i < sc.ent_type.length; i++) {
		const s = sc.shades[sc.ent_shade[i]];
		const key = [s.response, s.light, s.mirror, s.roughness].join(',');
		if (!mats.has(key)) mats.set(key, new SolidMaterial(s.response, !!s.light, !!s.mirror, s.roughness));
		const mat = mats.get(key);
		const tex = s.image ? images[s.image - 1] : new SolidTexture({ r: s.rgb[0], g: s.rgb[1], b: s.rgb[2], a: 1.0 });
		const sub = sc.ent_substance[i] >= 0 ? subs[sc.ent_substance[i]] : undefined;
		const g = sc.ent_geom.slice(9 * i, 9 * i + 9);
		let e;
		if (sc.ent_type[i] === 0) e = new SphereEntity(mat, tex, sub, g.slice(0, 3), g[3]);
		else if (sc.ent_type[i] === 1) e = new BoxEntity(mat, tex, sub, g.slice(0, 3), g[3]);
		else e = new FaceEntity(undefined, mat, tex, sub, g.slice(0, 3), g.slice(3, 6), g.slice(6, 9));
		e.__orig_id = i;
		ents.push(e);
	}
	for (let k = 0; k < n; k++) {
		const b = sc.node_ent_begin[k], c = sc.node_ent_count[k];
		for (let j = b; j < b + c; j++) {
			nodes[k].value.set.add(ents[sc.list_entity[j]]);
			ents[sc.list_entity[j]]._octree = nodes[k];
		}
	}
	return { root: nodes[0], nodes, entities: ents, substances: subs, images };
}

/** Camera-shaped object from an rt_camera_desc-like record. */
function camera(c) {
	return {
		conf: { screen_w: c.width, screen_h: c.height }, pos: { v: c.pos.slice() },
		norm_fr: { v: c.fr.slice() }, norm_lf: { v: c.lf.slice() }, norm_up: { v: c.up.slice() },
		rot_scan_h_v: { v: c.scan_h.slice() }, rot_scan_v_v: { v: c.scan_v.slice() },
		get_pos() { return this.pos; }
	};
}

class ExposureBuffer {
	constructor(w, h) { this.pixels = new Float32Array(w * h * 3); this.width = w; this.height = h; this.col_weight = 1; this.cleaned = 0; }
	clean_cache() { this.cleaned++; }
}

module.exports = { ImageTexture, inflate, camera, ExposureBuffer, SolidTexture, Substance, SphereEntity, BoxEntity,
	SolidMaterial, Octree, EntitySet, add_entity_to_octree };
