/*
 * refshape.js — TEST FIXTURE: plain objects laid out like the reference's scene classes
 * (Octree src/octree.ts:25-126, EntitySet src/octree_entity.ts:32-49, SphereEntity
 * src/entities/entity_sphere.ts:29-102, BoxEntity src/entities/entity_box.ts:29-108,
 * StaticMaterial src/material.ts:67-103, SolidTexture src/texture/texture_solid.ts:21-44,
 * Substance src/substance.ts, Camera src/view/camera.ts:50-59, ExposureBuffer
 * src/view/exposure_buffer.ts:26-66).  Field names only — no reference code.  Used because the
 * reference itself is not importable here (no TypeScript toolchain) nor present on the GPU box.
 */
'use strict';
const { FaceEntity } = require('../../raytracer.js_amd/js/raytracer.js');

class Octree {
	constructor(id, parent, value) { this.id = id; this.parent = parent; this.value = value; this.nodes = Array(8).fill(undefined); }
	get(n) { if (!(n >= 0 && n <= 7)) throw Error('Node index out of range (0..7)'); return this.nodes[n]; }
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
class BasicShape {
	constructor(material, texture, substance, pos) { this.material = material; this.texture = texture; this.substance = substance; this.pos = { v: pos }; }
	get_pos() { return this.pos; }
	get_material() { return this.material; }
	get_texture() { return this.texture; }
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
}
class BoxEntity extends BasicShape {
	constructor(m, t, s, pos, size) { super(m, t, s, pos); this.size = size; }
	get_size() { return this.size; }
	get_faces() { return []; }
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
		for (let j = b; j < b + c; j++) nodes[k].value.set.add(ents[sc.list_entity[j]]);
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

module.exports = { ImageTexture, inflate, camera, ExposureBuffer, SolidTexture, Substance };
