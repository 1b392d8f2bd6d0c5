/*
 * check_edit.js <scene.json> <ops.json> — CPU check of the drop-in's O(edit) path (no GPU, no addon).
 * A Raytracer's journal is started on the inflated scene as after its first frame; the ops are then
 * made through the reference's mutators; build_edit's rt_edit_desc is applied to a slot model of the
 * first linearisation (what rt_apply_edit does to the resident scene: records, sets, substances, DFS
 * ids with the shift) and the result must equal a fresh serialize_scene of the edited tree, node by
 * node in DFS order: cube, parent, children, EntitySet (entity ids, types, geometry bits, shades),
 * substances.  ops: [{op: 'move', entity, pos, depth} | {op: 'add_sphere', pos, d, depth, like} |
 * {op: 'shade', entity, like} | {op: 'substance', entity, like} | {op: 'setpos', entity, pos} |
 * {op: 'sync'}]: a 'sync' applies the
 * edit so far as a frame would (the model takes it, the Raytracer's _edit_applied starts a new
 * journal), so later ops form a second edit.  Prints 'edit ok' and a summary.
 */
'use strict';
const fs = require('fs');
const assert = require('assert');
const rs = require('./refshape.js');
const rt = require('../../raytracer.js_amd/js/raytracer.js');

const sc = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const ops = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
const world = rs.inflate(sc);
const sky = new rs.SolidTexture({ r: 0.5, g: 0.5, b: 0.5, a: 1 });
const tr = new rt.Raytracer({ refmax: 2, sky: { texture: sky } }, world.root, null, null, null, {});
tr._scene = rt.serialize_scene(world.root, undefined, undefined, sky);
tr._begin_journal(null, tr._scene.node_size.length);
const old = tr._scene;

// the slot model of the resident scene after the first (full, DFS-order) upload
const N0 = old.node_size.length;
const M = { cube: [], child: [], up: [], set: [], dfs: [] };
for (let k = 0; k < N0; k++) {
	M.cube[k] = [old.node_pos[3 * k], old.node_pos[3 * k + 1], old.node_pos[3 * k + 2], old.node_size[k]];
	M.child[k] = Array.from(old.node_child.subarray(8 * k, 8 * k + 8));
	M.up[k] = k === 0 ? -1 : old.node_parent[k];
	const b = old.node_ent_begin[k];
	M.set[k] = Array.from(old.list_entity.subarray(b, b + old.node_ent_count[k]));
	M.dfs[k] = k;
}
const E = { type: Array.from(old.ent_type), geom: [], shade: Array.from(old.ent_shade), sub: Array.from(old.ent_substance) };
for (let i = 0; i < old.ent_type.length; i++) E.geom[i] = Array.from(old.ent_geom.subarray(9 * i, 9 * i + 9));

// the edits, through the mutators
function do_op(o) {
	if (o.op === 'move') {
		const e = world.entities[o.entity];
		e._set_pos({ v: o.pos });
		rs.add_entity_to_octree(world.root, e, { max_in_depth: o.depth, max_out_depth: 0 });
	} else if (o.op === 'add_sphere') {
		const like = world.entities[o.like];
		const e = new rs.SphereEntity(like.get_material(), like.get_texture(), like.get_substance(), o.pos, o.d);
		rs.add_entity_to_octree(world.root, e, { max_in_depth: o.depth, max_out_depth: 0 });
		world.entities.push(e);                             // later ops name it by this index
	} else if (o.op === 'setpos') {                         // _set_pos alone: the entity stays in its node
		world.entities[o.entity]._set_pos({ v: o.pos });
	} else if (o.op === 'shade') {
		const e = world.entities[o.entity], like = world.entities[o.like];
		e.set_material(like.get_material());
		e.set_texture(like.get_texture());
	} else if (o.op === 'substance') {
		world.entities[o.entity].set_substance(world.entities[o.like].get_substance());
	} else throw Error('op ' + o.op);
}
function sync() {
const edit = rt._internal.build_edit(tr._scene, tr._st, tr._journal, undefined, sky);
assert(edit, 'build_edit refused an expressible edit');

// rt_apply_edit on the model
const old_slots = M.cube.length;
for (let k = 0; k < edit.rec_slot.length; k++) {
	const sl = edit.rec_slot[k];
	M.cube[sl] = Array.from(edit.rec_cube.subarray(4 * k, 4 * k + 4));
	M.child[sl] = Array.from(edit.rec_child.subarray(8 * k, 8 * k + 8));
	M.up[sl] = edit.rec_up[2 * k];
}
for (let k = 0; k < edit.set_slot.length; k++) {
	const b = edit.set_begin[k], c = edit.set_count[k];
	M.set[edit.set_slot[k]] = Array.from(edit.set_ent.subarray(b, b + c));
	for (let i = b; i < b + c; i++) {
		const id = edit.set_ent[i];
		E.type[id] = edit.set_type[i];
		E.geom[id] = Array.from(edit.set_geom.subarray(9 * i, 9 * i + 9));
		E.shade[id] = edit.set_shade[i];
	}
}
for (let i = 0; i < edit.sub_ent.length; i++) E.sub[edit.sub_ent[i]] = edit.sub_val[i];
for (let s = 0; s < old_slots; s++) {
	let a = M.dfs[s], add = 0;
	for (const g of edit.dfs_shift) if (g <= a) add++;
	M.dfs[s] = a + add;
}
for (let i = 0; i < edit.dfs_new_slot.length; i++) M.dfs[edit.dfs_new_slot[i]] = edit.dfs_new_val[i];
assert.strictEqual(M.cube.length, edit.n_slots);
tr._edit_applied(edit);
return edit;
}

let edit = null;
for (const o of ops) {
	if (o.op === 'sync') edit = sync();
	else do_op(o);
}
edit = sync();

// a fresh linearisation of the edited tree (stable entity ids), compared node by node
const neu = rt.serialize_scene(world.root, undefined, old, sky);
const N1 = neu.node_size.length;
assert.strictEqual(edit.n_slots, N1, 'slot count');
const slot_of_dfs = new Int32Array(N1).fill(-1);
for (let s = 0; s < edit.n_slots; s++) {
	assert(M.dfs[s] >= 0 && M.dfs[s] < N1 && slot_of_dfs[M.dfs[s]] < 0, 'dfs ids form a permutation');
	slot_of_dfs[M.dfs[s]] = s;
}
const shade_key = (tab, i) => [tab.shade_response[i], tab.shade_light[i], tab.shade_mirror[i], tab.shade_roughness[i],
	tab.shade_image[i], tab.shade_rgb[3 * i], tab.shade_rgb[3 * i + 1], tab.shade_rgb[3 * i + 2]].join(',');
for (let k = 0; k < N1; k++) {
	const s = slot_of_dfs[k];
	assert.deepStrictEqual(M.cube[s], [neu.node_pos[3 * k], neu.node_pos[3 * k + 1], neu.node_pos[3 * k + 2], neu.node_size[k]], 'cube ' + k);
	assert.strictEqual(M.up[s] < 0 ? -1 : M.dfs[M.up[s]], k === 0 ? -1 : neu.node_parent[k], 'parent ' + k);
	assert.deepStrictEqual(M.child[s].map((c) => (c < 0 ? -1 : M.dfs[c])), Array.from(neu.node_child.subarray(8 * k, 8 * k + 8)), 'children ' + k);
	const b = neu.node_ent_begin[k];
	const want = Array.from(neu.list_entity.subarray(b, b + neu.node_ent_count[k]));
	assert.deepStrictEqual(M.set[s] || [], want, 'set ' + k);
	for (const id of want) {
		assert.strictEqual(E.type[id], neu.ent_type[id]);
		assert.deepStrictEqual(E.geom[id], Array.from(neu.ent_geom.subarray(9 * id, 9 * id + 9)), 'geom ' + id);
		assert.strictEqual(shade_key(edit, E.shade[id]), shade_key(neu, neu.ent_shade[id]), 'shade ' + id);
		assert.strictEqual(E.sub[id], neu.ent_substance[id], 'substance ' + id);
	}
}
console.log('edit ok: ' + JSON.stringify({ slots: edit.n_slots, new_nodes: edit.n_slots - N0, rec: edit.rec_slot.length,
	sets: edit.set_slot.length, members: edit.set_ent.length, subs: edit.sub_ent.length }));
