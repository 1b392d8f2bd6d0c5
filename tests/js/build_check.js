/*
 * build_check.js <entities.json> <out.json> — builds a scene with the test fixture's restatement of
 * add_entity_to_octree (tests/js/refshape.js, written from src/octree_entity.ts:56-188 in JS) over
 * the entity list in order, and writes the drop-in's linearisation of it (serialize_scene: DFS
 * nodes, Set-order lists, with the list's entity ids mapped back to the input order).  The Python
 * side compares it with the native builder (rt_builder.cpp) and the C oracle: three restatements
 * of the reference's octree construction, in three languages.
 */
'use strict';
const fs = require('fs');
const rs = require('./refshape.js');
const rt = require('../../raytracer.js_amd/js/raytracer.js');

const sc = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const root = new rs.Octree({ pos: { v: sc.root_pos.slice() }, size: sc.root_size }, undefined, new rs.EntitySet());
const mat = new rs.SolidMaterial(0, false, false, 0), tex = new rs.SolidTexture({ r: 1, g: 1, b: 1, a: 1 });
sc.ents.forEach((x, i) => {
	const g = x.geom;
	let e;
	if (x.type === rt.RT_ENT_SPHERE) e = new rs.SphereEntity(mat, tex, undefined, g.slice(0, 3), g[3]);
	else if (x.type === rt.RT_ENT_BOX) e = new rs.BoxEntity(mat, tex, undefined, g.slice(0, 3), g[3]);
	else e = new rt.FaceEntity(undefined, mat, tex, undefined, g.slice(0, 3), g.slice(3, 6), g.slice(6, 9));
	e.__orig_id = i;
	rs.add_entity_to_octree(root, e, { max_in_depth: x.depth, max_out_depth: 0 });
});
const ser = rt.serialize_scene(root, undefined);
const orig = ser.entities.map((e) => e.__orig_id);
fs.writeFileSync(process.argv[3], JSON.stringify({
	node_pos: Array.from(ser.node_pos), node_size: Array.from(ser.node_size), node_parent: Array.from(ser.node_parent),
	node_child: Array.from(ser.node_child), node_ent_begin: Array.from(ser.node_ent_begin),
	node_ent_count: Array.from(ser.node_ent_count), list_entity: Array.from(ser.list_entity, (i) => orig[i])
}));
console.log('built: ' + ser.node_size.length + ' nodes, ' + ser.list_entity.length + ' list entries');
