/*
 * check_journal_cap.js <scene.json> — CPU check that a journal bounds itself (ADVICE r3): a Raytracer
 * dropped without close() keeps its journal in the module's JOURNALS set on Node 12 (no WeakRef), so
 * past its cap a journal forgets what it noted, marks itself `over` (its Raytracer's next sync is a
 * full re-read) and is skipped by every later mutator call; a live journal keeps noting.
 */
'use strict';
const fs = require('fs');
const assert = require('assert');
const rs = require('./refshape.js');
const rt = require('../../raytracer.js_amd/js/raytracer.js');

const world = rs.inflate(JSON.parse(fs.readFileSync(process.argv[2], 'utf8')));
const sky = new rs.SolidTexture({ r: 0.5, g: 0.5, b: 0.5, a: 1 });
const mk = () => {
	const tr = new rt.Raytracer({ refmax: 2, sky: { texture: sky } }, world.root, null, null, null, {});
	tr._scene = rt.serialize_scene(world.root, undefined, undefined, sky);
	tr._begin_journal(null, tr._scene.node_size.length);
	return tr;
};
const dropped = mk(), live = mk();
dropped._journal.cap = 4;                         // as if its scene were tiny
const n = Math.min(12, world.entities.length);
for (let i = 0; i < n; i++) world.entities[i].set_material(world.entities[(i + 1) % n].get_material());
const jd = dropped._journal, jl = live._journal;
assert(jd.over, 'the capped journal did not mark itself over');
assert.strictEqual(jd.nodes.size + jd.ents.size + jd.struct.size, 0, 'an over journal keeps nothing');
assert.strictEqual(jl.over, false);
assert.strictEqual(jl.ents.size, n, 'the live journal noted every edit');
world.entities[0].set_texture(world.entities[1].get_texture());
assert.strictEqual(jd.ents.size, 0, 'an over journal is skipped');
console.log('journal cap ok: ' + JSON.stringify({ noted: jl.ents.size }));
