/*
 * js_edit_time.js [n_entities] [width] — cost of scene edits through the JS drop-in on a GPU box.
 * Builds a scene of n random spheres (default 1M) with the test fixture's add_entity_to_octree
 * (max_in_depth 10), renders a first frame (full serialize + upload), then times, for 1 and 100
 * moves: the moves themselves, invalidate_scene() + trace_frame() through the journal (rt_apply_edit;
 * 15 repetitions: median, min, max and the first), and the same through a full re-read
 * (invalidate_scene({ full: true }), rt_update_scene; 2 repetitions), each against a plain
 * trace_frame() of the same frame.  One JSON line per case.
 */
'use strict';
const rs = require('../tests/js/refshape.js');
const rt = require('../raytracer.js_amd/js/raytracer.js');

const N = Number(process.argv[2] || 1000000), W = Number(process.argv[3] || 256);
let seed = 42;
function rnd() {                                   // Park-Miller minimal standard generator -> (0, 1)
	seed = (seed * 16807) % 2147483647;
	return seed / 2147483647;
}
const ms = (t) => { const d = process.hrtime(t); return d[0] * 1e3 + d[1] / 1e6; };

const root = new rs.Octree({ pos: { v: [0, 0, 0] }, size: 1 }, undefined, new rs.EntitySet());
const mats = [new rs.SolidMaterial(0, false, false, 0), new rs.SolidMaterial(0, false, true, 0), new rs.SolidMaterial(0, true, false, 0)];
const texs = [new rs.SolidTexture({ r: 0.8, g: 0.3, b: 0.2, a: 1 }), new rs.SolidTexture({ r: 1, g: 1, b: 1, a: 1 })];
const ents = [];
let t = process.hrtime();
for (let i = 0; i < N; i++) {
	const d = 0.0005 + 0.002 * rnd();
	const p = [d + (1 - 2 * d) * rnd(), d + (1 - 2 * d) * rnd(), d + (1 - 2 * d) * rnd()];
	const k = i % 97 === 0 ? 2 : (i % 7 === 0 ? 1 : 0);
	const e = new rs.SphereEntity(mats[k], texs[k === 2 ? 1 : 0], undefined, p, d);
	rs.add_entity_to_octree(root, e, { max_in_depth: 10, max_out_depth: 0 });
	ents.push(e);
}
const build_ms = ms(t);
const cam = rs.camera({ width: W, height: W, pos: [0.5, 0.5, -0.5], fr: [0, 0, 1], lf: [-1, 0, 0], up: [0, 1, 0],
	scan_h: [Math.cos(0.9 / W), Math.sin(0.9 / W)], scan_v: [Math.cos(0.9 / W), Math.sin(0.9 / W)] });
const eb = new rs.ExposureBuffer(W, W);
const tr = new rt.Raytracer({ refmax: 2, distance_attenuation_factor: 1, sky: { texture: texs[1] } }, root, cam, eb, null, {});
t = process.hrtime();
tr.trace_frame();
const first_ms = ms(t);
const frame = () => { const a = process.hrtime(); tr.trace_frame(); return ms(a); };
for (let i = 0; i < 3; i++) frame();
const plain = [];
for (let i = 0; i < 5; i++) plain.push(frame());
plain.sort((a, b) => a - b);
console.log(JSON.stringify({ n_entities: N, octree_build_ms: +build_ms.toFixed(1), first_frame_ms: +first_ms.toFixed(1),
	plain_frame_ms: +plain[2].toFixed(3), width: W }));

function moves(n) {
	const a = process.hrtime();
	for (let i = 0; i < n; i++) {
		const e = ents[Math.floor(rnd() * N)];
		const d = e.get_diameter();
		e._set_pos({ v: [d + (1 - 2 * d) * rnd(), d + (1 - 2 * d) * rnd(), d + (1 - 2 * d) * rnd()] });
		rs.add_entity_to_octree(root, e, { max_in_depth: 10, max_out_depth: 0 });
	}
	return ms(a);
}
for (const mode of ['journal', 'full']) {
	for (const n of [1, 100]) {
		const rows = [];
		for (let rep = 0; rep < (mode === 'full' ? 2 : 15); rep++) {
			const mv = moves(n);
			const a = process.hrtime();
			tr.invalidate_scene(mode === 'full' ? { full: true } : undefined);
			tr.trace_frame();
			const tot = ms(a);
			rows.push({ moves_ms: mv, sync_and_frame_ms: tot, update: tr.last_update });
		}
		const first = rows[0].sync_and_frame_ms;
		rows.sort((x, y) => x.sync_and_frame_ms - y.sync_and_frame_ms);
		const r = rows[rows.length >> 1];
		console.log(JSON.stringify({ mode, moves: n, reps: rows.length, moves_ms: +r.moves_ms.toFixed(3),
			invalidate_plus_frame_ms: +r.sync_and_frame_ms.toFixed(3), edit_cost_ms: +(r.sync_and_frame_ms - plain[2]).toFixed(3),
			first_ms: +first.toFixed(3), max_ms: +rows[rows.length - 1].sync_and_frame_ms.toFixed(3),
			min_ms: +rows[0].sync_and_frame_ms.toFixed(3), update: r.update }));
	}
}
tr.close();
