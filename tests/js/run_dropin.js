/*
 * run_dropin.js <scene.json> <out_prefix> [--serialize-only] [--scatter <seed>] [--edit A B C]
 *               [--devices 0,0,0] [--repeat N] [--plain]
 * Builds reference-shaped objects, checks serialize_scene() reproduces the linearised arrays, and
 * (unless --serialize-only) renders one frame with the drop-in Raytracer into ExposureBuffer.pixels.
 * --scatter: rough mirrors with options.scatter = 'counter', the rng's one draw = seed / 2^53.
 * --edit A B C x y z depth [--direct]: after the first frame, edit the live scene the way a host
 *   program does and render again into <out_prefix>.2.*: sphere A moves to (x, y, z) (_set_pos, then
 *   add_entity_to_octree with max_in_depth = depth, which may create nodes), and entity B takes
 *   entity C's material and texture (set_material / set_texture).  The drop-in journals these calls
 *   and sends only what they touched (rt_apply_edit).  --direct makes the same edit by writing the
 *   fields and Sets directly and calls invalidate_scene({ full: true }) (a full re-read, rt_update_scene).
 * --devices: options.devices (one context over several GPUs, or several parts on one GPU).
 * --plain: options {} (no ids, no counters), the default path a host takes; only pixels are written.
 * --lights JSON: options.lights / options.ambient (shadow rays, a build extension; include/rt.h).
 * --repeat N: after the first frame, N frames timed each with options.stats off, then N with it on
 *   (<out_prefix>.repeat.json).
 */
'use strict';
const fs = require('fs');
const assert = require('assert');
const rs = require('./refshape.js');
const rt = require('../../raytracer.js_amd/js/raytracer.js');

const [scene_path, out_prefix] = process.argv.slice(2, 4);
const only_ser = process.argv.includes('--serialize-only');
const sc = JSON.parse(fs.readFileSync(scene_path, 'utf8'));
const world = rs.inflate(sc);
const def_sub = sc.cfg.default_substance >= 0 ? world.substances[sc.cfg.default_substance] : undefined;

// 1. serialisation round trip (node order, list order, geometry bits)
const ser = rt.serialize_scene(world.root, def_sub);
assert.deepStrictEqual(Array.from(ser.node_pos), sc.node_pos);
assert.deepStrictEqual(Array.from(ser.node_size), sc.node_size);
assert.deepStrictEqual(Array.from(ser.node_parent), sc.node_parent);
assert.deepStrictEqual(Array.from(ser.node_child), sc.node_child);
assert.deepStrictEqual(Array.from(ser.node_ent_begin), sc.node_ent_begin);
assert.deepStrictEqual(Array.from(ser.node_ent_count), sc.node_ent_count);
const orig = ser.entities.map((e) => e.__orig_id);
assert.deepStrictEqual(Array.from(ser.list_entity).map((i) => orig[i]), sc.list_entity);
for (let i = 0; i < ser.entities.length; i++) {
	const o = orig[i];
	assert.strictEqual(ser.ent_type[i], sc.ent_type[o]);
	const want = sc.ent_geom.slice(9 * o, 9 * o + 9);
	const got = Array.from(ser.ent_geom.subarray(9 * i, 9 * i + 9));
	const n = sc.ent_type[o] === 0 ? 7 : (sc.ent_type[o] === 1 ? 4 : 9);
	assert.deepStrictEqual(got.slice(0, n), want.slice(0, n), 'entity ' + o);
}
console.log('serialize ok: ' + ser.node_size.length + ' nodes, ' + ser.entities.length + ' entities');
if (only_ser) process.exit(0);

// 2. one frame through the drop-in
const cam = rs.camera(sc.cam);
const eb = new rs.ExposureBuffer(sc.cam.width, sc.cam.height);
const config = {
	refmax: sc.cfg.refmax, default_substance: def_sub, distance_attenuation_factor: sc.cfg.atten,
	sky: { texture: sc.cfg.sky_image ? world.images[sc.cfg.sky_image - 1]
	                                 : new rs.SolidTexture({ r: sc.cfg.sky[0], g: sc.cfg.sky[1], b: sc.cfg.sky[2], a: 1 }) }
};
const si = process.argv.indexOf('--scatter');
const seed = si > 0 ? Number(process.argv[si + 1]) : null;
const rng = seed === null ? null : { next: () => seed / 9007199254740992 };
const di = process.argv.indexOf('--devices');
// --plain: the reference's trace_frame() as a host calls it (no ids, no counters: the split passes
// and, from RT_BAND_MIN pixels, row bands); only the pixels are written
const plain = process.argv.includes('--plain');
const opts = plain ? {} : { keep_ids: true, stats: true };
if (seed !== null) opts.scatter = 'counter';
if (di > 0) opts.devices = process.argv[di + 1].split(',').map(Number);
// --lights JSON: {"lights": [{"pos": [..], "rgb": [..]}], "ambient": a} (shadow rays, a build extension)
const li = process.argv.indexOf('--lights');
if (li > 0) {
	const L = JSON.parse(process.argv[li + 1]);
	opts.lights = L.lights.map((l) => ({ pos: { v: l.pos }, rgb: l.rgb }));
	opts.ambient = L.ambient;
}
const tracer = new rt.Raytracer(config, world.root, cam, eb, rng, opts);
const t0 = process.hrtime.bigint();
tracer.trace_frame();
const t1 = process.hrtime.bigint();
assert.strictEqual(eb.cleaned, 1);
fs.writeFileSync(out_prefix + '.rgb', Buffer.from(eb.pixels.buffer));
if (!plain) {
	const ids = Int32Array.from(tracer.last_hit_entity, (i) => (i >= 0 ? tracer._scene.entities[i].__orig_id : i));
	fs.writeFileSync(out_prefix + '.ent', Buffer.from(ids.buffer));
	fs.writeFileSync(out_prefix + '.node', Buffer.from(tracer.last_hit_node.buffer));
	fs.writeFileSync(out_prefix + '.status', Buffer.from(tracer.last_status.buffer));
}
fs.writeFileSync(out_prefix + '.json', JSON.stringify({ stats: tracer.last_stats, wall_ms: Number(t1 - t0) / 1e6 }));

function write_frame(prefix, extra) {
	const ids2 = Int32Array.from(tracer.last_hit_entity, (i) => (i >= 0 ? tracer._scene.entities[i].__orig_id : i));
	fs.writeFileSync(prefix + '.rgb', Buffer.from(eb.pixels.buffer));
	fs.writeFileSync(prefix + '.ent', Buffer.from(ids2.buffer));
	fs.writeFileSync(prefix + '.node', Buffer.from(tracer.last_hit_node.buffer));
	fs.writeFileSync(prefix + '.status', Buffer.from(tracer.last_status.buffer));
	fs.writeFileSync(prefix + '.json', JSON.stringify(Object.assign({ stats: tracer.last_stats }, extra)));
}

// --repeat N: N more frames timed one by one, without and then with the work counters
const ri = process.argv.indexOf('--repeat');
if (ri > 0) {
	const n = Number(process.argv[ri + 1]);
	const times = (stats) => {
		tracer.options.stats = stats;
		tracer.options.keep_ids = false;                        // the reference's trace_frame: pixels only
		const ms = [];
		for (let i = 0; i < n; i++) {
			const a = process.hrtime.bigint();
			tracer.trace_frame();
			ms.push(Number(process.hrtime.bigint() - a) / 1e6);
		}
		return ms;
	};
	const ms_plain = times(false), ms_counted = times(true);
	fs.writeFileSync(out_prefix + '.repeat.json', JSON.stringify({ frame_ms: ms_plain, frame_ms_stats: ms_counted }));
}

// --reopen: close() the context, then trace again: the next frame makes a new context, which must get
// the light list too (the drop-in keeps it; ADVICE r4)
if (process.argv.includes('--reopen')) {
	tracer.close();
	tracer.trace_frame();
	fs.writeFileSync(out_prefix + '.3.rgb', Buffer.from(eb.pixels.buffer));
}

const ei = process.argv.indexOf('--edit');
if (ei > 0) {
	const [A, B, C, px, py, pz, depth] = process.argv.slice(ei + 1, ei + 8).map(Number);
	const direct = process.argv.includes('--direct');
	const ea = world.entities[A], eb2 = world.entities[B], ec = world.entities[C];
	const p = [px, py, pz];
	if (!direct) {
		// through the reference's mutators (journaled): move_entity's steps, then the material swap
		ea._set_pos({ v: p });
		rs.add_entity_to_octree(world.root, ea, { max_in_depth: depth, max_out_depth: 0 });
		eb2.set_material(ec.get_material());
		eb2.set_texture(ec.get_texture());
		tracer.invalidate_scene();
	} else {
		// direct field writes that bypass the mutators: only a full re-read sees them
		const home = ea._octree;
		home.value.set.delete(ea);
		ea.pos = { v: p };
		ea.sphere_math._pos = ea.pos;
		ea.sphere_math._dot_pp = ((0 + p[0] * p[0]) + p[1] * p[1]) + p[2] * p[2];
		const t = rs.add_entity_to_octree(world.root, { get_aabb: () => ea.get_aabb(), set_octree() {} },
			{ max_in_depth: depth, max_out_depth: 0 });                // where it belongs (nodes made with Octree.set)
		t.value.set.add(ea);
		ea._octree = t;
		eb2.material = ec.material;
		eb2.texture = ec.texture;
		tracer.invalidate_scene({ full: true });
	}
	tracer.trace_frame();
	write_frame(out_prefix + '.2', { update: tracer.last_update });
}
tracer.close();
console.log('trace ok: ' + JSON.stringify(tracer.last_stats));
