'use strict';
// rt_path.js — the raytracer.js render path restated in plain JavaScript, run on Node (V8).
//
// TEST INFRASTRUCTURE / CPU BASELINE ONLY.  bench.py's cpu_baseline leg times it (BASELINE.md
// "CPU-baseline plan": the path in JS on the GPU box's host cores, 1 thread and a worker_threads
// split), and tests/test_js_baseline.py checks it against the C oracle bit for bit.  The product
// path never loads it.
//
// It keeps the reference's object model so that its speed stands for the reference's: Vector
// objects holding a `v` array and functional vector ops that allocate (src/math/vector.ts), an
// Octree of node objects with parent links and an insertion-ordered Set of entities per node
// (src/octree.ts, src/octree_entity.ts), a stateful OctreeWalker whose cur_node / next_pos are
// small objects (src/octree_space.ts:159-408), Box / Sphere line_intersection returning arrays of
// {parameter, normal} records filtered by select_parameters (src/math/intersection.ts:109-218),
// and Ray.trace's loop (src/raytracer.ts:168-277).  Operation order follows the C oracle
// (oracle/rt_oracle.c), which cites the reference line by line.  Scope: spheres, boxes, the
// build's triangles, reflection / matte / light / transmission, solid sky, refmax, the
// inverse-square law and the ExposureBuffer blend; textures and rough mirrors are not restated
// (a scene using them is rejected).
//
//   node rt_path.js DIR [--threads N] [--repeat R]
// DIR holds manifest.json + the scene / pixel arrays written by oracle/js_baseline.py; results go
// to DIR/out_*.bin and a JSON line on stdout.
const fs = require('fs');
const path = require('path');
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');

// ---- vector.ts -------------------------------------------------------------------------------
class Vector {
  constructor(v) { this.v = v; }
}
const vector = {
  vector: (x, y, z) => new Vector([x, y, z]),
  clone: (a) => new Vector(a.v.slice()),
  add: (a, b) => new Vector([a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2]]),
  sub: (a, b) => new Vector([a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2]]),
  scale: (a, k) => new Vector([a.v[0] * k, a.v[1] * k, a.v[2] * k]),
  negate: (a) => new Vector([-a.v[0], -a.v[1], -a.v[2]]),
  dot(a, b) {                                      // sum from +0, left to right
    let s = 0;
    for (let i = 0; i < 3; i++) s += a.v[i] * b.v[i];
    return s;
  },
  length(a) { return Math.sqrt(vector.dot(a, a)); },
  cross: (a, b) => new Vector([a.v[1] * b.v[2] - a.v[2] * b.v[1], a.v[2] * b.v[0] - a.v[0] * b.v[2],
                               a.v[0] * b.v[1] - a.v[1] * b.v[0]]),
  reflection(d, n) {                               // d + n * (-(d.n) * 2)
    const k = -vector.dot(d, n) * 2;
    return vector.add(d, vector.scale(n, k));
  },
};
const isNegative = (x) => x < 0 || Object.is(x, -0);

// ---- intersection.ts ---------------------------------------------------------------------------
const FACE_NORMALS = [vector.vector(-1, 0, 0), vector.vector(1, 0, 0), vector.vector(0, -1, 0),
                      vector.vector(0, 1, 0), vector.vector(0, 0, -1), vector.vector(0, 0, 1)];

class Box {
  constructor(pos, size) { this.pos = pos; this.size = size; }
  line_intersection(line) {
    const tl = vector.sub(this.pos, vector.scale(this.size, 0.5));
    const d = line.dir.v, o = line.start.v, s = this.size.v;
    const p = [-d[0], d[0], -d[1], d[1], -d[2], d[2]];
    const q = [o[0] - tl.v[0], tl.v[0] + s[0] - o[0], o[1] - tl.v[1], tl.v[1] + s[1] - o[1],
               o[2] - tl.v[2], tl.v[2] + s[2] - o[2]];
    let u1 = -Infinity, u2 = Infinity, i1, i2;
    for (let i = 0; i < 6; ++i) {
      const e = p[i];
      const u = q[i] / e;
      if (isNegative(e)) { if (u > u1) { u1 = u; i1 = i; } }
      else if (u < u2) { u2 = u; i2 = i; }
    }
    if (u1 > u2) return [];
    return [{ parameter: u1, normal: FACE_NORMALS[i1] }, { parameter: u2, normal: FACE_NORMALS[i2] }];
  }
}

class Sphere {
  constructor(pos, diameter) {
    this.pos = pos;
    this._radius = diameter / 2;
    this._dot_pp = vector.dot(pos, pos);
    this._radius_sq = this._radius * this._radius;
  }
  line_intersection(line) {
    const dist = vector.sub(line.start, this.pos);
    const a = vector.dot(line.dir, line.dir);
    const b = vector.dot(dist, line.dir) * 2;
    const c = vector.dot(line.start, line.start) + this._dot_pp - vector.dot(line.start, this.pos) * 2 - this._radius_sq;
    const delta = b * b - a * c * 4;
    if (delta < 0) return [];
    const sd = Math.sqrt(delta);
    const tmp1 = -b / (a * 2), tmp2 = sd / (a * 2);
    return [{ parameter: tmp1 - tmp2 }, { parameter: tmp1 + tmp2 }];
  }
}

const select_forward = (params) => params.filter((i) => i.parameter >= 0);
const intersection_point = (line, param) => vector.add(line.start, vector.scale(line.dir, param.parameter));

// ---- entities (src/entities/*) -----------------------------------------------------------------
class SphereEntity {
  constructor(id, g, shade, substance) {
    this.id = id; this.shade = shade; this.substance = substance;
    this.pos = vector.vector(g[0], g[1], g[2]);
    this.diameter = g[3];
    this.sphere_math = new Sphere(this.pos, g[3]);
    this._radius_sq = g[3] * g[3] / 4;
  }
  collision_info(line) {
    const ps = select_forward(this.sphere_math.line_intersection(line));
    if (ps.length === 0) return undefined;
    const point = intersection_point(line, ps[0]);
    let normal = vector.scale(vector.sub(point, this.pos), 2 / this.diameter);
    normal = vector.scale(normal, -Math.sign(vector.dot(line.dir, normal)));
    return { point, normal };
  }
  is_within(p) {
    const d = vector.sub(p, this.pos);
    return vector.dot(d, d) <= this._radius_sq;
  }
}

class BoxEntity {
  constructor(id, g, shade, substance) {
    this.id = id; this.shade = shade; this.substance = substance;
    this.pos = vector.vector(g[0], g[1], g[2]);
    this.size = g[3];
    this.box_math = new Box(this.pos, vector.scale(vector.vector(1, 1, 1), g[3]));
  }
  collision_info(line) {
    const ps = select_forward(this.box_math.line_intersection(line));
    if (ps.length === 0) return undefined;
    const point = intersection_point(line, ps[0]);
    if (ps[0].normal === undefined) throw new Error('vector.dot(dir, undefined)');
    const n = ps[0].normal;
    return { point, normal: vector.scale(n, -Math.sign(vector.dot(line.dir, n))) };
  }
  is_within(p) {                                   // pos as the MIN corner (reference inconsistency)
    const s = 1 * this.size;
    for (let i = 0; i < 3; i++) if (!(p.v[i] >= this.pos.v[i] && p.v[i] < this.pos.v[i] + s)) return false;
    return true;
  }
}

class FaceEntity {                                 // the build's triangle (DESIGN.md §3.2)
  constructor(id, g, shade, substance) {
    this.id = id; this.shade = shade; this.substance = substance;
    this.v0 = vector.vector(g[0], g[1], g[2]);
    this.v1 = vector.vector(g[3], g[4], g[5]);
    this.v2 = vector.vector(g[6], g[7], g[8]);
  }
  collision_info(line) {
    const e1 = vector.sub(this.v1, this.v0), e2 = vector.sub(this.v2, this.v0);
    const pv = vector.cross(line.dir, e2);
    const det = vector.dot(e1, pv);
    if (!(det != 0)) return undefined;
    const inv = 1 / det;
    const tv = vector.sub(line.start, this.v0);
    const u = vector.dot(tv, pv) * inv;
    if (!(u >= 0 && u <= 1)) return undefined;
    const qv = vector.cross(tv, e1);
    const v = vector.dot(line.dir, qv) * inv;
    if (!(v >= 0 && u + v <= 1)) return undefined;
    const t = vector.dot(e2, qv) * inv;
    if (!(t >= 0)) return undefined;
    const point = intersection_point(line, { parameter: t });
    const n = vector.cross(e1, e2);
    const nn = vector.scale(n, 1.0 / Math.sqrt(vector.dot(n, n)));
    return { point, normal: vector.scale(nn, -Math.sign(vector.dot(line.dir, nn))) };
  }
  is_within() { return false; }
}

// ---- octree.ts / octree_space.ts -----------------------------------------------------------------
class Octree {
  constructor(parent, pos, size) {
    this.parent = parent;
    this.children = [undefined, undefined, undefined, undefined, undefined, undefined, undefined, undefined];
    this.pos = pos;
    this.size = size;
    this.value = new Set();                        // EntitySet, insertion order
    this.dfs_id = -1;
  }
  get(n) {
    if (!(n >= 0 && n <= 7)) throw new Error('Node index out of range (0..7)');
    return this.children[n];
  }
  get_root() { let c = this; while (c.parent) c = c.parent; return c; }
}

const ToInt32 = (x) => x << 0;

function node_at_pos(octree, p) {                  // src/octree_space.ts:61-93, CLOSE_OPEN
  for (let i = 0; i < 3; i++) if (!(p.v[i] >= octree.pos.v[i] && p.v[i] < octree.pos.v[i] + octree.size)) return null;
  let cur = octree.get_root(), next = cur, index = 0;
  let npos = octree.pos.v.slice(), nsize = octree.size;
  while (next !== undefined) {
    const s = 2 / nsize;
    const ind = [(p.v[0] - npos[0]) * s, (p.v[1] - npos[1]) * s, (p.v[2] - npos[2]) * s];
    cur = next;
    index = (ToInt32(ind[2]) << 2) + (ToInt32(ind[1]) << 1) + (ToInt32(ind[0]) << 0);
    next = cur.get(index);
    nsize /= 2;
    for (let i = 0; i < 3; i++) npos[i] += ToInt32(ind[i]) * nsize;
  }
  return { tree: cur, octant: index };
}

function octant_adj_pos(t, p) {
  const h = t.size / 2;
  return ((p.v[2] >= t.pos.v[2] + h) << 2) | ((p.v[1] >= t.pos.v[1] + h) << 1) | (p.v[0] >= t.pos.v[0] + h);
}

function index_within_parent(c) {
  const p = c.parent;
  if (!p) return undefined;
  const s = 2 / p.size;
  const ind = [(c.pos.v[0] - p.pos.v[0]) * s, (c.pos.v[1] - p.pos.v[1]) * s, (c.pos.v[2] - p.pos.v[2]) * s];
  return (ToInt32(ind[2]) << 2) + (ToInt32(ind[1]) << 1) + (ToInt32(ind[0]) << 0);
}

class OctreeWalker {
  constructor(tree) {
    this.tree = tree;
    this.cur_node = undefined;
  }
  set_pos_and_dir(pos, dir, node) {
    this.direction = dir;
    this.cur_node = node !== undefined ? node : (node_at_pos(this.tree, pos) || undefined);
    this.pos = pos;
    return this.setup_cur_node();
  }
  reset_state() {
    this.next_pos = [this.pos, undefined];
    this.cur_returned = false;
    this.stepped_in = false;
    this.next_pos_is_ahead = false;
    this.depth = 0;
  }
  setup_cur_node() {
    this.reset_state();
    if (this.cur_node !== undefined) return true;
    const t = this.tree;
    const box = new Box(vector.add(t.pos, vector.scale(vector.vector(0.5, 0.5, 0.5), t.size)),
                        vector.scale(vector.vector(1, 1, 1), t.size));
    const line = { start: this.pos, dir: this.direction };
    const ps = select_forward(box.line_intersection(line));
    if (ps.length === 0) return false;
    const ip = intersection_point(line, ps[0]);
    this.cur_node = { tree: t, octant: undefined };
    this.next_pos = [ip, vector.negate(ps[0].normal)];
    return true;
  }
  step_back() {
    this.stepped_in = true;
    if (this.cur_node.octant === undefined) {
      this.cur_node = undefined;
      this.cur_returned = false;
      return;
    }
    if (this.depth > 0) { this.depth--; this.cur_returned = true; } else this.cur_returned = false;
    const gp = index_within_parent(this.cur_node.tree);
    if (gp !== undefined) this.cur_node = { tree: this.cur_node.tree.parent, octant: gp };
    else this.cur_node = { tree: this.cur_node.tree, octant: undefined };
  }
  update_next_pos() {
    const t = this.cur_node.tree, n = this.cur_node.octant;
    const half = t.size / 2;
    const dpos = vector.add(t.pos, vector.scale(vector.vector(n & 1, (n >> 1) & 1, (n >> 2) & 1), half));
    const box = new Box(vector.add(dpos, vector.scale(vector.vector(0.5, 0.5, 0.5), half)),
                        vector.scale(vector.vector(1, 1, 1), half));
    const line = { start: this.pos, dir: this.direction };
    const param = box.line_intersection(line).pop();
    const ip = intersection_point(line, param);     // [].pop() is undefined: throws here
    this.next_pos = [ip, param.normal];
  }
  next() {
    while (this.cur_node !== undefined) {
      const last = this.cur_node;
      const node = last.octant !== undefined ? last.tree.get(last.octant) : last.tree;
      if (!this.cur_returned && node !== undefined) {
        this.cur_returned = true;
        return { node, pos: last };
      }
      if (last.octant !== undefined) {
        if (!this.next_pos_is_ahead) {
          if (!this.stepped_in && node !== undefined) {
            this.depth++;
            this.cur_node = { tree: node, octant: octant_adj_pos(node, this.next_pos[0]) };
            this.cur_returned = false;
            continue;
          }
          this.update_next_pos();
        }
        const c = vector.vector(last.octant & 1, (last.octant >> 1) & 1, (last.octant >> 2) & 1);
        if (this.next_pos[1] === undefined) throw new Error('vector.add(v, undefined)');
        const nx = vector.add(c, this.next_pos[1]);
        if (!nx.v.some((x) => x < 0 || x > 1)) {
          this.cur_node = { tree: last.tree, octant: ToInt32(nx.v[0]) | (ToInt32(nx.v[1]) << 1) | (ToInt32(nx.v[2]) << 2) };
          this.cur_returned = false;
          this.stepped_in = false;
          this.next_pos_is_ahead = false;
          continue;
        }
        this.next_pos_is_ahead = true;
      }
      this.step_back();
    }
    return undefined;
  }
}

function entity_at_pos(root, p) {                  // src/octree_entity.ts:191-202
  const at = node_at_pos(root, p);
  let cur = at ? at.tree : undefined;
  while (cur !== undefined && cur !== null) {
    for (const e of cur.value) if (e.is_within(p)) return e;
    cur = cur.parent;
  }
  return undefined;
}

// ---- scene ---------------------------------------------------------------------------------------
function load(dir) {
  const m = JSON.parse(fs.readFileSync(path.join(dir, 'manifest.json'), 'utf8'));
  const arr = (name, T) => {
    const b = fs.readFileSync(path.join(dir, name + '.bin'));
    return new T(b.buffer, b.byteOffset, b.byteLength / T.BYTES_PER_ELEMENT);
  };
  const S = {
    node_pos: arr('node_pos', Float64Array), node_size: arr('node_size', Float64Array),
    node_parent: arr('node_parent', Int32Array), node_child: arr('node_child', Int32Array),
    node_ent_begin: arr('node_ent_begin', Int32Array), node_ent_count: arr('node_ent_count', Int32Array),
    list_entity: arr('list_entity', Int32Array), ent_type: arr('ent_type', Int32Array),
    ent_geom: arr('ent_geom', Float64Array), ent_shade: arr('ent_shade', Int32Array),
    ent_substance: arr('ent_substance', Int32Array), pixels: arr('pixels', Int32Array),
  };
  // entity objects
  const ents = [];
  for (let i = 0; i < S.ent_type.length; i++) {
    const g = Array.from(S.ent_geom.subarray(9 * i, 9 * i + 9));
    const K = [SphereEntity, BoxEntity, FaceEntity][S.ent_type[i]];
    ents.push(new K(i, g, S.ent_shade[i], S.ent_substance[i]));
  }
  // the octree (nodes in DFS order, parents first)
  const nodes = [];
  for (let n = 0; n < S.node_size.length; n++) {
    const par = S.node_parent[n] >= 0 ? nodes[S.node_parent[n]] : null;
    const t = new Octree(par, vector.vector(S.node_pos[3 * n], S.node_pos[3 * n + 1], S.node_pos[3 * n + 2]), S.node_size[n]);
    t.dfs_id = n;
    for (let k = 0; k < S.node_ent_count[n]; k++) t.value.add(ents[S.list_entity[S.node_ent_begin[n] + k]]);
    nodes.push(t);
  }
  for (let n = 0; n < nodes.length; n++)
    for (let c = 0; c < 8; c++) {
      const k = S.node_child[8 * n + c];
      if (k >= 0) nodes[n].children[c] = nodes[k];
    }
  for (const sh of m.shades) if (sh.image || sh.roughness > 0) throw new Error('textures / rough mirrors are not restated');
  if (m.config.sky_image) throw new Error('sky textures are not restated');
  return { m, root: nodes[0], ents, pixels: S.pixels };
}

// ---- camera (src/view/camera.ts:207-250), rows over height -------------------------------------
function rotate_vectors(a, b, rot) {
  const c = rot[0], s = rot[1];
  return [new Vector([a.v[0] * c + b.v[0] * s, a.v[1] * c + b.v[1] * s, a.v[2] * c + b.v[2] * s]),
          new Vector([a.v[0] * -s + b.v[0] * c, a.v[1] * -s + b.v[1] * c, a.v[2] * -s + b.v[2] * c])];
}

function camera_dirs(cam) {
  const W = cam.width, H = cam.height, dirs = new Float64Array(3 * W * H);
  const ch = [cam.scan_h[0], -cam.scan_h[1]], cv = [cam.scan_v[0], -cam.scan_v[1]];
  for (let half = 0; half < 2; half++) {
    const y0 = half === 0 ? H >> 1 : (H >> 1) - 1, y1 = half === 0 ? H : -1, dy = half === 0 ? 1 : -1;
    const rv = half === 0 ? cam.scan_v : cv;
    let fr = new Vector(cam.fr.slice()), up = new Vector(cam.up.slice());
    if (half === 1) [fr, up] = rotate_vectors(fr, up, rv);
    for (let y = y0; y !== y1; y += dy) {
      for (let hh = 0; hh < 2; hh++) {
        const x0 = hh === 0 ? W >> 1 : (W >> 1) - 1, x1 = hh === 0 ? W : -1, dx = hh === 0 ? 1 : -1;
        const rh = hh === 0 ? cam.scan_h : ch;
        let f = vector.clone(fr), l = new Vector(cam.lf.slice());
        if (hh === 1) [f, l] = rotate_vectors(f, l, rh);
        for (let x = x0; x !== x1; x += dx) {
          const o = 3 * (y * W + x);
          dirs[o] = f.v[0]; dirs[o + 1] = f.v[1]; dirs[o + 2] = f.v[2];
          [f, l] = rotate_vectors(f, l, rh);
        }
      }
      [fr, up] = rotate_vectors(fr, up, rv);
    }
  }
  return dirs;
}

// ---- Ray.trace (src/raytracer.ts:168-277) ----------------------------------------------------------
const ST_OK = 0, ST_WARN = 1, ST_FAULT = 2;

// ---- shadow rays: a BUILD EXTENSION the reference does not have (include/rt.h rt_set_lights,
// DESIGN.md §3.6), restated on this object model from the frozen definition: manifest.lights /
// manifest.ambient.  The C oracle's shadow_factor is the same definition.  The light is blocked when
// some entity of the tree that is not a light has a forward hit (or a throwing test) nearer than
// dist - 1e-3: an existence question, answered here by a descent that skips the subtrees whose
// entities' geometry bounds the segment cannot meet.
function geom_bounds(e) {                          // the collision geometry's bounds (not get_aabb)
  let lo, hi;
  if (e instanceof FaceEntity) {
    lo = [0, 1, 2].map((i) => Math.min(e.v0.v[i], e.v1.v[i], e.v2.v[i]));
    hi = [0, 1, 2].map((i) => Math.max(e.v0.v[i], e.v1.v[i], e.v2.v[i]));
  } else {
    const h = Math.abs(e instanceof SphereEntity ? e.diameter : e.size) * 0.5;
    lo = e.pos.v.map((x) => x - h);
    hi = e.pos.v.map((x) => x + h);
  }
  if (!lo.concat(hi).every(Number.isFinite)) return { lo: [-Infinity, -Infinity, -Infinity], hi: [Infinity, Infinity, Infinity] };
  return { lo, hi };
}

function subtree_bounds(t) {                       // cached on the node: { lo, hi, n }
  if (t.sb) return t.sb;
  const sb = { lo: [Infinity, Infinity, Infinity], hi: [-Infinity, -Infinity, -Infinity], n: t.value.size };
  const grow = (b) => { for (let i = 0; i < 3; i++) { sb.lo[i] = Math.min(sb.lo[i], b.lo[i]); sb.hi[i] = Math.max(sb.hi[i], b.hi[i]); } };
  for (const e of t.value) grow(e.sb || (e.sb = geom_bounds(e)));
  for (const c of t.children) {
    if (c === undefined) continue;
    const cb = subtree_bounds(c);
    if (cb.n) { sb.n += cb.n; grow(cb); }
  }
  return (t.sb = sb);
}

function seg_may_meet(q, u, dist, b) {             // conservative slab test (oracle seg_may_meet)
  let S = 1 + Math.abs(dist);
  for (let i = 0; i < 3; i++) {
    S = Math.max(S, Math.abs(q.v[i]));
    if (Number.isFinite(b.lo[i])) S = Math.max(S, Math.abs(b.lo[i]));
    if (Number.isFinite(b.hi[i])) S = Math.max(S, Math.abs(b.hi[i]));
  }
  const m = S * Math.pow(2, -20);
  let t0 = -m, t1 = dist + m;
  for (let i = 0; i < 3; i++) {
    const l = b.lo[i] - m, h = b.hi[i] + m;
    if (u.v[i] === 0) { if (q.v[i] < l || q.v[i] > h) return false; continue; }
    let a = (l - q.v[i]) / u.v[i], c = (h - q.v[i]) / u.v[i];
    if (a > c) { const x = a; a = c; c = x; }
    if (a > t0) t0 = a;
    if (c < t1) t1 = c;
    if (t0 > t1) return false;
  }
  return true;
}

function entity_blocks(sc, e, q, u, lim) {
  let hit;
  try {
    hit = e.collision_info({ start: q, dir: u });
  } catch (err) {                                  // a throwing test: its hit point decides
    hit = { point: intersection_point({ start: q, dir: u }, select_forward(e.box_math.line_intersection({ start: q, dir: u }))[0]) };
  }
  if (hit === undefined || sc.m.shades[e.shade].light) return false;
  return vector.length(vector.sub(hit.point, q)) < lim;
}

function subtree_blocks(sc, t, q, u, dist, lim) {
  const sb = subtree_bounds(t);
  if (!sb.n || !seg_may_meet(q, u, dist, sb)) return false;
  for (const e of t.value) {
    if (seg_may_meet(q, u, dist, e.sb) && entity_blocks(sc, e, q, u, lim)) return true;
  }
  for (const c of t.children) if (c !== undefined && subtree_blocks(sc, c, q, u, dist, lim)) return true;
  return false;
}

function shadow_blocked(sc, q, u, dist) {
  return subtree_blocks(sc, sc.root, q, u, dist, dist - 1e-3);
}

function shadow_factor(sc, p, nrm, path_len) {
  const a = sc.m.ambient, s = [a, a, a];
  for (const lt of sc.m.lights) {
    const v = vector.sub(new Vector(lt.pos.slice()), p);
    const dist = vector.length(v);
    if (!(dist > 0)) continue;
    const u = vector.scale(v, 1 / dist);
    const cosine = vector.dot(nrm, u);
    if (!(cosine > 0)) continue;
    const q = vector.add(p, vector.scale(u, 1e-3));
    if (shadow_blocked(sc, q, u, dist)) continue;
    const t = (path_len + dist) * sc.m.config.distance_attenuation_factor;
    const isl = 1.0 / (Number.EPSILON + t ** 2);
    const k = cosine * isl;
    for (let c = 0; c < 3; c++) s[c] += lt.rgb[c] * k;
  }
  return s;
}

// `out` holds the colour so far: a throw leaves the ray's colour at that point, as the oracle does
function trace_ray(sc, walker, start, dir0, start_node, start_sub, out) {
  const { m } = sc, cfg = m.config;
  let refpoint = vector.clone(start), dir = dir0;
  let col = [1, 1, 1], refcount = 0, light = false, cur_sub = start_sub, path_len = 0;
  out.rgb = col;
  walker.set_pos_and_dir(refpoint, dir, start_node);
  for (;;) {
    const stop = walker.next();
    if (stop === undefined) break;
    let hit, ent;
    for (const e of stop.node.value) {
      const c = e.collision_info({ start: refpoint, dir });
      if (c !== undefined) { hit = c; ent = e; break; }
    }
    if (hit === undefined) continue;
    if (out.hit_ent < 0 && out.segments === 1) { out.hit_ent = ent.id; out.hit_node = stop.node.dfs_id; }
    if (vector.dot(dir, hit.normal) >= 0) { out.status = ST_WARN; return out; }
    refcount++;
    const sh = m.shades[ent.shade];
    col = out.rgb = [col[0] * sh.rgb[0], col[1] * sh.rgb[1], col[2] * sh.rgb[2]];
    path_len += vector.length(vector.sub(hit.point, refpoint));
    refpoint = hit.point;
    if (sh.light) { light = true; break; }
    if (sh.response === 0) {                       // REFLECTION
      if (!sh.mirror) {
        if (m.lights && m.lights.length) {          // shadow rays (build extension)
          const sf = shadow_factor(sc, refpoint, hit.normal, path_len);
          col = out.rgb = [col[0] * sf[0], col[1] * sf[1], col[2] * sf[2]];
        }
        return out;
      }
      dir = vector.reflection(dir, hit.normal);
      refpoint = vector.add(refpoint, vector.scale(dir, 1e-3));
    } else if (sh.response === 1) {                // TRANSMISSION
      refpoint = vector.add(refpoint, vector.scale(dir, 1e-3));
      const e2 = entity_at_pos(sc.root, refpoint);
      const sub = e2 !== undefined ? e2.substance : cfg.default_substance;
      if (sub >= 0) {
        if (cur_sub < 0) throw new Error('undefined.refractive_index');
        const r = m.substance_ri[cur_sub] / m.substance_ri[sub], r_sq = r * r;
        const cosine = vector.dot(dir, hit.normal), cos_sq = cosine * cosine;
        const ref_sine_sq = (1 - cos_sq) * r_sq;
        if (ref_sine_sq <= 1) {
          const adj = vector.scale(hit.normal, Math.sqrt(1 - ref_sine_sq) - cosine);
          dir = vector.sub(vector.scale(dir, r), adj);
        } else {
          dir = vector.reflection(dir, hit.normal);
        }
        cur_sub = sub;
      }
    } else return out;
    walker.set_pos_and_dir(refpoint, dir);
    if (refcount >= cfg.refmax) { out.rgb = [0, 0, 0]; return out; }
    out.segments++;
  }
  if (!light) col = [col[0] * cfg.sky_rgb[0], col[1] * cfg.sky_rgb[1], col[2] * cfg.sky_rgb[2]];
  else {
    const t = path_len * cfg.distance_attenuation_factor;
    const isl = 1.0 / (Number.EPSILON + t ** 2);
    col = [col[0] * isl, col[1] * isl, col[2] * isl];
    out.rgb = col;
    walker.set_pos_and_dir(refpoint, dir);          // :276 (can throw)
  }
  out.rgb = col;
  return out;
}

// trace the pixels k = first, first + step, ... of the sample; returns typed arrays per sample slot
function trace_pixels(sc, dirs, first, step) {
  const { m, pixels } = sc, cam = m.camera, cfg = m.config;
  const start = vector.vector(cam.pos[0], cam.pos[1], cam.pos[2]);
  const at = node_at_pos(sc.root, start);
  const se = entity_at_pos(sc.root, start);
  const start_sub = se !== undefined ? se.substance : cfg.default_substance;
  const walker = new OctreeWalker(sc.root);
  const n = pixels.length;
  const rgb = new Float32Array(3 * n), hit_e = new Int32Array(n), hit_n = new Int32Array(n), segs = new Int32Array(n);
  const status = new Uint8Array(n);
  const w = cfg.col_weight;
  let segments = 0;
  for (let k = first; k < n; k += step) {
    const p = pixels[k];
    const dir = vector.vector(dirs[3 * p], dirs[3 * p + 1], dirs[3 * p + 2]);
    const r = { rgb: null, hit_ent: -1, hit_node: -1, segments: 1, status: ST_OK };
    try {
      trace_ray(sc, walker, start, dir, at ? { tree: at.tree, octant: at.octant } : undefined, start_sub, r);
    } catch (e) {
      r.status = ST_FAULT;                         // the reference throws out of trace_frame here
    }
    for (let c = 0; c < 3; c++) rgb[3 * k + c] = r.rgb[c] * w + 0 * (1 - w);   // ExposureBuffer.set_color_i on a reset buffer
    hit_e[k] = r.hit_ent; hit_n[k] = r.hit_node; segs[k] = r.segments; status[k] = r.status;
    segments += r.segments;
  }
  return { rgb, hit_e, hit_n, segs, status, segments };
}

// ---- entry -----------------------------------------------------------------------------------------
function write_out(dir, res) {
  fs.writeFileSync(path.join(dir, 'out_rgb.bin'), Buffer.from(res.rgb.buffer));
  fs.writeFileSync(path.join(dir, 'out_hit_entity.bin'), Buffer.from(res.hit_e.buffer));
  fs.writeFileSync(path.join(dir, 'out_hit_node.bin'), Buffer.from(res.hit_n.buffer));
  fs.writeFileSync(path.join(dir, 'out_segments.bin'), Buffer.from(res.segs.buffer));
  fs.writeFileSync(path.join(dir, 'out_status.bin'), Buffer.from(res.status.buffer));
}

if (isMainThread) {
  const argv = process.argv.slice(2);
  const dir = argv[0];
  const opt = (k, d) => { const i = argv.indexOf(k); return i >= 0 ? Number(argv[i + 1]) : d; };
  const threads = opt('--threads', 1), repeat = opt('--repeat', 1);
  const t0 = process.hrtime.bigint();
  const sc = load(dir);
  const dirs = camera_dirs(sc.m.camera);
  const t_setup = Number(process.hrtime.bigint() - t0) * 1e-9;
  const os = require('os');
  const info = { threads, cpus: os.cpus().length, cpu_model: os.cpus()[0] ? os.cpus()[0].model : '', node: process.version,
                 pixels: sc.pixels.length, setup_s: t_setup };
  if (threads <= 1) {
    let res, best = Infinity;
    for (let r = 0; r < repeat; r++) {
      const a = process.hrtime.bigint();
      res = trace_pixels(sc, dirs, 0, 1);
      best = Math.min(best, Number(process.hrtime.bigint() - a) * 1e-9);
    }
    write_out(dir, res);
    console.log(JSON.stringify(Object.assign(info, { trace_s: best, segments: res.segments })));
  } else {
    // worker_threads tile split: worker t traces sample slots t, t + N, ...; each builds its own
    // scene (as a per-core copy of the reference would), then all start together
    const ws = [], ready = [], done = [];
    const dirs_sh = new SharedArrayBuffer(dirs.byteLength);
    new Float64Array(dirs_sh).set(dirs);
    for (let t = 0; t < threads; t++) {
      const w = new Worker(__filename, { workerData: { dir, first: t, step: threads, dirs: dirs_sh } });
      ws.push(w);
      ready.push(new Promise((res) => w.once('message', res)));
    }
    Promise.all(ready).then(() => {
      const a = process.hrtime.bigint();
      for (const w of ws) {
        done.push(new Promise((res) => w.once('message', res)));
        w.postMessage('go');
      }
      return Promise.all(done).then((parts) => {
        const wall = Number(process.hrtime.bigint() - a) * 1e-9;
        const n = sc.pixels.length;
        const res = { rgb: new Float32Array(3 * n), hit_e: new Int32Array(n), hit_n: new Int32Array(n),
                      segs: new Int32Array(n), status: new Uint8Array(n), segments: 0 };
        parts.forEach((p, t) => {
          for (let k = t; k < n; k += threads) {
            for (let c = 0; c < 3; c++) res.rgb[3 * k + c] = p.rgb[3 * k + c];
            res.hit_e[k] = p.hit_e[k]; res.hit_n[k] = p.hit_n[k]; res.segs[k] = p.segs[k]; res.status[k] = p.status[k];
          }
          res.segments += p.segments;
        });
        write_out(dir, res);
        for (const w of ws) w.terminate();
        console.log(JSON.stringify(Object.assign(info, { trace_s: wall, segments: res.segments })));
      });
    });
  }
} else {
  const { dir, first, step, dirs } = workerData;
  const sc = load(dir);
  const d = new Float64Array(dirs);
  parentPort.once('message', () => {
    const r = trace_pixels(sc, d, first, step);
    parentPort.postMessage(r);
  });
  parentPort.postMessage('ready');
}
