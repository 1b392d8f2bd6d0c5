// gen_scatter.js — golden vectors for rough-mirror scattering, computed by V8 itself.
//
// Ray.reflect_ray + Ray.scatter_ray (src/raytracer.ts:117-133) with isotropic_sphere_sample
// (src/math/vector_utils.ts:8-14) and the vector helpers they call (src/math/vector.ts: dot, add,
// scale, scale_self, length, normalize_self, reflection) sit in TypeScript files this image cannot
// compile.  This is a plain-JS transliteration (same operation order), run by node, with the rng
// replaced by the RT_SCATTER_COUNTER stream of include/rt.h: draw n of pixel p =
// (mix64(seed + p*0x9E3779B97F4A7C15 + (n+1)*0xD1B54A32D192ED03) >> 11) / 2^53.
// Output: tests/golden/scatter_vectors.json.
//
//   node tests/golden/gen_scatter.js > tests/golden/scatter_vectors.json
'use strict';

const M = (1n << 64n) - 1n;
function mix64(z) {
    z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & M;
    z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & M;
    return z ^ (z >> 31n);
}

class CounterRng {                 // the RNG interface scatter_ray uses: next() in [0, 1)
    constructor(seed, pixel) { this.seed = BigInt(seed); this.pixel = BigInt(pixel); this.n = 0n; }
    next() {
        const x = mix64((this.seed + this.pixel * 0x9E3779B97F4A7C15n + (this.n + 1n) * 0xD1B54A32D192ED03n) & M);
        this.n += 1n;
        return Number(x >> 11n) / 9007199254740992;
    }
}

// src/math/vector.ts, on plain arrays
function dot(a, b) { let s = 0; for (let i = 0; i < a.length; i++) s += a[i] * b[i]; return s; }
function add(a, b) { const r = []; for (let i = 0; i < a.length; i++) r[i] = a[i] + b[i]; return r; }
function scale(a, k) { const r = []; for (let i = 0; i < a.length; ++i) r[i] = a[i] * k; return r; }
function scale_self(a, k) { for (let i = 0; i < a.length; i++) a[i] *= k; return a; }
function length(a) { return Math.sqrt(dot(a, a)); }
function normalize_self(a) { return scale_self(a, 1.0 / length(a)); }
function reflection(v, n) { return add(v, scale(n, -dot(v, n) * 2)); }

function isotropic_sphere_sample(rng) {
    let vec;
    do {
        vec = [rng.next() * 2 - 1, rng.next() * 2 - 1, rng.next() * 2 - 1];
    } while (dot(vec, vec) > 1);
    return vec;
}

function scatter_ray(dir, normal, roughness, rng) {
    const rand_vec = isotropic_sphere_sample(rng);
    if (dot(rand_vec, normal) < 0) scale_self(rand_vec, -1);
    const ref_vec = add(scale(dir, 1 - roughness), scale(rand_vec, roughness));
    return normalize_self(ref_vec);
}

// splitmix64 stream for the case inputs (fixtures carry the inputs themselves)
function* stream(seed) {
    let s = BigInt(seed);
    for (;;) {
        s = (s + 0x9E3779B97F4A7C15n) & M;
        yield Number(mix64(s) >> 11n) / 9007199254740992;
    }
}

const hex = (x) => { const b = Buffer.alloc(8); b.writeDoubleLE(x); return b.toString('hex'); };
const g = stream(77);
const unit = () => {
    for (;;) {
        const v = [g.next().value * 2 - 1, g.next().value * 2 - 1, g.next().value * 2 - 1];
        const l = length(v);
        if (l > 0.1 && l <= 1) return scale(v, 1 / l);
    }
};

const cases = [];
const roughs = [1e-9, 0.05, 0.25, 0.5, 0.75, 1.0, 0.999, 0.3];
for (let k = 0; k < 64; k++) {
    const normal = k % 8 === 0 ? [0, 0, k % 16 === 0 ? 1 : -1] : unit();
    let dir = unit();
    if (dot(dir, normal) >= 0) dir = scale(dir, -1);
    if (k % 5 === 0) dir = scale(dir, 3.5);          // camera rays are unnormalised (keep_dir_unnormalized)
    const seed = k < 32 ? 12345 : Number(mix64(BigInt(k)) >> 11n);
    const pixel = k * 7919 + (k % 3) * 2073600;
    const roughness = roughs[k % roughs.length];
    const rng = new CounterRng(seed, pixel);
    const refl = reflection(dir, normal);
    const out = scatter_ray(refl.slice(), normal, roughness, rng);
    cases.push({
        seed: String(seed), pixel, roughness_hex: hex(roughness),
        dir_hex: dir.map(hex), normal_hex: normal.map(hex), reflected_hex: refl.map(hex),
        out_hex: out.map(hex), draws: Number(rng.n),
    });
}
// the stream itself: first draws of a few (seed, pixel) keys
const draws = [];
for (const [seed, pixel] of [[0, 0], [1, 0], [0, 1], [12345, 2073599], ['18446744073709551615', 7]]) {
    const rng = new CounterRng(seed, pixel);
    draws.push({ seed: String(seed), pixel, values_hex: [0, 1, 2, 3, 4, 5].map(() => hex(rng.next())) });
}
process.stdout.write(JSON.stringify({ generator: 'tests/golden/gen_scatter.js', node: process.version, cases, draws }) + '\n');
