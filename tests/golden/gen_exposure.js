// gen_exposure.js — golden vectors for the ExposureBuffer consumers, computed by V8 itself.
//
// The reference's exposure statistics, tone-mapper range and canvas conversion
// (src/view/exposure_buffer.ts:90-158, src/view/tone_mapping.ts:36-80,
// src/view/screen_canvas.ts:45-55,92-94) are plain JS number / typed-array code but sit in
// TypeScript files this image cannot compile.  This is a transliteration of those operations in
// plain JS (same operation order, same typed arrays), run by node, so Float32Array / Uint8ClampedArray
// stores, Math.min/max/sqrt and `<< 0` are V8's own.  Output: tests/golden/exposure_vectors.json.
//
//   node tests/golden/gen_exposure.js > tests/golden/exposure_vectors.json
'use strict';

// splitmix64 on BigInt: a deterministic f32 stream shared with nothing (fixtures carry the inputs)
function* stream(seed) {
    let s = BigInt(seed);
    const M = (1n << 64n) - 1n;
    for (;;) {
        s = (s + 0x9E3779B97F4A7C15n) & M;
        let z = s;
        z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & M;
        z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & M;
        z = z ^ (z >> 31n);
        yield Number(z >> 11n) / 9007199254740992;
    }
}

function luma(p, i) {                       // rgb_to_y: W_R*r + W_G*g + W_B*b
    return 0.299 * p[i] + 0.587 * p[i + 1] + 0.114 * p[i + 2];
}

function stats(p, n) {                      // get_mean, get_variance(mean), get_absolute_dev(mean)
    let mean = 0;
    for (let i = 0; i < n * 3; i += 3) mean += luma(p, i);
    mean /= n;
    let variance = 0;
    for (let i = 0; i < n * 3; i += 3) { const d = luma(p, i) - mean; variance += d * d; }
    variance /= n;
    let dev = 0;
    for (let i = 0; i < n * 3; i += 3) dev += Math.abs(luma(p, i) - mean);
    dev /= n;
    return [mean, variance, dev];
}

const clamp = (x, lo, hi) => Math.max(Math.min(x, hi), lo);

function range(mode, st, dr, min_d, max_d) {   // ToneMapper_{Identity,StdDevAroundMean,AbsDevAroundMean}
    if (mode === 0) return [0, 1];
    const coef = 1 << dr;
    const dev = mode === 1 ? Math.sqrt(st[1]) : st[2];
    let hi = Math.min(st[0] + dev, max_d);
    let lo = hi / coef;
    if (lo < min_d) { lo = min_d; hi = lo * coef; }
    return [lo, hi];
}

function tonemap(p, n, lo, hi) {            // discretize_to_screen + CanvasScreen.set_pixel_i
    const out = new Uint8ClampedArray(n * 4);
    const drange = hi - lo;
    for (let k = 0, i = 0; k < n; ++k, i += 3) {
        const y = luma(p, i);
        const scale = ((y - lo) / drange) / (y + Number.EPSILON);
        const c = p.slice(i, i + 2).map((v) => clamp(v * scale, 0.0, 1.0));
        const u8 = c.map((x) => (clamp(x, 0, 1) * 255) << 0);
        out[4 * k] = u8[0];
        out[4 * k + 1] = u8[1];
        out[4 * k + 2] = u8[2];
        out[4 * k + 3] = 0xff;
    }
    return out;
}

const hex = (x) => { const b = Buffer.alloc(8); b.writeDoubleLE(x); return b.toString('hex'); };

const cases = [];
const specs = [
    { name: 'uniform_0_2', n: 257, seed: 1, gen: (r) => 2 * r },
    { name: 'dark', n: 64, seed: 2, gen: (r) => 1e-4 * r },
    { name: 'bright_hdr', n: 100, seed: 3, gen: (r) => 50 * r * r * r },
    { name: 'edges', n: 8, seed: 4, gen: null },
];
for (const sp of specs) {
    const p = new Float32Array(sp.n * 3);
    if (sp.gen) {
        const g = stream(sp.seed);
        for (let i = 0; i < p.length; i++) p[i] = sp.gen(g.next().value);
    } else {
        p.set([0, 0, 0, 1, 1, 1, 0.5, 0.25, 0.125, 1e30, 0, 0, Infinity, 1, 1, 3, 2, 1, 1e-38, 0, 1e-45, 0.2, 0.7, 0.1]);
    }
    const n = sp.n;
    const st = stats(p, n);
    const ranges = [0, 1, 2].map((m) => range(m, st, 8, 1.0 / (1 << 8), 8.0));
    cases.push({
        name: sp.name,
        n_pixels: n,
        rgb_f32_hex: Buffer.from(p.buffer).toString('hex'),
        stats_hex: st.map(hex),
        ranges_hex: ranges.map((r) => r.map(hex)),
        rgba_stddev: Array.from(tonemap(p, n, ranges[1][0], ranges[1][1])),
        rgba_identity: Array.from(tonemap(p, n, 0, 1)),
    });
}
process.stdout.write(JSON.stringify({ generator: 'tests/golden/gen_exposure.js', node: process.version, cases }) + '\n');
