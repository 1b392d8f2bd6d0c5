// gen_texture.js — golden vectors for image textures, computed by V8 itself.
//
// Math.atan2 (V8's fdlibm port), uv_map_sphere (src/math/uv_mapping.ts:19-25) and the texel that
// ImageTexture.get_color (src/texture/texture_image.ts:40-63) reads, for random and special
// directions and several image sizes.  The TypeScript sources cannot be compiled here; this is a
// plain-JS transliteration of those expressions (same operation order), run by node.
// Output: tests/golden/texture_vectors.json.
//
//   node tests/golden/gen_texture.js > tests/golden/texture_vectors.json
'use strict';

const M = (1n << 64n) - 1n;
let s = 0x7E57n;
function rnd() {
    s = (s + 0x9E3779B97F4A7C15n) & M;
    let z = s;
    z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & M;
    z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & M;
    z ^= z >> 31n;
    return Number(z >> 11n) / 9007199254740992;
}
const hex = (x) => { const b = Buffer.alloc(8); b.writeDoubleLE(x); return b.toString('hex'); };

function uv_map_sphere(d) {
    const len = Math.sqrt((0 + d[0] * d[0]) + d[1] * d[1]);      // vector.length(vector.reduce(dir, 2))
    const u = Math.atan2(d[1], d[0]) / Math.PI / 2.0 + 0.5 - Number.EPSILON;
    const v = Math.atan2(d[2], len) / Math.PI + 0.5 - Number.EPSILON;
    return [u, v];
}

function texel(u, v, width, height) {
    if (u < 0 - Number.EPSILON || u > 1 - Number.EPSILON || v < 0 - Number.EPSILON || v > 1 - Number.EPSILON)
        return -1;
    const u_i = (u * width) << 0;
    const v_i = (v * height) << 0;
    return v_i * width + u_i;
}

const special = [0, -0, 1, -1, Infinity, -Infinity, NaN, 1e-300, -1e-300, 5e-324, 1e300, 0.5, 2.4375,
    1.1875, 0.4375, 0.6875, 0.75, 2 ** -27, 2 ** -29, 2 ** 66, 3, -2.5];
const atan2 = [];
for (const a of special) for (const b of special) atan2.push([a, b]);
for (let i = 0; i < 1500; i++) {
    let y = rnd() * 2 - 1, x = rnd() * 2 - 1;
    if (i % 3 === 1) y *= 10 ** Math.floor(rnd() * 20 - 10);
    if (i % 3 === 2) { x *= 10 ** Math.floor(rnd() * 40 - 20); y *= 10 ** Math.floor(rnd() * 40 - 20); }
    atan2.push([y, x]);
}
const sizes = [[1, 1], [7, 5], [64, 32], [1024, 512], [4096, 2048]];
const dirs = [[0, 0, 1], [0, 0, -1], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [-1, -0, 0], [-1, 0, -0],
    [0, 0, 0], [1, 1, 1], [-3.5, 2, 0.25]];
for (let i = 0; i < 1000; i++) {
    const d = [rnd() * 2 - 1, rnd() * 2 - 1, rnd() * 2 - 1];
    if (i % 4 === 1) d[2] = 0;
    if (i % 4 === 2) { const k = 10 ** (rnd() * 6 - 3); d[0] *= k; d[1] *= k; d[2] *= k; }
    dirs.push(d);
}
const uv = dirs.map((d) => {
    const [u, v] = uv_map_sphere(d);
    return { d_hex: d.map(hex), uv_hex: [hex(u), hex(v)], texel: sizes.map(([w, h]) => texel(u, v, w, h)) };
});
process.stdout.write(JSON.stringify({
    generator: 'tests/golden/gen_texture.js', node: process.version, sizes,
    atan2: atan2.map(([y, x]) => [hex(y), hex(x), hex(Math.atan2(y, x))]), uv,
}) + '\n');
