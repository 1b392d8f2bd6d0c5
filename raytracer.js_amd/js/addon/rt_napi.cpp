// rt_napi.cpp — N-API (v8) binding of librt_amd.so for the JavaScript drop-in (../raytracer.js).
//
// Exports create / uploadScene / traceFrame / destroy / lastError / abiVersion (and setLights).  Typed arrays are
// passed zero-copy (napi_get_typedarray_info) and are only read/written during the call; the call is
// synchronous and blocks the event loop exactly like the reference's Raytracer.trace_frame()
// (src/raytracer.ts:308-330).  A negative RT_E_* code becomes a thrown JS Error whose `code` is
// the RT_E_* name, matching the reference's "errors are thrown JS Errors" contract.
#include <chrono>
#include <node_api.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "rt.h"

namespace {

const char *code_name(int rc)
{
    switch (rc) {
    case RT_E_INVALID: return "RT_E_INVALID";
    case RT_E_HIP: return "RT_E_HIP";
    case RT_E_UNSUPPORTED: return "RT_E_UNSUPPORTED";
    case RT_E_NOSCENE: return "RT_E_NOSCENE";
    case RT_E_FAULT: return "RT_E_FAULT";
    case RT_E_NODEVICE: return "RT_E_NODEVICE";
    case RT_E_TREE: return "RT_E_TREE";
    case RT_E_STALE: return "RT_E_STALE";
    default: return "RT_E_UNKNOWN";
    }
}

bool throw_rc(napi_env env, int rc)
{
    if (rc >= 0) return false;
    napi_throw_error(env, code_name(rc), rt_last_error());
    return true;
}

#define NAPI_TRY(call)                                                        \
    do {                                                                      \
        if ((call) != napi_ok) {                                              \
            const napi_extended_error_info *info_ = nullptr;                  \
            napi_get_last_error_info(env, &info_);                            \
            bool pending_ = false;                                            \
            napi_is_exception_pending(env, &pending_);                        \
            if (!pending_)                                                    \
                napi_throw_error(env, "RT_E_INVALID",                         \
                                 info_ && info_->error_message ? info_->error_message : #call); \
            return nullptr;                                                   \
        }                                                                     \
    } while (0)

struct Typed {
    void *data = nullptr;
    size_t length = 0;          // elements
    napi_typedarray_type type = napi_int8_array;
};

// Read a typed array property (optional: returns false when undefined/null)
bool get_typed(napi_env env, napi_value obj, const char *key, napi_typedarray_type want, Typed &out, bool required)
{
    napi_value v;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok) return false;
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_undefined || t == napi_null) {
        if (required) napi_throw_error(env, "RT_E_INVALID", (std::string("missing typed array: ") + key).c_str());
        return false;
    }
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) {
        napi_throw_error(env, "RT_E_INVALID", (std::string("not a typed array: ") + key).c_str());
        return false;
    }
    napi_value ab;
    size_t off;
    napi_get_typedarray_info(env, v, &out.type, &out.length, &out.data, &ab, &off);
    if (out.type != want) {
        napi_throw_error(env, "RT_E_INVALID", (std::string("wrong typed array type: ") + key).c_str());
        return false;
    }
    return true;
}

bool get_number(napi_env env, napi_value obj, const char *key, double &out)
{
    napi_value v;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok) return false;
    if (napi_get_value_double(env, v, &out) != napi_ok) {
        napi_throw_error(env, "RT_E_INVALID", (std::string("not a number: ") + key).c_str());
        return false;
    }
    return true;
}

// optional numeric property: `out` keeps its value when the property is absent / undefined
bool get_number_opt(napi_env env, napi_value obj, const char *key, double &out)
{
    bool has = false;
    if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return true;
    napi_value v;
    napi_valuetype vt;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok || napi_typeof(env, v, &vt) != napi_ok) return false;
    if (vt == napi_undefined) return true;
    return get_number(env, obj, key, out);
}

bool get_vec(napi_env env, napi_value obj, const char *key, double *out, uint32_t n)
{
    napi_value v;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok) return false;
    for (uint32_t i = 0; i < n; i++) {
        napi_value e;
        if (napi_get_element(env, v, i, &e) != napi_ok || napi_get_value_double(env, e, &out[i]) != napi_ok) {
            napi_throw_error(env, "RT_E_INVALID", (std::string("bad numeric array: ") + key).c_str());
            return false;
        }
    }
    return true;
}

rt_ctx *unwrap(napi_env env, napi_value v)
{
    void *p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_error(env, "RT_E_INVALID", "not a live rt context");
        return nullptr;
    }
    rt_ctx **slot = static_cast<rt_ctx **>(p);
    if (!*slot) {
        napi_throw_error(env, "RT_E_INVALID", "rt context already destroyed");
        return nullptr;
    }
    return *slot;
}

void finalize_ctx(napi_env, void *data, void *)
{
    rt_ctx **slot = static_cast<rt_ctx **>(data);
    if (*slot) rt_destroy(*slot);
    delete slot;
}

// create(device) or create([devices...], stripe_rows): rt_create_desc (include/rt.h).  A list
// makes one context drive several GPUs: row stripes per device, gathered on devices[0] over RCCL.
napi_value Create(napi_env env, napi_callback_info info)
{
    size_t argc = 2;
    napi_value argv[2];
    NAPI_TRY(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    rt_create_desc d;
    memset(&d, 0, sizeof d);
    bool is_list = false;
    if (argc >= 1) NAPI_TRY(napi_is_array(env, argv[0], &is_list));
    if (is_list) {
        uint32_t n = 0;
        NAPI_TRY(napi_get_array_length(env, argv[0], &n));
        if (n < 1 || n > RT_MAX_DEVICES) {
            napi_throw_error(env, "RT_E_INVALID", "devices: a list of 1..8 GPU ordinals");
            return nullptr;
        }
        d.n_devices = (int32_t)n;
        for (uint32_t k = 0; k < n; k++) {
            napi_value v;
            NAPI_TRY(napi_get_element(env, argv[0], k, &v));
            if (napi_get_value_int32(env, v, &d.devices[k]) != napi_ok) {
                napi_throw_error(env, "RT_E_INVALID", "devices: a list of 1..8 GPU ordinals");
                return nullptr;
            }
        }
    } else if (argc >= 1) {
        napi_get_value_int32(env, argv[0], &d.device);
    }
    if (argc >= 2) napi_get_value_int32(env, argv[1], &d.stripe_rows);
    rt_ctx *ctx = nullptr;
    if (throw_rc(env, rt_create(&d, &ctx))) return nullptr;
    rt_ctx **slot = new rt_ctx *(ctx);
    napi_value ext;
    NAPI_TRY(napi_create_external(env, slot, finalize_ctx, nullptr, &ext));
    return ext;
}

napi_value Destroy(napi_env env, napi_callback_info info)
{
    size_t argc = 1;
    napi_value argv[1];
    NAPI_TRY(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    void *p = nullptr;
    if (argc < 1 || napi_get_value_external(env, argv[0], &p) != napi_ok || !p) return nullptr;
    rt_ctx **slot = static_cast<rt_ctx **>(p);
    if (*slot) rt_destroy(*slot);
    *slot = nullptr;
    return nullptr;
}

napi_value set_num(napi_env env, napi_value obj, const char *k, double v);
napi_value update_stats_obj(napi_env env, const rt_update_stats &st);

// uploadScene(ctx, scene) / updateScene(ctx, scene) -> stats: the flattened scene as typed arrays.
napi_value scene_call(napi_env env, napi_callback_info info, bool update)
{
    size_t argc = 2;
    napi_value argv[2];
    NAPI_TRY(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 2) { napi_throw_error(env, "RT_E_INVALID", "uploadScene(ctx, scene)"); return nullptr; }
    rt_ctx *ctx = unwrap(env, argv[0]);
    if (!ctx) return nullptr;
    napi_value s = argv[1];
    Typed npos, nsize, npar, nch, nb, nc, list, et, eg, es, esub, sresp, slight, smirror, srough, srgb, ri, simg;
    if (!get_typed(env, s, "node_pos", napi_float64_array, npos, true) ||
        !get_typed(env, s, "node_size", napi_float64_array, nsize, true) ||
        !get_typed(env, s, "node_parent", napi_int32_array, npar, true) ||
        !get_typed(env, s, "node_child", napi_int32_array, nch, true) ||
        !get_typed(env, s, "node_ent_begin", napi_int32_array, nb, true) ||
        !get_typed(env, s, "node_ent_count", napi_int32_array, nc, true) ||
        !get_typed(env, s, "list_entity", napi_int32_array, list, true) ||
        !get_typed(env, s, "ent_type", napi_int32_array, et, true) ||
        !get_typed(env, s, "ent_geom", napi_float64_array, eg, true) ||
        !get_typed(env, s, "ent_shade", napi_int32_array, es, true) ||
        !get_typed(env, s, "ent_substance", napi_int32_array, esub, true) ||
        !get_typed(env, s, "shade_response", napi_int32_array, sresp, true) ||
        !get_typed(env, s, "shade_light", napi_int32_array, slight, true) ||
        !get_typed(env, s, "shade_mirror", napi_int32_array, smirror, true) ||
        !get_typed(env, s, "shade_roughness", napi_float64_array, srough, true) ||
        !get_typed(env, s, "shade_rgb", napi_float64_array, srgb, true) ||
        !get_typed(env, s, "substance_ri", napi_float64_array, ri, true))
        return nullptr;
    // ImageTextures: shade_image (Int32Array, optional) and images [{width, height, rgb: Uint8Array}]
    bool has_simg = false;
    napi_has_named_property(env, s, "shade_image", &has_simg);
    if (has_simg && !get_typed(env, s, "shade_image", napi_int32_array, simg, true)) return nullptr;
    std::vector<rt_image_desc> images;
    bool has_images = false;
    napi_has_named_property(env, s, "images", &has_images);
    if (has_images) {
        napi_value arr;
        uint32_t ni = 0;
        NAPI_TRY(napi_get_named_property(env, s, "images", &arr));
        NAPI_TRY(napi_get_array_length(env, arr, &ni));
        images.resize(ni);
        for (uint32_t i = 0; i < ni; i++) {
            napi_value im;
            NAPI_TRY(napi_get_element(env, arr, i, &im));
            double w = 0, h = 0;
            Typed px;
            if (!get_number(env, im, "width", w) || !get_number(env, im, "height", h) ||
                !get_typed(env, im, "rgb", napi_uint8_array, px, true))
                return nullptr;
            if (px.length < (size_t)w * (size_t)h * 3) {
                napi_throw_error(env, "RT_E_INVALID", "uploadScene: image rgb shorter than width*height*3");
                return nullptr;
            }
            images[i].width = (int32_t)w;
            images[i].height = (int32_t)h;
            images[i].rgb = (const uint8_t *)px.data;
        }
    }
    const size_t n = nsize.length, ne = et.length, ns = sresp.length;
    if (npos.length != 3 * n || npar.length != n || nch.length != 8 * n || nb.length != n || nc.length != n ||
        eg.length != 9 * ne || es.length != ne || esub.length != ne || slight.length != ns || smirror.length != ns ||
        srough.length != ns || srgb.length != 3 * ns || (has_simg && simg.length != ns)) {
        napi_throw_error(env, "RT_E_INVALID", "uploadScene: inconsistent array lengths");
        return nullptr;
    }
    std::vector<rt_shade> shades(ns);
    for (size_t i = 0; i < ns; i++) {
        rt_shade &sh = shades[i];
        memset(&sh, 0, sizeof sh);
        sh.response = static_cast<int32_t *>(sresp.data)[i];
        sh.light = static_cast<int32_t *>(slight.data)[i];
        sh.mirror = static_cast<int32_t *>(smirror.data)[i];
        sh.roughness = static_cast<double *>(srough.data)[i];
        sh.image = has_simg ? static_cast<int32_t *>(simg.data)[i] : 0;
        for (int k = 0; k < 3; k++) sh.rgb[k] = static_cast<double *>(srgb.data)[3 * i + k];
    }
    rt_scene_desc d;
    memset(&d, 0, sizeof d);
    d.n_nodes = (int32_t)n;
    d.n_list = (int32_t)list.length;
    d.n_entities = (int32_t)ne;
    d.n_shades = (int32_t)ns;
    d.n_substances = (int32_t)ri.length;
    d.node_pos = (const double *)npos.data;
    d.node_size = (const double *)nsize.data;
    d.node_parent = (const int32_t *)npar.data;
    d.node_child = (const int32_t *)nch.data;
    d.node_ent_begin = (const int32_t *)nb.data;
    d.node_ent_count = (const int32_t *)nc.data;
    d.list_entity = (const int32_t *)list.data;
    d.ent_type = (const int32_t *)et.data;
    d.ent_geom = (const double *)eg.data;
    d.ent_shade = (const int32_t *)es.data;
    d.ent_substance = (const int32_t *)esub.data;
    d.shades = shades.data();
    d.substance_ri = (const double *)ri.data;
    d.n_images = (int32_t)images.size();
    d.images = images.data();
    if (!update) {
        throw_rc(env, rt_upload_scene(ctx, &d));
        return nullptr;
    }
    rt_update_stats st;
    if (throw_rc(env, rt_update_scene(ctx, &d, &st))) return nullptr;
    return update_stats_obj(env, st);
}

napi_value UploadScene(napi_env env, napi_callback_info info) { return scene_call(env, info, false); }
napi_value UpdateScene(napi_env env, napi_callback_info info) { return scene_call(env, info, true); }

napi_value update_stats_obj(napi_env env, const rt_update_stats &st)
{
    napi_value o;
    napi_create_object(env, &o);
    set_num(env, o, "full", st.full);
    set_num(env, o, "dirty_nodes", st.dirty_nodes);
    set_num(env, o, "new_nodes", st.new_nodes);
    set_num(env, o, "moved_regions", st.moved_regions);
    set_num(env, o, "changed_entities", st.changed_entities);
    set_num(env, o, "bytes", (double)st.bytes);
    set_num(env, o, "host_ms", st.host_ms);
    set_num(env, o, "total_ms", st.total_ms);
    return o;
}

// applyEdit(ctx, edit) -> stats, or null when the resident scene cannot take it (RT_E_STALE: the
// caller uploads in full).  `edit` carries rt_edit_desc's arrays (include/rt.h) as typed arrays and
// the whole shade / substance tables in uploadScene's form.
// sceneSlots(ctx, n) -> {slots: Int32Array (slot of each DFS id of the last uploaded desc), n_slots},
// or null after an edit
napi_value SceneSlots(napi_env env, napi_callback_info info)
{
    size_t argc = 2;
    napi_value argv[2];
    NAPI_TRY(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 2) { napi_throw_error(env, "RT_E_INVALID", "sceneSlots(ctx, n)"); return nullptr; }
    rt_ctx *ctx = unwrap(env, argv[0]);
    if (!ctx) return nullptr;
    int32_t n = 0;
    NAPI_TRY(napi_get_value_int32(env, argv[1], &n));
    if (n < 0) { napi_throw_error(env, "RT_E_INVALID", "sceneSlots: n < 0"); return nullptr; }
    void *data = nullptr;
    napi_value ab, arr;
    NAPI_TRY(napi_create_arraybuffer(env, sizeof(int32_t) * (size_t)n, &data, &ab));
    NAPI_TRY(napi_create_typedarray(env, napi_int32_array, (size_t)n, ab, 0, &arr));
    int32_t n_slots = 0;
    const int r = rt_scene_node_slots(ctx, (int32_t *)data, n, &n_slots);
    if (r == RT_E_STALE) {
        napi_value nul;
        napi_get_null(env, &nul);
        return nul;
    }
    if (throw_rc(env, r)) return nullptr;
    napi_value o;
    napi_create_object(env, &o);
    NAPI_TRY(napi_set_named_property(env, o, "slots", arr));
    set_num(env, o, "n_slots", n_slots);
    return o;
}

// setLights(ctx, [{pos: [x, y, z], rgb: [r, g, b]}, ...], ambient): rt_set_lights, the shadow-ray
// build extension (include/rt.h); an empty list restores the reference
napi_value SetLights(napi_env env, napi_callback_info info)
{
    size_t argc = 3;
    napi_value argv[3];
    NAPI_TRY(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 2) { napi_throw_error(env, "RT_E_INVALID", "setLights(ctx, lights, ambient)"); return nullptr; }
    rt_ctx *ctx = unwrap(env, argv[0]);
    if (!ctx) return nullptr;
    bool is_list = false;
    NAPI_TRY(napi_is_array(env, argv[1], &is_list));
    if (!is_list) { napi_throw_error(env, "RT_E_INVALID", "setLights: lights must be an array"); return nullptr; }
    uint32_t n = 0;
    NAPI_TRY(napi_get_array_length(env, argv[1], &n));
    if (n > RT_MAX_LIGHTS) { napi_throw_error(env, "RT_E_INVALID", "setLights: too many lights"); return nullptr; }
    rt_light lights[RT_MAX_LIGHTS];
    memset(lights, 0, sizeof lights);
    for (uint32_t k = 0; k < n; k++) {
        napi_value e;
        NAPI_TRY(napi_get_element(env, argv[1], k, &e));
        if (!get_vec(env, e, "pos", lights[k].pos, 3) || !get_vec(env, e, "rgb", lights[k].rgb, 3)) return nullptr;
    }
    double ambient = 0;
    if (argc >= 3) NAPI_TRY(napi_get_value_double(env, argv[2], &ambient));
    if (throw_rc(env, rt_set_lights(ctx, lights, (int32_t)n, ambient))) return nullptr;
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

napi_value ApplyEdit(napi_env env, napi_callback_info info)
{
    size_t argc = 2;
    napi_value argv[2];
    NAPI_TRY(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 2) { napi_throw_error(env, "RT_E_INVALID", "applyEdit(ctx, edit)"); return nullptr; }
    rt_ctx *ctx = unwrap(env, argv[0]);
    if (!ctx) return nullptr;
    napi_value s = argv[1];
    Typed rs, rc, rch, ru, ss, sb, sc, se, st, ssh, sg, ue, uv, dns, dnv, dsh, sresp, slight, smirror, srough, srgb, simg, ri;
    if (!get_typed(env, s, "rec_slot", napi_int32_array, rs, true) ||
        !get_typed(env, s, "rec_cube", napi_float64_array, rc, true) ||
        !get_typed(env, s, "rec_child", napi_int32_array, rch, true) ||
        !get_typed(env, s, "rec_up", napi_int32_array, ru, true) ||
        !get_typed(env, s, "set_slot", napi_int32_array, ss, true) ||
        !get_typed(env, s, "set_begin", napi_int32_array, sb, true) ||
        !get_typed(env, s, "set_count", napi_int32_array, sc, true) ||
        !get_typed(env, s, "set_ent", napi_int32_array, se, true) ||
        !get_typed(env, s, "set_type", napi_int32_array, st, true) ||
        !get_typed(env, s, "set_shade", napi_int32_array, ssh, true) ||
        !get_typed(env, s, "set_geom", napi_float64_array, sg, true) ||
        !get_typed(env, s, "sub_ent", napi_int32_array, ue, true) ||
        !get_typed(env, s, "sub_val", napi_int32_array, uv, true) ||
        !get_typed(env, s, "dfs_new_slot", napi_int32_array, dns, true) ||
        !get_typed(env, s, "dfs_new_val", napi_int32_array, dnv, true) ||
        !get_typed(env, s, "dfs_shift", napi_int32_array, dsh, true) ||
        !get_typed(env, s, "shade_response", napi_int32_array, sresp, true) ||
        !get_typed(env, s, "shade_light", napi_int32_array, slight, true) ||
        !get_typed(env, s, "shade_mirror", napi_int32_array, smirror, true) ||
        !get_typed(env, s, "shade_roughness", napi_float64_array, srough, true) ||
        !get_typed(env, s, "shade_rgb", napi_float64_array, srgb, true) ||
        !get_typed(env, s, "shade_image", napi_int32_array, simg, true) ||
        !get_typed(env, s, "substance_ri", napi_float64_array, ri, true))
        return nullptr;
    double n_slots = 0, n_ent = 0, scatter = 0;
    if (!get_number(env, s, "n_slots", n_slots) || !get_number(env, s, "n_entities", n_ent) ||
        !get_number(env, s, "scatter", scatter))
        return nullptr;
    const size_t nr = rs.length, nset = ss.length, nm = se.length, ns = sresp.length;
    if (rc.length != 4 * nr || rch.length != 8 * nr || ru.length != 2 * nr || sb.length != nset || sc.length != nset ||
        st.length != nm || ssh.length != nm || sg.length != 9 * nm || uv.length != ue.length ||
        dnv.length != dns.length || slight.length != ns || smirror.length != ns || srough.length != ns ||
        srgb.length != 3 * ns || simg.length != ns) {
        napi_throw_error(env, "RT_E_INVALID", "applyEdit: inconsistent array lengths");
        return nullptr;
    }
    std::vector<rt_shade> shades(ns);
    for (size_t i = 0; i < ns; i++) {
        rt_shade &sh = shades[i];
        memset(&sh, 0, sizeof sh);
        sh.response = static_cast<int32_t *>(sresp.data)[i];
        sh.light = static_cast<int32_t *>(slight.data)[i];
        sh.mirror = static_cast<int32_t *>(smirror.data)[i];
        sh.roughness = static_cast<double *>(srough.data)[i];
        sh.image = static_cast<int32_t *>(simg.data)[i];
        for (int k = 0; k < 3; k++) sh.rgb[k] = static_cast<double *>(srgb.data)[3 * i + k];
    }
    rt_edit_desc d;
    memset(&d, 0, sizeof d);
    d.n_slots = (int32_t)n_slots;
    d.n_entities = (int32_t)n_ent;
    d.n_rec = (int32_t)nr;
    d.rec_slot = (const int32_t *)rs.data;
    d.rec_cube = (const double *)rc.data;
    d.rec_child = (const int32_t *)rch.data;
    d.rec_up = (const int32_t *)ru.data;
    d.n_set = (int32_t)nset;
    d.set_slot = (const int32_t *)ss.data;
    d.set_begin = (const int32_t *)sb.data;
    d.set_count = (const int32_t *)sc.data;
    d.n_member = (int32_t)nm;
    d.set_ent = (const int32_t *)se.data;
    d.set_type = (const int32_t *)st.data;
    d.set_shade = (const int32_t *)ssh.data;
    d.set_geom = (const double *)sg.data;
    d.n_sub = (int32_t)ue.length;
    d.sub_ent = (const int32_t *)ue.data;
    d.sub_val = (const int32_t *)uv.data;
    d.n_dfs_new = (int32_t)dns.length;
    d.dfs_new_slot = (const int32_t *)dns.data;
    d.dfs_new_val = (const int32_t *)dnv.data;
    d.n_dfs_shift = (int32_t)dsh.length;
    d.dfs_shift = (const int32_t *)dsh.data;
    d.scatter = scatter != 0;
    d.n_shades = (int32_t)ns;
    d.shades = shades.data();
    d.n_substances = (int32_t)ri.length;
    d.substance_ri = (const double *)ri.data;
    rt_update_stats u;
    memset(&u, 0, sizeof u);
    const int r = rt_apply_edit(ctx, &d, &u);
    if (r == RT_E_STALE) {
        napi_value nul;
        napi_get_null(env, &nul);
        return nul;
    }
    if (throw_rc(env, r)) return nullptr;
    return update_stats_obj(env, u);
}

napi_value set_num(napi_env env, napi_value obj, const char *k, double v)
{
    napi_value x;
    napi_create_double(env, v, &x);
    napi_set_named_property(env, obj, k, x);
    return obj;
}

napi_value TraceFrame(napi_env env, napi_callback_info info)
{
    size_t argc = 8;
    napi_value argv[8];
    NAPI_TRY(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 4) {
        napi_throw_error(env, "RT_E_INVALID", "traceFrame(ctx, cam, cfg, pixels[, hitEntity, hitNode, status, wantStats])");
        return nullptr;
    }
    rt_ctx *ctx = unwrap(env, argv[0]);
    if (!ctx) return nullptr;
    rt_camera_desc cam;
    rt_config_desc cfg;
    memset(&cam, 0, sizeof cam);
    memset(&cfg, 0, sizeof cfg);
    double w, h, refmax, defsub, att, wgt;
    if (!get_number(env, argv[1], "width", w) || !get_number(env, argv[1], "height", h) ||
        !get_vec(env, argv[1], "pos", cam.pos, 3) || !get_vec(env, argv[1], "fr", cam.fr, 3) ||
        !get_vec(env, argv[1], "lf", cam.lf, 3) || !get_vec(env, argv[1], "up", cam.up, 3) ||
        !get_vec(env, argv[1], "scan_h", cam.scan_h, 2) || !get_vec(env, argv[1], "scan_v", cam.scan_v, 2))
        return nullptr;
    if (!get_number(env, argv[2], "refmax", refmax) || !get_number(env, argv[2], "default_substance", defsub) ||
        !get_vec(env, argv[2], "sky_rgb", cfg.sky_rgb, 3) ||
        !get_number(env, argv[2], "distance_attenuation_factor", att) || !get_number(env, argv[2], "col_weight", wgt))
        return nullptr;
    cam.width = (int32_t)w;
    cam.height = (int32_t)h;
    cfg.refmax = (int32_t)refmax;
    cfg.default_substance = (int32_t)defsub;
    cfg.distance_attenuation_factor = att;
    cfg.col_weight = wgt;
    double seed = 0, smode = RT_SCATTER_REJECT, sky_image = 0;
    if (!get_number_opt(env, argv[2], "scatter_seed", seed) || !get_number_opt(env, argv[2], "scatter_mode", smode) ||
        !get_number_opt(env, argv[2], "sky_image", sky_image))
        return nullptr;
    cfg.sky_image = (int32_t)sky_image;
    cfg.scatter_seed = seed > 0 ? (uint64_t)seed : 0;
    cfg.scatter_mode = (int32_t)smode;
    auto typed_arg = [&](size_t i, napi_typedarray_type want, Typed &t) -> bool {
        if (argc <= i) return false;
        napi_valuetype vt;
        napi_typeof(env, argv[i], &vt);
        if (vt == napi_undefined || vt == napi_null) return false;
        napi_value ab;
        size_t off;
        bool is_ta = false;
        napi_is_typedarray(env, argv[i], &is_ta);
        if (!is_ta) return false;
        napi_get_typedarray_info(env, argv[i], &t.type, &t.length, &t.data, &ab, &off);
        return t.type == want;
    };
    Typed px, he, hn, st;
    if (!typed_arg(3, napi_float32_array, px)) { napi_throw_error(env, "RT_E_INVALID", "pixels must be a Float32Array"); return nullptr; }
    const size_t P = (size_t)cam.width * (size_t)cam.height;
    if (px.length != 3 * P) { napi_throw_error(env, "RT_E_INVALID", "pixels length != width*height*3"); return nullptr; }
    bool has_he = typed_arg(4, napi_int32_array, he), has_hn = typed_arg(5, napi_int32_array, hn),
         has_st = typed_arg(6, napi_uint8_array, st);
    if ((has_he && he.length != P) || (has_hn && hn.length != P) || (has_st && st.length != P)) {
        napi_throw_error(env, "RT_E_INVALID", "id buffers must have width*height elements");
        return nullptr;
    }
    // work counters are opt-in (wantStats): counting runs the fused stats kernel, not the split
    // passes, so a plain frame only reports its wall time
    bool want_stats = false;
    if (argc > 7) {
        napi_valuetype vt;
        napi_typeof(env, argv[7], &vt);
        if (vt == napi_boolean) napi_get_value_bool(env, argv[7], &want_stats);
    }
    rt_stats stats;
    memset(&stats, 0, sizeof stats);
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = rt_trace_frame(ctx, &cam, &cfg, (float *)px.data, has_he ? (int32_t *)he.data : nullptr,
                                  has_hn ? (int32_t *)hn.data : nullptr, has_st ? (uint8_t *)st.data : nullptr,
                                  want_stats ? &stats : nullptr);
    if (throw_rc(env, rc)) return nullptr;
    napi_value out;
    napi_create_object(env, &out);
    if (!want_stats) {
        set_num(env, out, "frame_ms", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        return out;
    }
    set_num(env, out, "segments", (double)stats.segments);
    set_num(env, out, "n_ret", (double)stats.n_ret);
    set_num(env, out, "n_slot", (double)stats.n_slot);
    set_num(env, out, "n_loc", (double)stats.n_loc);
    set_num(env, out, "n_sph", (double)stats.n_sph);
    set_num(env, out, "n_box", (double)stats.n_box);
    set_num(env, out, "n_tri", (double)stats.n_tri);
    set_num(env, out, "n_hit", (double)stats.n_hit);
    set_num(env, out, "primary", (double)stats.primary);
    set_num(env, out, "n_warn", (double)stats.n_warn);
    set_num(env, out, "n_fault", (double)stats.n_fault);
    set_num(env, out, "kernel_ms", stats.kernel_ms);
    set_num(env, out, "frame_ms", stats.frame_ms);
    return out;
}

napi_value LastError(napi_env env, napi_callback_info)
{
    napi_value s;
    napi_create_string_utf8(env, rt_last_error(), NAPI_AUTO_LENGTH, &s);
    return s;
}

napi_value AbiVersion(napi_env env, napi_callback_info)
{
    napi_value v;
    napi_create_int32(env, rt_abi_version(), &v);
    return v;
}

napi_value Init(napi_env env, napi_value exports)
{
    napi_property_descriptor props[] = {
        {"create", nullptr, Create, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"destroy", nullptr, Destroy, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"uploadScene", nullptr, UploadScene, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"updateScene", nullptr, UpdateScene, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"applyEdit", nullptr, ApplyEdit, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"sceneSlots", nullptr, SceneSlots, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"setLights", nullptr, SetLights, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"traceFrame", nullptr, TraceFrame, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"lastError", nullptr, LastError, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"abiVersion", nullptr, AbiVersion, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
    };
    napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
