// rt_scene_json.cpp — scene description input.
//
// The reference hard-codes its scene in the shader: 7 materials
// (raytrace_compute.glsl:74-157), 3 lights (:199-224), 5 time-animated objects
// (:261-321) and an orbiting camera (:334-364). rt_scene_desc_parse reads the
// same content from JSON text, so a scene is data instead of code:
//
//   {
//     "materials": "reference" | [ {"name": "gold", "ambient": [r,g,b,a],
//                    "diffuse": [...], "specular": [...], "shininess": s,
//                    "emissive": [...], "reflectivity": x, "transparency": x,
//                    "refraction_index": x}, ... ],
//     "lights":    "reference" | [ {"position": [x,y,z], "ambient": [...],
//                    "diffuse": [...], "specular": [...]}, ... ],
//     "objects":   "reference" | [ item, ... ],
//     "camera":    "reference" | {"position": [...], "angles": [pitch, yaw, roll],
//                    "v_fov": deg, "aspect": a, "near": n, "far": f}
//   }
//
// An object item is {"sphere": {"position": [...], "radius": r}, "material": m},
// {"box": {"mins": [...], "maxs": [...], "position": [...], "angles": [...]},
// "material": m}, {"reference_objects": true} (the shipped scene at `time`,
// :236-321 — the reference's animation rules), {"room": true} (the benchmark
// room box, ±11, wall material) or {"bench_spheres": {"count": n, "seed": s}}
// (rt_bench_objects' seeded spheres without the room). A material is an index
// into the scene's table or a name: a "name" given in "materials", or one of
// the reference names (material1, material2, red_glass, green_glass,
// blue_glass, mirror, wall) while the reference table is used. Missing
// sections default to "reference"; missing material fields to 0 (ambient,
// emissive, ...) except refraction_index (1) and alpha channels given as 3
// components (1). Colours take 3 or 4 components.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "rt_internal.h"

using namespace rtamd;

namespace {

// ---- a small JSON reader (objects, arrays, numbers, strings, literals) ----
struct Json {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Json> items;                              // Array
    std::vector<std::pair<std::string, Json>> members;  // Object, in order
    const Json *get(const char *key) const {
        for (const auto &m : members)
            if (m.first == key) return &m.second;
        return nullptr;
    }
};

struct Parser {
    const char *p, *end;
    std::string err;
    int depth = 0;
    void ws() {
        while (p < end && std::isspace(static_cast<unsigned char>(*p))) ++p;
    }
    bool fail(const std::string &msg) {
        if (err.empty()) err = msg;
        return false;
    }
    bool literal(const char *word) {
        const size_t n = std::strlen(word);
        if (static_cast<size_t>(end - p) < n || std::strncmp(p, word, n) != 0) return false;
        p += n;
        return true;
    }
    bool string(std::string &out) {
        if (p >= end || *p != '"') return fail("expected a string");
        ++p;
        while (p < end && *p != '"') {
            char c = *p++;
            if (c == '\\') {
                if (p >= end) return fail("unterminated escape");
                const char e = *p++;
                switch (e) {
                    case '"': case '\\': case '/': c = e; break;
                    case 'b': c = '\b'; break;
                    case 'f': c = '\f'; break;
                    case 'n': c = '\n'; break;
                    case 'r': c = '\r'; break;
                    case 't': c = '\t'; break;
                    case 'u': {  // keep ASCII; other code points become '?'
                        if (end - p < 4) return fail("bad \\u escape");
                        const unsigned long v = std::strtoul(std::string(p, p + 4).c_str(), nullptr, 16);
                        c = v < 128 ? static_cast<char>(v) : '?';
                        p += 4;
                        break;
                    }
                    default: return fail("bad escape");
                }
            }
            out.push_back(c);
        }
        if (p >= end) return fail("unterminated string");
        ++p;
        return true;
    }
    bool value(Json &v) {
        if (++depth > 64) return fail("nesting too deep");
        ws();
        if (p >= end) return fail("unexpected end of input");
        bool ok = true;
        if (*p == '{') {
            ++p;
            v.kind = Json::Object;
            ws();
            if (p < end && *p == '}') {
                ++p;
            } else {
                for (;;) {
                    ws();
                    std::string key;
                    if (!string(key)) return false;
                    ws();
                    if (p >= end || *p != ':') return fail("expected ':'");
                    ++p;
                    Json m;
                    if (!value(m)) return false;
                    v.members.emplace_back(std::move(key), std::move(m));
                    ws();
                    if (p < end && *p == ',') { ++p; continue; }
                    if (p < end && *p == '}') { ++p; break; }
                    return fail("expected ',' or '}'");
                }
            }
        } else if (*p == '[') {
            ++p;
            v.kind = Json::Array;
            ws();
            if (p < end && *p == ']') {
                ++p;
            } else {
                for (;;) {
                    Json item;
                    if (!value(item)) return false;
                    v.items.push_back(std::move(item));
                    ws();
                    if (p < end && *p == ',') { ++p; continue; }
                    if (p < end && *p == ']') { ++p; break; }
                    return fail("expected ',' or ']'");
                }
            }
        } else if (*p == '"') {
            v.kind = Json::String;
            ok = string(v.str);
        } else if (literal("true")) {
            v.kind = Json::Bool;
            v.b = true;
        } else if (literal("false")) {
            v.kind = Json::Bool;
        } else if (literal("null")) {
            v.kind = Json::Null;
        } else {
            char *q = nullptr;
            const std::string tok(p, static_cast<size_t>(std::min<ptrdiff_t>(end - p, 64)));
            v.num = std::strtod(tok.c_str(), &q);
            if (q == tok.c_str()) return fail("unexpected character '" + std::string(1, *p) + "'");
            p += q - tok.c_str();
            v.kind = Json::Number;
        }
        --depth;
        return ok;
    }
};

// ---- scene construction ---------------------------------------------------
const char *const kRefMaterialNames[RT_REFERENCE_MATERIALS] = {"material1",   "material2",  "red_glass", "green_glass",
                                                              "blue_glass", "mirror", "wall"};

struct Builder {
    std::string err;
    bool fail(const std::string &msg) {
        if (err.empty()) err = msg;
        return false;
    }
    bool number(const Json *j, const char *what, float &out) {
        if (!j) return true;  // keep the default
        if (j->kind != Json::Number) return fail(std::string(what) + ": expected a number");
        out = static_cast<float>(j->num);
        return true;
    }
    // 3 or 4 components (a 3-component colour gets alpha `w3`)
    bool vec(const Json *j, const char *what, float *out, int n, float w3 = 1.0f) {
        if (!j) return true;
        if (j->kind != Json::Array || (j->items.size() != static_cast<size_t>(n) &&
                                       !(n == 4 && j->items.size() == 3)))
            return fail(std::string(what) + ": expected " + std::to_string(n) + " numbers");
        for (size_t i = 0; i < j->items.size(); ++i) {
            if (j->items[i].kind != Json::Number) return fail(std::string(what) + ": expected numbers");
            out[i] = static_cast<float>(j->items[i].num);
        }
        if (n == 4 && j->items.size() == 3) out[3] = w3;
        return true;
    }
    static bool is_reference(const Json *j) { return !j || (j->kind == Json::String && j->str == "reference"); }
};

}  // namespace

extern "C" int rt_scene_desc_parse(const char *json, float time, rt_object *objs, int max_objs, int *n_objs,
                                   rt_material *mats, int max_mats, int *n_mats, rt_light *lights, int max_lights,
                                   int *n_lights, rt_camera *cam, int *has_camera) {
    if (!json || !objs || !n_objs || !mats || !n_mats || !lights || !n_lights || max_objs < 0 || max_mats <= 0 ||
        max_lights < 0) {
        set_error("rt_scene_desc_parse: bad arguments");
        return RT_ERR_INVALID;
    }
    Parser ps{json, json + std::strlen(json)};
    Json root;
    if (!ps.value(root)) {
        set_error("rt_scene_desc_parse: JSON: " + ps.err + " at offset " + std::to_string(ps.p - json));
        return RT_ERR_INVALID;
    }
    ps.ws();
    if (ps.p != ps.end) {
        set_error("rt_scene_desc_parse: JSON: trailing characters at offset " + std::to_string(ps.p - json));
        return RT_ERR_INVALID;
    }
    if (root.kind != Json::Object) {
        set_error("rt_scene_desc_parse: the scene must be a JSON object");
        return RT_ERR_INVALID;
    }
    Builder B;
    // materials
    std::map<std::string, int> names;
    int nm = 0;
    const Json *jm = root.get("materials");
    if (Builder::is_reference(jm)) {
        if (max_mats < RT_REFERENCE_MATERIALS) B.fail("materials: need room for the 7 reference materials");
        else {
            rt_reference_materials(mats);
            nm = RT_REFERENCE_MATERIALS;
            for (int i = 0; i < nm; ++i) names[kRefMaterialNames[i]] = i;
        }
    } else if (jm->kind != Json::Array) {
        B.fail("materials: expected \"reference\" or an array");
    } else {
        for (const Json &m : jm->items) {
            if (nm >= max_mats || nm >= RT_MAX_MATERIALS) { B.fail("materials: too many"); break; }
            if (m.kind != Json::Object) { B.fail("materials: expected objects"); break; }
            rt_material r{};
            r.refraction_index = 1.0f;
            B.vec(m.get("ambient"), "ambient", r.ambient, 4);
            B.vec(m.get("diffuse"), "diffuse", r.diffuse, 4);
            B.vec(m.get("specular"), "specular", r.specular, 4);
            B.vec(m.get("emissive"), "emissive", r.emissive, 4);
            B.number(m.get("shininess"), "shininess", r.shininess);
            B.number(m.get("reflectivity"), "reflectivity", r.reflectivity);
            B.number(m.get("transparency"), "transparency", r.transparency);
            B.number(m.get("refraction_index"), "refraction_index", r.refraction_index);
            if (const Json *n = m.get("name")) {
                if (n->kind != Json::String) B.fail("materials: name must be a string");
                else names[n->str] = nm;
            }
            mats[nm++] = r;
        }
    }
    // lights
    int nl = 0;
    const Json *jl = root.get("lights");
    if (Builder::is_reference(jl)) {
        if (max_lights < RT_REFERENCE_LIGHTS) B.fail("lights: need room for the 3 reference lights");
        else {
            rt_reference_lights(lights);
            nl = RT_REFERENCE_LIGHTS;
        }
    } else if (jl->kind != Json::Array) {
        B.fail("lights: expected \"reference\" or an array");
    } else {
        for (const Json &l : jl->items) {
            if (nl >= max_lights || nl >= RT_MAX_LIGHTS) { B.fail("lights: too many"); break; }
            if (l.kind != Json::Object) { B.fail("lights: expected objects"); break; }
            rt_light r{};
            B.vec(l.get("position"), "position", r.position, 3);
            B.vec(l.get("ambient"), "ambient", r.ambient, 4);
            B.vec(l.get("diffuse"), "diffuse", r.diffuse, 4);
            B.vec(l.get("specular"), "specular", r.specular, 4);
            lights[nl++] = r;
        }
    }
    // objects
    int no = 0;
    auto room = [&](int at) -> bool {
        std::vector<rt_object> tmp(1);
        rt_bench_objects(0, 0, tmp.data());
        objs[at] = tmp[0];
        return true;
    };
    auto material = [&](const Json *j, int32_t &out) -> bool {
        if (!j) return B.fail("objects: every object needs a material");
        if (j->kind == Json::Number) {
            out = static_cast<int32_t>(j->num);
        } else if (j->kind == Json::String) {
            const auto it = names.find(j->str);
            if (it == names.end()) return B.fail("objects: unknown material \"" + j->str + "\"");
            out = it->second;
        } else {
            return B.fail("objects: material must be an index or a name");
        }
        if (out < 0 || out >= nm) return B.fail("objects: material index out of range");
        return true;
    };
    const Json *jo = root.get("objects");
    if (Builder::is_reference(jo)) {
        if (max_objs < RT_REFERENCE_OBJECTS) B.fail("objects: need room for the 5 reference objects");
        else {
            rt_reference_objects(time, objs);
            no = RT_REFERENCE_OBJECTS;
        }
    } else if (jo->kind != Json::Array) {
        B.fail("objects: expected \"reference\" or an array");
    } else {
        for (const Json &o : jo->items) {
            if (!B.err.empty()) break;
            if (o.kind != Json::Object) { B.fail("objects: expected objects"); break; }
            auto room_left = [&](int n) { return no + n <= max_objs && no + n <= RT_MAX_OBJECTS; };
            if (const Json *r = o.get("reference_objects")) {
                if (r->kind != Json::Bool || !r->b) continue;
                if (!room_left(RT_REFERENCE_OBJECTS)) { B.fail("objects: too many"); break; }
                rt_reference_objects(time, objs + no);
                no += RT_REFERENCE_OBJECTS;
            } else if (const Json *r2 = o.get("room")) {
                if (r2->kind != Json::Bool || !r2->b) continue;
                if (!room_left(1)) { B.fail("objects: too many"); break; }
                room(no++);
            } else if (const Json *bs = o.get("bench_spheres")) {
                float count = 0.0f, seed = 0.0f;
                if (bs->kind != Json::Object) { B.fail("bench_spheres: expected an object"); break; }
                B.number(bs->get("count"), "count", count);
                B.number(bs->get("seed"), "seed", seed);
                // integers in range (a float outside int / uint64 range would
                // make the conversions undefined)
                if (!(count >= 0.0f && count <= static_cast<float>(RT_MAX_OBJECTS)) || count != std::floor(count)) {
                    B.fail("bench_spheres: count must be an integer in [0, " + std::to_string(RT_MAX_OBJECTS) + "]");
                    break;
                }
                if (!(seed >= 0.0f && seed < 9007199254740992.0f) || seed != std::floor(seed)) {
                    B.fail("bench_spheres: seed must be a non-negative integer below 2^53");
                    break;
                }
                const int n = static_cast<int>(count);
                if (!room_left(n)) { B.fail("objects: too many"); break; }
                std::vector<rt_object> tmp(static_cast<size_t>(n) + 1);
                rt_bench_objects(n, static_cast<uint64_t>(seed), tmp.data());
                for (int i = 0; i < n; ++i) objs[no++] = tmp[static_cast<size_t>(i) + 1];
            } else if (const Json *sp = o.get("sphere")) {
                if (!room_left(1)) { B.fail("objects: too many"); break; }
                if (sp->kind != Json::Object) { B.fail("sphere: expected an object"); break; }
                rt_object r{};  // null box (:178): a sphere
                B.vec(sp->get("position"), "position", r.position, 3);
                B.number(sp->get("radius"), "radius", r.radius);
                if (!material(o.get("material"), r.material)) break;
                objs[no++] = r;
            } else if (const Json *bx = o.get("box")) {
                if (!room_left(1)) { B.fail("objects: too many"); break; }
                if (bx->kind != Json::Object) { B.fail("box: expected an object"); break; }
                rt_object r{};
                r.radius = -1.0f;  // null sphere (:179)
                B.vec(bx->get("mins"), "mins", r.box_mins, 3);
                B.vec(bx->get("maxs"), "maxs", r.box_maxs, 3);
                B.vec(bx->get("position"), "position", r.position, 3);
                B.vec(bx->get("angles"), "angles", r.angles, 3);
                if (!material(o.get("material"), r.material)) break;
                objs[no++] = r;
            } else {
                B.fail("objects: unknown item (sphere, box, room, bench_spheres, reference_objects)");
            }
        }
    }
    // camera
    int hc = 0;
    const Json *jc = root.get("camera");
    if (jc && !Builder::is_reference(jc)) {
        if (jc->kind != Json::Object) {
            B.fail("camera: expected \"reference\" or an object");
        } else if (cam) {
            rt_camera c;
            rt_reference_camera(time, &c);  // defaults: the reference's lens
            B.vec(jc->get("position"), "position", c.position, 3);
            B.vec(jc->get("angles"), "angles", c.angles, 3);
            B.number(jc->get("v_fov"), "v_fov", c.v_fov);
            B.number(jc->get("aspect"), "aspect", c.aspect);
            B.number(jc->get("near"), "near", c.near_plane);
            B.number(jc->get("far"), "far", c.far_plane);
            *cam = c;
            hc = 1;
        }
    }
    if (!B.err.empty()) {
        set_error("rt_scene_desc_parse: " + B.err);
        return RT_ERR_INVALID;
    }
    *n_objs = no;
    *n_mats = nm;
    *n_lights = nl;
    if (has_camera) *has_camera = hc;
    return RT_OK;
}
