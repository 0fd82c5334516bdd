/*
 * glref — TEST INFRASTRUCTURE ONLY (oracle). Never linked into the product.
 *
 * Runs the reference's own compute shader,
 *   /root/reference/OpenGLRaytracer/raytrace_compute.glsl,
 * on Mesa llvmpipe (software GL on the host cores) with no window system:
 * the DRI swrast driver is dlopen()ed, a surfaceless OpenGL 4.3 core context
 * is created and made current, and the shader is dispatched exactly like the
 * reference's frame driver does (OpenGLRaytracer/main.cpp:219-238:
 * glUseProgram, glBindImageTexture unit 0, glUniform1f("time"),
 * glDispatchCompute(W,H,1), glFinish).
 *
 * The shader text is NOT in the repository: oracle/Makefile links the file
 * from /root/reference into oracle/_ref/libglref.so (git-ignored) as a binary
 * blob. Patches are applied here, at run time, by exact string substitution;
 * each one must match exactly once or the render fails loudly:
 *   P1 (always)   raytrace_compute.glsl:7  `uniform image2D output_texture;`
 *                 -> `writeonly uniform ...` (Mesa refuses an image uniform
 *                 with neither a format qualifier nor writeonly; no semantic
 *                 change).
 *   P2 (depth)    :22  MAX_RAYTRACE_DEPTH = <D>.
 *   P3 (scene)    :261-321  objects[] / objects_count replaced by caller GLSL.
 *   P5 (crop)     :327-329,404  width/height/pixel offset from uniforms so a
 *                 sub-rectangle of a large frame can be rendered; the pixel
 *                 -> ray mapping is unchanged.
 *   P4 (probe)    :401  the colour is replaced by an intermediate value
 *                 (ray dir, closest hit, shadow mask, normal, hit point,
 *                 and (probe 5) the camera matrices: pixel (x,y) holds element
 *                 [x%4][y%4] of inverse(proj*view), view and proj; (probe 7)
 *                 object (x/4)'s box transforms: element [x%4][y%4] of
 *                 calc_transform_matrix, its inverse and the normal matrix
 *                 transpose(inverse(mat3(.))) as intersect_box_object forms them).
 * The output texture is RGBA32F (unclamped floats) instead of the shipped
 * RGBA8 (main.cpp:152-159,223); alpha is always 0 (raytrace_compute.glsl:404).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <GL/glcorearb.h>
#include <GL/internal/dri_interface.h>

extern const char _binary_raytrace_compute_glsl_start[];
extern const char _binary_raytrace_compute_glsl_end[];

static char g_err[1024];
static void set_err(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}
const char *glref_last_error(void) { return g_err; }

/* ---- GL entry points (resolved through libglapi's dispatch) ---------- */
#define GLFUNCS(X)                                                        \
    X(PFNGLCREATESHADERPROC, glCreateShader)                              \
    X(PFNGLSHADERSOURCEPROC, glShaderSource)                              \
    X(PFNGLCOMPILESHADERPROC, glCompileShader)                            \
    X(PFNGLGETSHADERIVPROC, glGetShaderiv)                                \
    X(PFNGLGETSHADERINFOLOGPROC, glGetShaderInfoLog)                      \
    X(PFNGLCREATEPROGRAMPROC, glCreateProgram)                            \
    X(PFNGLATTACHSHADERPROC, glAttachShader)                              \
    X(PFNGLLINKPROGRAMPROC, glLinkProgram)                                \
    X(PFNGLGETPROGRAMIVPROC, glGetProgramiv)                              \
    X(PFNGLGETPROGRAMINFOLOGPROC, glGetProgramInfoLog)                    \
    X(PFNGLDELETESHADERPROC, glDeleteShader)                              \
    X(PFNGLDELETEPROGRAMPROC, glDeleteProgram)                            \
    X(PFNGLUSEPROGRAMPROC, glUseProgram)                                  \
    X(PFNGLGETUNIFORMLOCATIONPROC, glGetUniformLocation)                  \
    X(PFNGLUNIFORM1FPROC, glUniform1f)                                    \
    X(PFNGLUNIFORM2IPROC, glUniform2i)                                    \
    X(PFNGLGENTEXTURESPROC, glGenTextures)                                \
    X(PFNGLDELETETEXTURESPROC, glDeleteTextures)                          \
    X(PFNGLBINDTEXTUREPROC, glBindTexture)                                \
    X(PFNGLTEXSTORAGE2DPROC, glTexStorage2D)                              \
    X(PFNGLBINDIMAGETEXTUREPROC, glBindImageTexture)                      \
    X(PFNGLDISPATCHCOMPUTEPROC, glDispatchCompute)                        \
    X(PFNGLMEMORYBARRIERPROC, glMemoryBarrier)                            \
    X(PFNGLFINISHPROC, glFinish)                                          \
    X(PFNGLGETTEXIMAGEPROC, glGetTexImage)                                \
    X(PFNGLGETSTRINGPROC, glGetString)                                    \
    X(PFNGLGETERRORPROC, glGetError)

#define DECL(T, n) static T p_##n;
GLFUNCS(DECL)
#undef DECL

static int g_ready;

static void loader_get_drawable_info(__DRIdrawable *d, int *x, int *y, int *w, int *h, void *p) {
    (void)d; (void)p;
    *x = *y = 0;
    *w = *h = 1;
}
static void loader_put_image(__DRIdrawable *d, int op, int x, int y, int w, int h, char *data, void *p) {
    (void)d; (void)op; (void)x; (void)y; (void)w; (void)h; (void)data; (void)p;
}
static void loader_get_image(__DRIdrawable *d, int x, int y, int w, int h, char *data, void *p) {
    (void)d; (void)x; (void)y; (void)p;
    memset(data, 0, (size_t)w * h * 4);
}

static const __DRIswrastLoaderExtension g_swrast_loader = {
    {__DRI_SWRAST_LOADER, 1}, loader_get_drawable_info, loader_put_image, loader_get_image,
    NULL, NULL, NULL, NULL, NULL, NULL};
static const __DRIextension *g_loader_exts[] = {&g_swrast_loader.base, NULL};

static const __DRIextension *find_ext(const __DRIextension **exts, const char *name) {
    for (int i = 0; exts && exts[i]; i++)
        if (strcmp(exts[i]->name, name) == 0) return exts[i];
    return NULL;
}

/* Create the headless llvmpipe context once per process. */
int glref_init(void) {
    if (g_ready) return 0;
    const char *paths[] = {"/usr/lib/x86_64-linux-gnu/dri/swrast_dri.so", "swrast_dri.so", NULL};
    void *glapi = dlopen("libglapi.so.0", RTLD_NOW | RTLD_GLOBAL);
    if (!glapi) { set_err("dlopen libglapi.so.0: %s", dlerror()); return -1; }
    void *drv = NULL;
    for (int i = 0; paths[i] && !drv; i++) drv = dlopen(paths[i], RTLD_NOW | RTLD_GLOBAL);
    if (!drv) { set_err("dlopen swrast_dri.so: %s", dlerror()); return -1; }
    const __DRIextension **(*get_exts)(void) =
        (const __DRIextension **(*)(void))dlsym(drv, "__driDriverGetExtensions_swrast");
    if (!get_exts) { set_err("no __driDriverGetExtensions_swrast"); return -1; }
    const __DRIextension **drv_exts = get_exts();
    const __DRIcoreExtension *core = (const __DRIcoreExtension *)find_ext(drv_exts, __DRI_CORE);
    const __DRIswrastExtension *sw = (const __DRIswrastExtension *)find_ext(drv_exts, __DRI_SWRAST);
    if (!core || !sw || sw->base.version < 4) { set_err("swrast driver lacks DRI_Core/DRI_SWRast v4"); return -1; }
    const __DRIconfig **configs = NULL;
    __DRIscreen *scr = sw->createNewScreen2(0, g_loader_exts, drv_exts, &configs, NULL);
    if (!scr) { set_err("createNewScreen2 failed"); return -1; }
    uint32_t attribs[] = {__DRI_CTX_ATTRIB_MAJOR_VERSION, 4, __DRI_CTX_ATTRIB_MINOR_VERSION, 3};
    unsigned err = 0;
    __DRIcontext *ctx = sw->createContextAttribs(scr, __DRI_API_OPENGL_CORE, configs ? configs[0] : NULL,
                                                 NULL, 2, attribs, &err, NULL);
    if (!ctx) { set_err("createContextAttribs failed (error %u)", err); return -1; }
    if (!core->bindContext(ctx, NULL, NULL)) { set_err("bindContext (surfaceless) failed"); return -1; }
    void *(*gpa)(const char *) = (void *(*)(const char *))dlsym(glapi, "_glapi_get_proc_address");
    if (!gpa) { set_err("no _glapi_get_proc_address"); return -1; }
#define LOAD(T, n)                                                   \
    p_##n = (T)gpa(#n);                                              \
    if (!p_##n) { set_err("missing GL entry point %s", #n); return -1; }
    GLFUNCS(LOAD)
#undef LOAD
    g_ready = 1;
    return 0;
}

const char *glref_renderer(void) {
    if (glref_init()) return NULL;
    static char buf[512];
    snprintf(buf, sizeof buf, "%s | %s", (const char *)p_glGetString(GL_RENDERER),
             (const char *)p_glGetString(GL_VERSION));
    return buf;
}

/* FNV-1a 64 of the embedded (unpatched) shader, recorded in fixture metadata. */
unsigned long long glref_shader_hash(void) {
    unsigned long long h = 1469598103934665603ULL;
    for (const char *c = _binary_raytrace_compute_glsl_start; c < _binary_raytrace_compute_glsl_end; c++) {
        h ^= (unsigned char)*c;
        h *= 1099511628211ULL;
    }
    return h;
}
long glref_shader_size(void) { return (long)(_binary_raytrace_compute_glsl_end - _binary_raytrace_compute_glsl_start); }

/* ---- string patching ------------------------------------------------- */
typedef struct { char *s; size_t n; } str_t;

static int count_occ(const char *hay, const char *needle) {
    int c = 0;
    size_t nl = strlen(needle);
    for (const char *p = strstr(hay, needle); p; p = strstr(p + nl, needle)) c++;
    return c;
}

/* Replace the unique occurrence of `from` by `to`. */
static int patch(str_t *src, const char *tag, const char *from, const char *to) {
    if (count_occ(src->s, from) != 1) {
        set_err("patch %s: pattern found %d times (want 1): %.60s", tag, count_occ(src->s, from), from);
        return -1;
    }
    char *p = strstr(src->s, from);
    size_t pre = (size_t)(p - src->s), fl = strlen(from), tl = strlen(to);
    size_t n = src->n - fl + tl;
    char *o = (char *)malloc(n + 1);
    memcpy(o, src->s, pre);
    memcpy(o + pre, to, tl);
    memcpy(o + pre + tl, p + fl, src->n - pre - fl + 1);
    free(src->s);
    src->s = o;
    src->n = n;
    return 0;
}

/* Replace the unique span [begin, end-marker-inclusive) by `to`. */
static int patch_span(str_t *src, const char *tag, const char *begin, const char *end, const char *to) {
    if (count_occ(src->s, begin) != 1 || count_occ(src->s, end) != 1) {
        set_err("patch %s: span markers not unique", tag);
        return -1;
    }
    char *b = strstr(src->s, begin), *e = strstr(src->s, end);
    if (e < b) { set_err("patch %s: span end before begin", tag); return -1; }
    e += strlen(end);
    size_t n_old = (size_t)(e - b);
    char *from = (char *)malloc(n_old + 1);
    memcpy(from, b, n_old);
    from[n_old] = 0;
    int r = patch(src, tag, from, to);
    free(from);
    return r;
}

static const char *PROBE_FN =
    "\nvec3 glref_probe(Ray r)\n{\n"
    "  if (GLREF_PROBE == 1) return r.dir;\n"
    "  Collision c = get_closest_collision(r);\n"
    "  if (GLREF_PROBE == 2) {\n"
    "    float mask = 0.0;\n"
    "    if (c.object_index != -1) {\n"
    "      for (int j = 0; j < lights_count; j++) {\n"
    "        Ray lr; lr.start = c.p + c.n * 0.01; lr.dir = lights[j].position - c.p;\n"
    "        Collision cs = get_closest_collision(lr);\n"
    "        if (cs.object_index != -1 && cs.t < 1.0) mask += float(1 << j);\n"
    "      }\n"
    "    }\n"
    "    return vec3(float(c.object_index), c.t, mask);\n"
    "  }\n"
    "  if (c.object_index == -1) return vec3(0.0);\n"
    "  if (GLREF_PROBE == 3) return c.n;\n"
    "  return c.p;\n"
    "}\n";

/* Build the patched source. objects_glsl: NULL = shipped scene. */
static char *build_source(const char *objects_glsl, int max_depth, int crop, int probe) {
    str_t s;
    s.n = (size_t)(_binary_raytrace_compute_glsl_end - _binary_raytrace_compute_glsl_start);
    s.s = (char *)malloc(s.n + 1);
    memcpy(s.s, _binary_raytrace_compute_glsl_start, s.n);
    s.s[s.n] = 0;
    char buf[256];
    /* P1 */
    if (patch(&s, "P1", "uniform image2D output_texture;", "writeonly uniform image2D output_texture;")) goto fail;
    /* P2 */
    if (max_depth != 0) {
        snprintf(buf, sizeof buf, "const int MAX_RAYTRACE_DEPTH = %d;", max_depth);
        if (patch(&s, "P2", "const int MAX_RAYTRACE_DEPTH = 0;", buf)) goto fail;
    }
    /* P3 */
    if (objects_glsl) {
        if (patch_span(&s, "P3", "Object[] objects =", "int objects_count = 5;", objects_glsl)) goto fail;
    }
    /* P5 */
    if (crop) {
        if (patch(&s, "P5a", "uniform float time;",
                  "uniform float time;\nuniform ivec2 glref_size;\nuniform ivec2 glref_offset;")) goto fail;
        if (patch(&s, "P5b", "int width = int(gl_NumWorkGroups.x);", "int width = glref_size.x;")) goto fail;
        if (patch(&s, "P5c", "int height = int(gl_NumWorkGroups.y);", "int height = glref_size.y;")) goto fail;
        if (patch(&s, "P5d", "ivec2 pixel = ivec2(gl_GlobalInvocationID.xy);",
                  "ivec2 pixel = ivec2(gl_GlobalInvocationID.xy) + glref_offset;")) goto fail;
        if (patch(&s, "P5e", "imageStore(output_texture, pixel, vec4(final_color,0.0));",
                  "imageStore(output_texture, ivec2(gl_GlobalInvocationID.xy), vec4(final_color,0.0));")) goto fail;
    }
    /* P4 */
    if (probe) {
        snprintf(buf, sizeof buf,
                 "const int GLREF_PROBE = %d;\nvec3 glref_probe(Ray r);\n"
                 "mat4 calc_transform_matrix(vec3 position, vec3 angles);\nvoid main()", probe);
        if (patch(&s, "P4a", "void main()", buf)) goto fail;
        if (patch(&s, "P4b", "vec3 final_color = recursive_raytrace(world_ray, MAX_RAYTRACE_DEPTH);",
                  "vec3 final_color = glref_probe(world_ray);\n"
                  "\tif (GLREF_PROBE == 5) final_color = vec3(inverse_proj_mat[pixel.x % 4][pixel.y % 4],"
                  " view_mat[pixel.x % 4][pixel.y % 4], proj_mat[pixel.x % 4][pixel.y % 4]);\n"
                  "\tif (GLREF_PROBE == 6) final_color = vec3((proj_mat * view_mat)[pixel.x % 4][pixel.y % 4], 0.0, 0.0);\n"
                  "\tif (GLREF_PROBE == 7) { int k = (pixel.x / 4) % objects_count;"
                  " mat4 lw = calc_transform_matrix(objects[k].position, objects[k].angles);"
                  " mat4 wl = inverse(lw); mat3 nm = transpose(inverse(mat3(lw)));"
                  " final_color = vec3(lw[pixel.x % 4][pixel.y % 4], wl[pixel.x % 4][pixel.y % 4],"
                  " (pixel.x % 4 < 3 && pixel.y % 4 < 3) ? nm[pixel.x % 4][pixel.y % 4] : 0.0); }")) goto fail;
        size_t pl = strlen(PROBE_FN);
        s.s = (char *)realloc(s.s, s.n + pl + 1);
        memcpy(s.s + s.n, PROBE_FN, pl + 1);
        s.n += pl;
    }
    return s.s;
fail:
    free(s.s);
    return NULL;
}

/* Debug helper: return the patched source (caller frees with glref_free). */
char *glref_patched_source(const char *objects_glsl, int max_depth, int crop, int probe) {
    return build_source(objects_glsl, max_depth, crop, probe);
}
void glref_free(void *p) { free(p); }

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int cmp_d(const void *a, const void *b) {
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

/*
 * Render the (patched) reference shader.
 *  frame  width x height (what the shader sees as the image size)
 *  crop   [x0, x0+w) x [y0, y0+h) of that frame; out is w*h RGBA32F, row-major,
 *         row 0 = frame row y0 (GL y=0 is the first row, main.cpp:152-159).
 *  repeats  timed dispatches (after one untimed warm-up that JITs the shader);
 *           times[0..repeats) receive wall seconds per dispatch (+glFinish).
 * Returns 0 or -1 (glref_last_error()).
 */
static int run_program(char *src, float time_s, int width, int height, int crop, int x0, int y0, int w,
                       int h, int repeats, void *out, double *times);
/* output surface: 0 RGBA32F (default), 1 the shipped app's GL_RGBA8
 * (main.cpp:152-159, :223) read back as bytes */
static int g_rgba8 = 0;

int glref_render(const char *objects_glsl, int max_depth, float time_s, int width, int height,
                 int x0, int y0, int w, int h, int probe, int repeats, float *out, double *times) {
    if (glref_init()) return -1;
    if (w <= 0 || h <= 0 || x0 < 0 || y0 < 0 || x0 + w > width || y0 + h > height) {
        set_err("bad crop");
        return -1;
    }
    int crop = !(x0 == 0 && y0 == 0 && w == width && h == height);
    char *src = build_source(objects_glsl, max_depth, crop, probe);
    if (!src) return -1;
    return run_program(src, time_s, width, height, crop, x0, y0, w, h, repeats, out, times);
}

/* The same render into the shipped app's GL_RGBA8 image (glBindImageTexture
 * GL_RGBA8, main.cpp:223): out receives w*h*4 bytes, the driver's float ->
 * unorm8 conversion of imageStore(vec4(final_color, 0.0)) (:404). */
int glref_render_rgba8(const char *objects_glsl, int max_depth, float time_s, int width, int height, int x0, int y0,
                       int w, int h, unsigned char *out) {
    g_rgba8 = 1;
    int rc = glref_render(objects_glsl, max_depth, time_s, width, height, x0, y0, w, h, 0, 0, (float *)(void *)out,
                          NULL);
    g_rgba8 = 0;
    return rc;
}

/* Arithmetic probe: run an arbitrary compute shader (NOT the reference) that
 * writes rgba32f image unit 0 of size w x h, to study llvmpipe's builtins
 * (sin/cos/pow/inverse/normalize) that the reference's results depend on. */
int glref_run_source(const char *source, float time_s, int w, int h, float *out) {
    if (glref_init()) return -1;
    size_t n = strlen(source);
    char *src = (char *)malloc(n + 1);
    memcpy(src, source, n + 1);
    return run_program(src, time_s, w, h, 0, 0, 0, w, h, 0, out, NULL);
}

static int run_program(char *src, float time_s, int width, int height, int crop, int x0, int y0, int w,
                       int h, int repeats, void *out, double *times) {
    GLuint sh = p_glCreateShader(GL_COMPUTE_SHADER);
    const GLchar *srcs[1] = {src};
    p_glShaderSource(sh, 1, srcs, NULL);
    p_glCompileShader(sh);
    free(src);
    GLint ok = 0;
    p_glGetShaderiv(sh, GL_COMPILE_STATUS, &ok);
    if (!ok) {
        char log[2048];
        p_glGetShaderInfoLog(sh, sizeof log, NULL, log);
        set_err("compile failed: %s", log);
        p_glDeleteShader(sh);
        return -1;
    }
    GLuint prog = p_glCreateProgram();
    p_glAttachShader(prog, sh);
    p_glLinkProgram(prog);
    p_glGetProgramiv(prog, GL_LINK_STATUS, &ok);
    p_glDeleteShader(sh);
    if (!ok) {
        char log[2048];
        p_glGetProgramInfoLog(prog, sizeof log, NULL, log);
        set_err("link failed: %s", log);
        p_glDeleteProgram(prog);
        return -1;
    }
    GLuint tex;
    p_glGenTextures(1, &tex);
    p_glBindTexture(GL_TEXTURE_2D, tex);
    p_glTexStorage2D(GL_TEXTURE_2D, 1, g_rgba8 ? GL_RGBA8 : GL_RGBA32F, w, h);
    p_glUseProgram(prog);
    p_glBindImageTexture(0, tex, 0, GL_FALSE, 0, GL_WRITE_ONLY, g_rgba8 ? GL_RGBA8 : GL_RGBA32F);
    p_glUniform1f(p_glGetUniformLocation(prog, "time"), time_s);
    if (crop) {
        p_glUniform2i(p_glGetUniformLocation(prog, "glref_size"), width, height);
        p_glUniform2i(p_glGetUniformLocation(prog, "glref_offset"), x0, y0);
    }
    int rc = 0;
    for (int it = -1; it < repeats; it++) {
        double t0 = now_s();
        p_glDispatchCompute((GLuint)w, (GLuint)h, 1);
        p_glFinish();
        double t1 = now_s();
        if (it >= 0 && times) times[it] = t1 - t0;
    }
    p_glMemoryBarrier(GL_TEXTURE_UPDATE_BARRIER_BIT);
    p_glGetTexImage(GL_TEXTURE_2D, 0, GL_RGBA, g_rgba8 ? GL_UNSIGNED_BYTE : GL_FLOAT, out);
    GLenum e = p_glGetError();
    if (e != GL_NO_ERROR) { set_err("GL error 0x%x", e); rc = -1; }
    p_glDeleteTextures(1, &tex);
    p_glDeleteProgram(prog);
    if (times && repeats > 1) qsort(times, (size_t)repeats, sizeof(double), cmp_d);
    return rc;
}
