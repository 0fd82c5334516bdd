// rt_multi.hip — one frame on several GPUs of this process (SURVEY.md §8(b),
// (e); BASELINE config 4: the frame row-tiled across the GPUs of a node and
// assembled with an RCCL gather over xGMI).
//
// The reference renders a frame with ONE glDispatchCompute(W, H, 1) and
// glFinish (OpenGLRaytracer/main.cpp:228-238). Here the frame's rows are dealt
// in interleaved blocks of `block_rows` rows to the group's GPUs (the
// rt_shard_rows / rt_render_shard layout: cost varies by row, interleaving
// balances it); every GPU renders its blocks densely into a shard buffer on
// its own stream, one gather brings the shards to the first GPU (the root) —
// RCCL point-to-point sends/receives fused in one group, or peer copies —
// and a small HBM-bound kernel on the root de-interleaves the shards into the
// frame. The root renders its own shard straight into the gather buffer.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "rt_internal.h"

namespace rtamd {
namespace {

// Frame row r of the assembled frame comes from shard s = (r / B) % n, row
// (r / (B n)) B + r % B of that shard (rt_shard_rows' dealing). One work-group
// row per frame row; T = uint4 when a row is a multiple of 16 bytes.
template <class T>
__global__ void __launch_bounds__(256) deinterleave(const unsigned char *gather, const size_t *shard_off,
                                                    unsigned char *frame, int row_units, int height, int block_rows,
                                                    int n_shards) {
    const int r = static_cast<int>(blockIdx.y);
    if (r >= height) return;
    const int blk = r / block_rows;
    const int s = blk % n_shards;
    const int local = (blk / n_shards) * block_rows + (r - blk * block_rows);
    const size_t row_bytes = static_cast<size_t>(row_units) * sizeof(T);
    const T *src = reinterpret_cast<const T *>(gather + shard_off[s] + static_cast<size_t>(local) * row_bytes);
    T *dst = reinterpret_cast<T *>(frame + static_cast<size_t>(r) * row_bytes);
    for (int i = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x); i < row_units;
         i += static_cast<int>(gridDim.x) * 256)
        dst[i] = src[i];
}

int nccl_fail(const char *what, ncclResult_t r) {
    set_error(std::string(what) + ": " + ncclGetErrorString(r));
    return RT_ERR_HIP;
}

}  // namespace
}  // namespace rtamd

using namespace rtamd;

struct rt_multi {
    int n = 0;
    int transport = RT_MULTI_RCCL;
    std::vector<rt_context *> ctx;
    std::vector<ncclComm_t> comm;
    std::vector<void *> shard;            // device i's shard buffer (i >= 1)
    std::vector<size_t> shard_cap;
    void *gather = nullptr;               // root: every shard, in shard order
    size_t gather_cap = 0;
    size_t *offsets = nullptr;            // root: byte offset of each shard in `gather` (device copy)
    void *frame = nullptr;                // root: assembled frame for host-destination renders
    size_t frame_cap = 0;
    std::vector<hipEvent_t> rendered;     // device i: its shard is complete
    hipEvent_t g0 = nullptr, g1 = nullptr, a1 = nullptr;  // root: gather start / end, assembly end
    bool timed = false;
};

namespace {

void release(rt_multi *m) {
    if (!m) return;
    for (int i = 0; i < m->n; ++i) {
        if (i < static_cast<int>(m->ctx.size()) && m->ctx[i]) {
            (void)hipSetDevice(m->ctx[i]->device);
            (void)hipStreamSynchronize(m->ctx[i]->stream);
        }
        if (i < static_cast<int>(m->shard.size()) && m->shard[i]) (void)hipFree(m->shard[i]);
        if (i < static_cast<int>(m->rendered.size()) && m->rendered[i]) (void)hipEventDestroy(m->rendered[i]);
    }
    for (ncclComm_t c : m->comm)
        if (c) (void)ncclCommDestroy(c);
    if (m->n > 0 && m->ctx[0]) (void)hipSetDevice(m->ctx[0]->device);
    if (m->gather) (void)hipFree(m->gather);
    if (m->offsets) (void)hipFree(m->offsets);
    if (m->frame) (void)hipFree(m->frame);
    for (hipEvent_t e : {m->g0, m->g1, m->a1})
        if (e) (void)hipEventDestroy(e);
    delete m;
}

// (re)allocate `*buf` on the current device to at least `bytes`
int ensure(void **buf, size_t *cap, size_t bytes, const char *what) {
    if (*cap >= bytes) return RT_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(buf, bytes);
    if (e != hipSuccess) return hip_fail(what, e);
    *cap = bytes;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_multi_create(int n_gpus, rt_context *const *ctxs, int transport, rt_multi **out) {
    if (!out) {
        set_error("rt_multi_create: null out");
        return RT_ERR_INVALID;
    }
    *out = nullptr;
    if (n_gpus <= 0 || !ctxs || (transport != RT_MULTI_RCCL && transport != RT_MULTI_COPY)) {
        set_error("rt_multi_create: need n_gpus >= 1 contexts and a transport (RT_MULTI_RCCL / RT_MULTI_COPY)");
        return RT_ERR_INVALID;
    }
    for (int i = 0; i < n_gpus; ++i) {
        if (!ctxs[i]) {
            set_error("rt_multi_create: context " + std::to_string(i) + " is null");
            return RT_ERR_INVALID;
        }
        for (int j = 0; j < i && transport == RT_MULTI_RCCL; ++j)
            if (ctxs[j]->device == ctxs[i]->device) {
                set_error("rt_multi_create: RCCL needs one context per device (contexts " + std::to_string(j) +
                          " and " + std::to_string(i) + " share device " + std::to_string(ctxs[i]->device) +
                          "); RT_MULTI_COPY serves contexts that share a device");
                return RT_ERR_INVALID;
            }
    }
    rt_multi *m = new (std::nothrow) rt_multi;
    if (!m) {
        set_error("rt_multi_create: out of memory");
        return RT_ERR_NOMEM;
    }
    m->n = n_gpus;
    m->transport = transport;
    m->ctx.assign(ctxs, ctxs + n_gpus);
    m->shard.assign(n_gpus, nullptr);
    m->shard_cap.assign(n_gpus, 0);
    m->rendered.assign(n_gpus, nullptr);
    hipError_t e;
    for (int i = 0; i < n_gpus; ++i) {
        if ((e = hipSetDevice(ctxs[i]->device)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&m->rendered[i], hipEventDisableTiming)) != hipSuccess) {
            release(m);
            return hip_fail("rt_multi_create", e);
        }
    }
    if ((e = hipSetDevice(ctxs[0]->device)) != hipSuccess || (e = hipEventCreate(&m->g0)) != hipSuccess ||
        (e = hipEventCreate(&m->g1)) != hipSuccess || (e = hipEventCreate(&m->a1)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void **>(&m->offsets), sizeof(size_t) * n_gpus)) != hipSuccess) {
        release(m);
        return hip_fail("rt_multi_create", e);
    }
    if (transport == RT_MULTI_RCCL) {
        std::vector<int> devs(n_gpus);
        for (int i = 0; i < n_gpus; ++i) devs[i] = ctxs[i]->device;
        m->comm.assign(n_gpus, nullptr);
        ncclResult_t r = ncclCommInitAll(m->comm.data(), n_gpus, devs.data());
        if (r != ncclSuccess) {
            m->comm.clear();
            release(m);
            return nccl_fail("rt_multi_create: ncclCommInitAll", r);
        }
    }
    *out = m;
    return RT_OK;
}

void rt_multi_destroy(rt_multi *m) { release(m); }

int rt_render_multi_view(rt_multi *m, const rt_scene *const *scenes, const rt_view *view, int width, int height,
                         int max_depth, int block_rows, float *out, int out_is_device) {
    if (!m || !scenes || !view || !out || block_rows <= 0) {
        set_error("rt_render_multi: null group / scenes / view / output, or block_rows < 1");
        return RT_ERR_INVALID;
    }
    const int n = m->n;
    const int fmt = m->ctx[0]->output;
    const size_t bpp = surface_bytes(fmt);
    for (int i = 0; i < n; ++i) {
        int rc = check_render_args(m->ctx[i], scenes[i], width, height, max_depth);
        if (rc != RT_OK) return rc;
        if (m->ctx[i]->output != fmt) {
            set_error("rt_render_multi: every context of the group needs the root's surface format");
            return RT_ERR_INVALID;
        }
    }
    const size_t row_bytes = static_cast<size_t>(width) * bpp;
    std::vector<size_t> off(n + 1, 0);
    std::vector<int> rows(n);
    for (int i = 0; i < n; ++i) {
        rows[i] = rt_shard_rows(height, block_rows, n, i);
        off[i + 1] = off[i] + static_cast<size_t>(rows[i]) * row_bytes;
    }
    rt_context *root = m->ctx[0];
    hipError_t e;
    // buffers: the root's gather buffer (its own shard at offset 0) and the
    // other devices' shard buffers; reused across frames
    if ((e = hipSetDevice(root->device)) != hipSuccess) return hip_fail("hipSetDevice", e);
    int rc = ensure(&m->gather, &m->gather_cap, off[n], "hipMalloc(gather)");
    if (rc != RT_OK) return rc;
    if ((e = hipMemcpyAsync(m->offsets, off.data(), sizeof(size_t) * n, hipMemcpyHostToDevice, root->stream)) !=
        hipSuccess)
        return hip_fail("hipMemcpyAsync(offsets)", e);
    if (!out_is_device && (rc = ensure(&m->frame, &m->frame_cap, static_cast<size_t>(height) * row_bytes,
                                       "hipMalloc(frame)")) != RT_OK)
        return rc;
    // (every scene's origin-sphere lists, before any device starts: a first
    // deep render builds them, rt_internal.h)
    for (int i = 0; i < n; ++i)
        if ((rc = ensure_origin_lists(m->ctx[i], scenes[i], max_depth)) != RT_OK) return rc;
    // every device renders its row blocks on its context's stream
    for (int i = 0; i < n; ++i) {
        rt_context *c = m->ctx[i];
        if ((e = hipSetDevice(c->device)) != hipSuccess) return hip_fail("hipSetDevice", e);
        void *dst = m->gather;
        if (i > 0) {
            if ((rc = ensure(&m->shard[i], &m->shard_cap[i], std::max<size_t>(off[i + 1] - off[i], 16),
                             "hipMalloc(shard)")) != RT_OK)
                return rc;
            dst = m->shard[i];
        }
        if (rows[i] == 0) c->timed = false;  // no kernel of this device in this frame
        if (rows[i] > 0) {
            LaunchParams p = base_params(c, scenes[i], view, 1, width, height);
            p.row_begin = 0;
            p.n_rows = rows[i];
            p.block_rows = block_rows;
            p.n_shards = n;
            p.shard = i;
            p.out = static_cast<float4 *>(dst);
            if ((rc = launch(c, p, max_depth, c->stream)) != RT_OK) return rc;
            if ((rc = note_scene_use(scenes[i], c->stream)) != RT_OK) return rc;
        }
        if ((e = hipEventRecord(m->rendered[i], c->stream)) != hipSuccess) return hip_fail("hipEventRecord", e);
    }
    // gather to the root, timed from the moment every shard is complete
    if ((e = hipSetDevice(root->device)) != hipSuccess) return hip_fail("hipSetDevice", e);
    for (int i = 1; i < n; ++i)
        if ((e = hipStreamWaitEvent(root->stream, m->rendered[i], 0)) != hipSuccess)
            return hip_fail("hipStreamWaitEvent", e);
    if ((e = hipEventRecord(m->g0, root->stream)) != hipSuccess) return hip_fail("hipEventRecord", e);
    if (n > 1 && m->transport == RT_MULTI_RCCL) {
        ncclResult_t r = ncclGroupStart();
        for (int i = 1; i < n && r == ncclSuccess; ++i) {
            const size_t bytes = off[i + 1] - off[i];
            if (!bytes) continue;
            r = ncclSend(m->shard[i], bytes, ncclUint8, 0, m->comm[i], m->ctx[i]->stream);
            if (r == ncclSuccess)
                r = ncclRecv(static_cast<unsigned char *>(m->gather) + off[i], bytes, ncclUint8, i, m->comm[0],
                             root->stream);
        }
        const ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess) return nccl_fail("rt_render_multi: ncclSend/ncclRecv", r);
        if (r2 != ncclSuccess) return nccl_fail("rt_render_multi: ncclGroupEnd", r2);
    } else {
        for (int i = 1; i < n; ++i) {
            const size_t bytes = off[i + 1] - off[i];
            if (!bytes) continue;
            void *dst = static_cast<unsigned char *>(m->gather) + off[i];
            e = m->ctx[i]->device == root->device
                    ? hipMemcpyAsync(dst, m->shard[i], bytes, hipMemcpyDeviceToDevice, root->stream)
                    : hipMemcpyPeerAsync(dst, root->device, m->shard[i], m->ctx[i]->device, bytes, root->stream);
            if (e != hipSuccess) return hip_fail("rt_render_multi: peer copy", e);
        }
    }
    if ((e = hipEventRecord(m->g1, root->stream)) != hipSuccess) return hip_fail("hipEventRecord", e);
    // de-interleave into the frame (the caller's device buffer, or staging)
    unsigned char *frame = static_cast<unsigned char *>(out_is_device ? static_cast<void *>(out) : m->frame);
    const bool wide = row_bytes % 16 == 0;
    const int units = static_cast<int>(row_bytes / (wide ? 16 : 4));
    dim3 grid(std::max(1, std::min((units + 255) / 256, 64)), height);
    if (wide)
        hipLaunchKernelGGL(deinterleave<uint4>, grid, dim3(256), 0, root->stream,
                           static_cast<const unsigned char *>(m->gather), m->offsets, frame, units, height, block_rows, n);
    else
        hipLaunchKernelGGL(deinterleave<uint32_t>, grid, dim3(256), 0, root->stream,
                           static_cast<const unsigned char *>(m->gather), m->offsets, frame, units, height, block_rows, n);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail("rt_render_multi: assembly launch", e);
    if ((e = hipEventRecord(m->a1, root->stream)) != hipSuccess) return hip_fail("hipEventRecord", e);
    if (!out_is_device &&
        (e = hipMemcpyAsync(out, m->frame, static_cast<size_t>(height) * row_bytes, hipMemcpyDeviceToHost,
                            root->stream)) != hipSuccess)
        return hip_fail("hipMemcpyAsync(out)", e);
    // glFinish (main.cpp:238): the frame is complete when the call returns
    if ((e = hipStreamSynchronize(root->stream)) != hipSuccess) return hip_fail("rt_render_multi", e);
    m->timed = true;
    return RT_OK;
}

int rt_render_multi(rt_multi *m, const rt_scene *const *scenes, const rt_camera *cam, float time, int width,
                    int height, int max_depth, int block_rows, float *out, int out_is_device) {
    rt_view view;
    int rc = rt_make_view(cam, time, &view);
    if (rc != RT_OK) return rc;
    return rt_render_multi_view(m, scenes, &view, width, height, max_depth, block_rows, out, out_is_device);
}

int rt_multi_last_ms(rt_multi *m, float *kernel_ms, float *gather_ms, float *assemble_ms) {
    if (!m || !m->timed) {
        set_error("rt_multi_last_ms: nothing rendered yet");
        return RT_ERR_INVALID;
    }
    hipError_t e;
    for (int i = 0; kernel_ms && i < m->n; ++i) {
        kernel_ms[i] = -1.0f;  // the context's timing is off, or the shard was empty
        rt_context *c = m->ctx[i];
        if (!c->timed) continue;
        if ((e = hipSetDevice(c->device)) != hipSuccess) return hip_fail("hipSetDevice", e);
        if ((e = hipEventSynchronize(c->ev1)) != hipSuccess ||
            (e = hipEventElapsedTime(&kernel_ms[i], c->ev0, c->ev1)) != hipSuccess)
            return hip_fail("rt_multi_last_ms", e);
    }
    if ((e = hipSetDevice(m->ctx[0]->device)) != hipSuccess) return hip_fail("hipSetDevice", e);
    if (gather_ms && (e = hipEventElapsedTime(gather_ms, m->g0, m->g1)) != hipSuccess)
        return hip_fail("rt_multi_last_ms", e);
    if (assemble_ms && (e = hipEventElapsedTime(assemble_ms, m->g1, m->a1)) != hipSuccess)
        return hip_fail("rt_multi_last_ms", e);
    return RT_OK;
}

}  // extern "C"
