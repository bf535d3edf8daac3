// ou_program.hip -- native launch list ("program") + hipGraph replay.
//
// The reference drives its sampler from a Python loop (universe.py:334-343)
// that re-enters ATen for every op.  Here the Python host records the whole
// enhance() launch sequence for one (batch, length, options) shape once, as
// an ou_program; replays run natively (no per-op Python), and
// ou_program_capture() turns the list into a single hipGraph so a replay is
// one host call regardless of the ~500 kernels inside.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "../../include/ouhip.h"
#include "ou_common.h"

struct ou_program {
    struct Op {
        int kind;
        std::vector<unsigned char> desc;
    };
    std::vector<Op> ops;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    hipStream_t cap_stream = nullptr;
};

static size_t expected_size(int op)
{
    switch (op) {
    case OU_OP_CONV: return sizeof(ou_conv_desc);
    case OU_OP_GRU: return sizeof(ou_gru_desc);
    case OU_OP_EMBED: return sizeof(ou_embed_desc);
    case OU_OP_HEAD: return sizeof(ou_head_desc);
    case OU_OP_NORMALIZE: return sizeof(ou_norm_args);
    case OU_OP_INV_RMS: return sizeof(ou_rms_args);
    case OU_OP_RMS: return sizeof(ou_rms_args);
    case OU_OP_POWER: return sizeof(ou_power_args);
    case OU_OP_PAD: return sizeof(ou_pad_args);
    case OU_OP_SCALE: return sizeof(ou_scale_args);
    case OU_OP_FINISH: return sizeof(ou_finish_args);
    case OU_OP_SNAKE: return sizeof(ou_snake_desc);
    case OU_OP_MEMSET: return sizeof(ou_memset_desc);
    case OU_OP_ENSEMBLE: return sizeof(ou_ensemble_args);
    }
    return 0;
}

static int run_op(int kind, const void* p, hipStream_t s)
{
    switch (kind) {
    case OU_OP_CONV: return ou_conv((const ou_conv_desc*)p, s);
    case OU_OP_GRU: return ou_gru((const ou_gru_desc*)p, s);
    case OU_OP_EMBED: return ou_embed((const ou_embed_desc*)p, s);
    case OU_OP_HEAD: return ou_head((const ou_head_desc*)p, s);
    case OU_OP_NORMALIZE: {
        auto a = (const ou_norm_args*)p;
        return ou_normalize(a->x, a->y, a->batch, a->n, a->level, a->eps, s);
    }
    case OU_OP_INV_RMS: {
        auto a = (const ou_rms_args*)p;
        return ou_inv_rms(a->x, a->out, a->batch, a->n, a->denom, a->eps, s);
    }
    case OU_OP_RMS: {
        auto a = (const ou_rms_args*)p;
        return ou_rms(a->x, a->out, a->batch, a->n, s);
    }
    case OU_OP_POWER: {
        auto a = (const ou_power_args*)p;
        return ou_power(a->x, a->y, a->batch, a->nf, a->frames, s);
    }
    case OU_OP_PAD: {
        auto a = (const ou_pad_args*)p;
        return ou_pad(a->x, a->x_bstride, a->y, a->batch, a->n_in, a->n_out, a->left, s);
    }
    case OU_OP_SCALE: {
        auto a = (const ou_scale_args*)p;
        return ou_scale(a->z, a->y, a->n, a->scale, a->add, s);
    }
    case OU_OP_FINISH: {
        auto a = (const ou_finish_args*)p;
        return ou_finish(a->x, a->x_bstride, a->left, a->y, a->batch, a->len, a->mix_rms, s);
    }
    case OU_OP_SNAKE: return ou_snake_aa((const ou_snake_desc*)p, s);
    case OU_OP_MEMSET: {
        auto a = (const ou_memset_desc*)p;
        OU_HIP_CHECK(hipMemsetAsync(a->ptr, 0, a->bytes, s), "memset");
        return 0;
    }
    case OU_OP_ENSEMBLE: {
        auto a = (const ou_ensemble_args*)p;
        if (a->mode == 2) {
            if (a->batch <= 0 || a->n % a->batch) return ou_fail(-1, "ensemble: bad batch");
            return ou_signal_median(a->x, a->y, a->ensemble, a->batch, a->n / a->batch, a->counts, s);
        }
        return ou_ensemble_reduce(a->x, a->y, a->ensemble, a->n, a->mode, s);
    }
    }
    return ou_fail(-1, "program: unknown op %d", kind);
}

static void drop_graph(ou_program* p)
{
    if (p->exec) (void)hipGraphExecDestroy(p->exec);
    if (p->graph) (void)hipGraphDestroy(p->graph);
    p->exec = nullptr;
    p->graph = nullptr;
}

extern "C" {

int ou_abi_version(void) { return OUHIP_ABI_VERSION; }
const char* ou_last_error(void) { return ouhip_detail::err_buf(); }

ou_program* ou_program_create(void) { return new ou_program(); }

void ou_program_destroy(ou_program* p)
{
    if (!p) return;
    drop_graph(p);
    if (p->cap_stream) (void)hipStreamDestroy(p->cap_stream);
    delete p;
}

int ou_program_add(ou_program* p, int op, const void* desc, size_t bytes)
{
    if (!p || !desc) return ou_fail(-1, "program_add: null");
    const size_t want = expected_size(op);
    if (want == 0) return ou_fail(-1, "program_add: unknown op %d", op);
    if (bytes != want)
        return ou_fail(-1, "program_add: op %d descriptor is %zu bytes, expected %zu", op, bytes,
                       want);
    ou_program::Op o;
    o.kind = op;
    o.desc.assign((const unsigned char*)desc, (const unsigned char*)desc + bytes);
    p->ops.push_back(std::move(o));
    drop_graph(p);
    return 0;
}

int ou_program_size(const ou_program* p) { return p ? (int)p->ops.size() : -1; }

int ou_program_run(ou_program* p, void* stream)
{
    if (!p) return ou_fail(-1, "program_run: null");
    hipStream_t s = (hipStream_t)stream;
    for (size_t i = 0; i < p->ops.size(); ++i) {
        const int rc = run_op(p->ops[i].kind, p->ops[i].desc.data(), s);
        if (rc) return rc;
    }
    return 0;
}

int ou_program_capture(ou_program* p)
{
    if (!p) return ou_fail(-1, "program_capture: null");
    drop_graph(p);
    if (!p->cap_stream)
        OU_HIP_CHECK(hipStreamCreateWithFlags(&p->cap_stream, hipStreamNonBlocking),
                     "capture stream");
    OU_HIP_CHECK(hipStreamBeginCapture(p->cap_stream, hipStreamCaptureModeThreadLocal),
                 "begin capture");
    int rc = 0;
    for (size_t i = 0; i < p->ops.size() && rc == 0; ++i)
        rc = run_op(p->ops[i].kind, p->ops[i].desc.data(), p->cap_stream);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(p->cap_stream, &g);
    if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (e != hipSuccess) return ou_fail(-100, "end capture: %s", hipGetErrorString(e));
    p->graph = g;
    e = hipGraphInstantiate(&p->exec, g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        drop_graph(p);
        return ou_fail(-100, "graph instantiate: %s", hipGetErrorString(e));
    }
    return 0;
}

int ou_program_launch(ou_program* p, void* stream)
{
    if (!p || !p->exec) return ou_fail(-1, "program_launch: not captured");
    OU_HIP_CHECK(hipGraphLaunch(p->exec, (hipStream_t)stream), "graph launch");
    return 0;
}

int ou_program_op_kind(const ou_program* p, int i)
{
    if (!p || i < 0 || i >= (int)p->ops.size()) return -1;
    return p->ops[i].kind;
}

int ou_program_profile(ou_program* p, void* stream, float* ms)
{
    if (!p || !ms) return ou_fail(-1, "program_profile: null");
    hipStream_t s = (hipStream_t)stream;
    const size_t n = p->ops.size();
    std::vector<hipEvent_t> ev(n + 1);
    for (auto& e : ev) OU_HIP_CHECK(hipEventCreate(&e), "event create");
    int rc = 0;
    (void)hipEventRecord(ev[0], s);
    for (size_t i = 0; i < n && rc == 0; ++i) {
        rc = run_op(p->ops[i].kind, p->ops[i].desc.data(), s);
        (void)hipEventRecord(ev[i + 1], s);
    }
    if (rc == 0) {
        hipError_t e = hipEventSynchronize(ev[n]);
        if (e != hipSuccess) rc = ou_fail(-100, "profile sync: %s", hipGetErrorString(e));
    }
    for (size_t i = 0; i < n && rc == 0; ++i) {
        float t = 0.f;
        (void)hipEventElapsedTime(&t, ev[i], ev[i + 1]);
        ms[i] = t;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    return rc;
}

}  // extern "C"
