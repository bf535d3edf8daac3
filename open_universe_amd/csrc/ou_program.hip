// ou_program.hip -- native launch list ("program") + hipGraph replay.
//
// The reference drives its sampler from a Python loop (universe.py:334-343)
// that re-enters ATen for every op.  Here the Python host records the whole
// enhance() launch sequence for one (batch, length, options) shape once, as
// an ou_program; replays run natively (no per-op Python), and
// ou_program_capture() turns the list into a single hipGraph so a replay is
// one host call regardless of the ~500 kernels inside.
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
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
    // lanes: lane 0 runs on the caller's (or the capture) stream, lane i > 0
    // on a side stream; SIGNAL / WAIT ops order them through events[]
    std::vector<hipEvent_t> events;
    // segmented capture: every maximal run of kernels on one lane between two
    // sync ops is its own hipGraph, launched on the lane's stream; the sync
    // ops stay host-side events between them (real streams, real concurrency)
    struct Seg {
        int lane;
        size_t first, last;   // ops [first, last)
        hipGraphExec_t exec;  // null: a single op, launched directly
    };
    std::vector<Seg> segs;
};

// Streams the programs use besides the caller's: one capture stream and the
// side-lane streams, per device, shared by every program of the process.
// Each HIP stream is bound to one of a few hardware queues (GPU_MAX_HW_QUEUES,
// 4 by default); per-program streams multiplied them until two independent
// callers' streams shared a queue and serialised (enhance_many on two streams:
// 626x instead of 832x real time).  Captures run one at a time (host side),
// so one capture stream suffices.
namespace {
constexpr int kMaxDev = 64, kMaxSide = 8;
constexpr int kMaxEvents = 4096;   // a chunked enhance signals ~10 events per diffusion step
hipStream_t g_cap[kMaxDev];
hipStream_t g_side[kMaxDev][kMaxSide];

int shared_stream(hipStream_t* slot, hipStream_t* out)
{
    if (!*slot) OU_HIP_CHECK(hipStreamCreateWithFlags(slot, hipStreamNonBlocking), "program stream");
    *out = *slot;
    return 0;
}

int side_stream(int dev, int lane, hipStream_t* out)
{
    return shared_stream(&g_side[dev][lane - 1], out);
}

int current_device(int* dev)
{
    OU_HIP_CHECK(hipGetDevice(dev), "program: device");
    if (*dev < 0 || *dev >= kMaxDev) return ou_fail(-1, "program: device %d out of range", *dev);
    return 0;
}
}  // namespace

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
    case OU_OP_BLOCK: return sizeof(ou_block_desc);
    case OU_OP_LANE: case OU_OP_SIGNAL: case OU_OP_WAIT: return sizeof(ou_sync_args);
    }
    return 0;
}

static int run_op(int kind, const void* p, hipStream_t s);

static bool is_sync(int kind) { return kind == OU_OP_LANE || kind == OU_OP_SIGNAL || kind == OU_OP_WAIT; }

// Lane structure check: every lane > 0 starts with a WAIT (it joins the
// caller's stream / the capture through an event recorded on another lane),
// every SIGNAL'd event is recorded before it is waited on, and the program
// ends on lane 0 after waiting for the last SIGNAL of every other lane that
// ran ops (so the caller's stream, and a captured graph, end after all of it).
static int validate_lanes(const ou_program* p, int* n_lanes, int* n_events)
{
    int lane = 0, nl = 1, ne = 0;
    std::vector<int> seen(1, 1), last_sig(1, -1), ops_in(1, 0);
    std::vector<int> recorded, ev_lane;
    for (const auto& o : p->ops) {
        if (!is_sync(o.kind)) {
            ops_in[lane]++;
            continue;
        }
        const int v = ((const ou_sync_args*)o.desc.data())->id;
        if (v < 0 || v >= (o.kind == OU_OP_LANE ? kMaxSide + 1 : kMaxEvents))
            return ou_fail(-1, "program: sync id %d out of range", v);
        if (o.kind == OU_OP_LANE) {
            if (v >= nl) {
                nl = v + 1;
                seen.resize(nl, 0), last_sig.resize(nl, -1), ops_in.resize(nl, 0);
            }
            lane = v;
            continue;
        }
        if ((int)recorded.size() <= v) recorded.resize(v + 1, 0), ev_lane.resize(v + 1, -1);
        ne = std::max(ne, v + 1);
        if (o.kind == OU_OP_SIGNAL) {
            if (lane > 0 && !seen[lane]) return ou_fail(-1, "program: lane %d signals before it waited", lane);
            recorded[v] = 1;
            ev_lane[v] = lane;
            last_sig[lane] = v;
        } else {
            if (!recorded[v]) return ou_fail(-1, "program: wait on event %d before it is signalled", v);
            seen[lane] = 1;
        }
    }
    if (lane != 0) return ou_fail(-1, "program: must end on lane 0");
    for (int l = 1; l < nl; ++l) {
        if (!ops_in[l]) continue;
        if (last_sig[l] < 0) return ou_fail(-1, "program: lane %d never signals lane 0", l);
    }
    // lane 0 must wait on every side lane's final signal after it was recorded
    {
        std::vector<int> done(nl, 0);
        int cur = 0;
        for (const auto& o : p->ops) {
            if (!is_sync(o.kind)) continue;
            const int v = ((const ou_sync_args*)o.desc.data())->id;
            if (o.kind == OU_OP_LANE) cur = v;
            else if (o.kind == OU_OP_WAIT && cur == 0 && ev_lane[v] > 0 && last_sig[ev_lane[v]] == v)
                done[ev_lane[v]] = 1;
        }
        for (int l = 1; l < nl; ++l)
            if (ops_in[l] && !done[l]) return ou_fail(-1, "program: lane 0 never joins lane %d", l);
    }
    *n_lanes = nl;
    *n_events = ne;
    return 0;
}

static int ensure_sync(ou_program* p, int n_lanes, int n_events)
{
    if (n_lanes - 1 > kMaxSide) return ou_fail(-1, "program: %d lanes (max %d)", n_lanes, kMaxSide + 1);
    while ((int)p->events.size() < n_events) {
        hipEvent_t e = nullptr;
        OU_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming), "program event");
        p->events.push_back(e);
    }
    return 0;
}

// Replay the op list with lanes on `s0` (lane 0) and the side streams.
static int run_lanes(ou_program* p, hipStream_t s0)
{
    int nl = 1, ne = 0;
    int rc = validate_lanes(p, &nl, &ne);
    if (rc) return rc;
    rc = ensure_sync(p, nl, ne);
    if (rc) return rc;
    hipStream_t side[kMaxSide] = {};
    if (nl > 1) {
        int dev = 0;
        if ((rc = current_device(&dev))) return rc;
        for (int l = 1; l < nl; ++l)
            if ((rc = side_stream(dev, l, &side[l - 1]))) return rc;
    }
    hipStream_t cur = s0;
    static const bool trace = std::getenv("OUHIP_PROG_TRACE") != nullptr;   // diagnostics
    for (size_t i = 0; i < p->ops.size(); ++i) {
        const auto& o = p->ops[i];
        if (trace) {
            std::fprintf(stderr, "[prog] op %zu kind %d id %d\n", i, o.kind,
                         is_sync(o.kind) ? ((const ou_sync_args*)o.desc.data())->id : -1);
            std::fflush(stderr);
        }
        if (is_sync(o.kind)) {
            const int v = ((const ou_sync_args*)o.desc.data())->id;
            if (o.kind == OU_OP_LANE) cur = v == 0 ? s0 : side[v - 1];
            else if (o.kind == OU_OP_SIGNAL) OU_HIP_CHECK(hipEventRecord(p->events[v], cur), "program signal");
            else OU_HIP_CHECK(hipStreamWaitEvent(cur, p->events[v], 0), "program wait");
            continue;
        }
        rc = run_op(o.kind, o.desc.data(), cur);
        if (rc) return rc;
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
    case OU_OP_BLOCK: return ou_block((const ou_block_desc*)p, s);
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
    for (auto& sg : p->segs)
        if (sg.exec) (void)hipGraphExecDestroy(sg.exec);
    p->segs.clear();
}

extern "C" {

int ou_abi_version(void) { return OUHIP_ABI_VERSION; }
const char* ou_last_error(void) { return ouhip_detail::err_buf(); }

ou_program* ou_program_create(void) { return new ou_program(); }

void ou_program_destroy(ou_program* p)
{
    if (!p) return;
    drop_graph(p);
    for (auto e : p->events) (void)hipEventDestroy(e);
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

int ou_program_patch(ou_program* p, int index, int op, const void* desc, size_t bytes)
{
    if (!p || !desc) return ou_fail(-1, "program_patch: null");
    if (index < 0 || index >= (int)p->ops.size()) return ou_fail(-1, "program_patch: no op %d", index);
    if (p->ops[index].kind != op || bytes != p->ops[index].desc.size())
        return ou_fail(-1, "program_patch: op %d is kind %d (%zu bytes), not %d (%zu bytes)", index,
                       p->ops[index].kind, p->ops[index].desc.size(), op, bytes);
    p->ops[index].desc.assign((const unsigned char*)desc, (const unsigned char*)desc + bytes);
    drop_graph(p);
    return 0;
}

int ou_program_size(const ou_program* p) { return p ? (int)p->ops.size() : -1; }

int ou_program_run(ou_program* p, void* stream)
{
    if (!p) return ou_fail(-1, "program_run: null");
    return run_lanes(p, (hipStream_t)stream);
}

// Side lanes that wait on each other's events (directly or around a cycle
// of side lanes) crash the HIP runtime's stream capture (seen on ROCm 7.2:
// a segfault inside the capture): refuse such a program before capturing.
static int check_side_cycles(const ou_program* p)
{
    constexpr int N = kMaxSide + 1;
    bool edge[N][N] = {};
    std::vector<int> ev_lane;
    int lane = 0;
    for (const auto& o : p->ops) {
        if (!is_sync(o.kind)) continue;
        const int v = ((const ou_sync_args*)o.desc.data())->id;
        if (o.kind == OU_OP_LANE) lane = v;
        else if (o.kind == OU_OP_SIGNAL) {
            if ((int)ev_lane.size() <= v) ev_lane.resize(v + 1, -1);
            ev_lane[v] = lane;
        } else if (v < (int)ev_lane.size() && ev_lane[v] > 0 && lane > 0 && ev_lane[v] != lane)
            edge[lane][ev_lane[v]] = true;   // side lane `lane` waits on side lane ev_lane[v]
    }
    // reachability (Floyd-Warshall over <= 9 lanes)
    for (int k = 1; k < N; ++k)
        for (int i = 1; i < N; ++i)
            for (int j = 1; j < N; ++j)
                if (edge[i][k] && edge[k][j]) edge[i][j] = true;
    for (int i = 1; i < N; ++i)
        if (edge[i][i]) return ou_fail(-1, "program: side lane %d waits on itself through other side lanes "
                                           "(route cross-lane edges through lane 0 for a hipGraph)", i);
    return 0;
}

int ou_program_capture(ou_program* p)
{
    if (!p) return ou_fail(-1, "program_capture: null");
    drop_graph(p);
    int dev = 0, rc0 = current_device(&dev);
    if (rc0) return rc0;
    hipStream_t cap = nullptr;
    if ((rc0 = shared_stream(&g_cap[dev], &cap))) return rc0;
    OU_HIP_CHECK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal),
                 "begin capture");
    int nl = 1, ne = 0;
    int rc = validate_lanes(p, &nl, &ne);
    if (rc == 0) rc = check_side_cycles(p);
    if (rc == 0) rc = ensure_sync(p, nl, ne);
    if (rc) {
        hipGraph_t g0 = nullptr;
        (void)hipStreamEndCapture(cap, &g0);
        if (g0) (void)hipGraphDestroy(g0);
        return rc;
    }
    rc = run_lanes(p, cap);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(cap, &g);
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

int ou_program_validate(const ou_program* p)
{
    if (!p) return ou_fail(-1, "program_validate: null");
    int nl = 1, ne = 0;
    const int rc = validate_lanes(p, &nl, &ne);
    return rc ? rc : check_side_cycles(p);
}

int ou_program_capture_segments(ou_program* p)
{
    if (!p) return ou_fail(-1, "program_capture_segments: null");
    drop_graph(p);
    int nl = 1, ne = 0;
    int rc = validate_lanes(p, &nl, &ne);
    if (rc == 0) rc = ensure_sync(p, nl, ne);
    if (rc) return rc;
    int dev = 0;
    if ((rc = current_device(&dev))) return rc;
    hipStream_t cap = nullptr;
    if ((rc = shared_stream(&g_cap[dev], &cap))) return rc;
    int lane = 0;
    const size_t n = p->ops.size();
    for (size_t i = 0; i < n;) {
        const auto& o = p->ops[i];
        if (is_sync(o.kind)) {
            if (o.kind == OU_OP_LANE) lane = ((const ou_sync_args*)o.desc.data())->id;
            ++i;
            continue;
        }
        size_t j = i;
        while (j < n && !is_sync(p->ops[j].kind)) ++j;
        ou_program::Seg sg{lane, i, j, nullptr};
        if (j - i >= 2) {
            OU_HIP_CHECK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal), "begin capture");
            for (size_t k = i; k < j && rc == 0; ++k) rc = run_op(p->ops[k].kind, p->ops[k].desc.data(), cap);
            hipGraph_t g = nullptr;
            hipError_t e = hipStreamEndCapture(cap, &g);
            if (rc == 0 && e != hipSuccess) rc = ou_fail(-100, "end capture: %s", hipGetErrorString(e));
            if (rc == 0) {
                e = hipGraphInstantiate(&sg.exec, g, nullptr, nullptr, 0);
                if (e != hipSuccess) rc = ou_fail(-100, "graph instantiate: %s", hipGetErrorString(e));
            }
            if (g) (void)hipGraphDestroy(g);
            if (rc) {
                drop_graph(p);
                return rc;
            }
        }
        p->segs.push_back(sg);
        i = j;
    }
    return 0;
}

// Replay a segmented capture: lanes on s0 and the side streams as run_lanes,
// each segment one graph launch.
static int launch_segments(ou_program* p, hipStream_t s0)
{
    int nl = 1, ne = 0, rc = validate_lanes(p, &nl, &ne);
    if (rc) return rc;
    hipStream_t side[kMaxSide] = {};
    if (nl > 1) {
        int dev = 0;
        if ((rc = current_device(&dev))) return rc;
        for (int l = 1; l < nl; ++l)
            if ((rc = side_stream(dev, l, &side[l - 1]))) return rc;
    }
    hipStream_t cur = s0;
    size_t si = 0;
    for (size_t i = 0; i < p->ops.size();) {
        const auto& o = p->ops[i];
        if (is_sync(o.kind)) {
            const int v = ((const ou_sync_args*)o.desc.data())->id;
            if (o.kind == OU_OP_LANE) cur = v == 0 ? s0 : side[v - 1];
            else if (o.kind == OU_OP_SIGNAL) OU_HIP_CHECK(hipEventRecord(p->events[v], cur), "program signal");
            else OU_HIP_CHECK(hipStreamWaitEvent(cur, p->events[v], 0), "program wait");
            ++i;
            continue;
        }
        if (si >= p->segs.size() || p->segs[si].first != i) return ou_fail(-1, "program: segment table out of step");
        const auto& sg = p->segs[si++];
        if (sg.exec) OU_HIP_CHECK(hipGraphLaunch(sg.exec, cur), "segment graph launch");
        else if ((rc = run_op(o.kind, o.desc.data(), cur))) return rc;
        i = sg.last;
    }
    return 0;
}

int ou_program_launch(ou_program* p, void* stream)
{
    if (p && !p->exec && !p->segs.empty()) return launch_segments(p, (hipStream_t)stream);
    if (!p || !p->exec) return ou_fail(-1, "program_launch: not captured");
    OU_HIP_CHECK(hipGraphLaunch(p->exec, (hipStream_t)stream), "graph launch");
    return 0;
}

int ou_program_op_kind(const ou_program* p, int i)
{
    if (!p || i < 0 || i >= (int)p->ops.size()) return -1;
    return p->ops[i].kind;
}

// Eager replay with the lanes on their streams (as ou_program_run) and a
// timing event before and after every op on its lane: t0[i] / t1[i] = ms from
// the replay's start (an event on lane 0 before the first op) to the moment
// op i's stream reached the op / finished it (-1 for sync ops).  Concurrency
// is kept, so the timeline shows the critical path of the lane schedule.
int ou_program_trace(ou_program* p, void* stream, float* t0, float* t1)
{
    if (!p || !t0 || !t1) return ou_fail(-1, "program_trace: null");
    hipStream_t s0 = (hipStream_t)stream;
    int nl = 1, ne = 0;
    int rc = validate_lanes(p, &nl, &ne);
    if (rc) return rc;
    if ((rc = ensure_sync(p, nl, ne))) return rc;
    hipStream_t side[kMaxSide] = {};
    if (nl > 1) {
        int dev = 0;
        if ((rc = current_device(&dev))) return rc;
        for (int l = 1; l < nl; ++l)
            if ((rc = side_stream(dev, l, &side[l - 1]))) return rc;
    }
    const size_t n = p->ops.size();
    // every failure below sets rc and falls through: whatever was enqueued is
    // drained and the timing events destroyed on every path
    std::vector<hipEvent_t> ev(2 * n + 1, nullptr);
    for (auto& e : ev)
        if (rc == 0 && hipEventCreate(&e) != hipSuccess) rc = ou_fail(-100, "program_trace: event create");
    if (rc == 0) (void)hipEventRecord(ev[2 * n], s0);
    hipStream_t cur = s0;
    for (size_t i = 0; i < n && rc == 0; ++i) {
        const auto& o = p->ops[i];
        if (is_sync(o.kind)) {
            const int v = ((const ou_sync_args*)o.desc.data())->id;
            hipError_t e = hipSuccess;
            if (o.kind == OU_OP_LANE) cur = v == 0 ? s0 : side[v - 1];
            else if (o.kind == OU_OP_SIGNAL) e = hipEventRecord(p->events[v], cur);
            else e = hipStreamWaitEvent(cur, p->events[v], 0);
            if (e != hipSuccess) rc = ou_fail(-100, "program_trace: lane sync: %s", hipGetErrorString(e));
            continue;
        }
        (void)hipEventRecord(ev[2 * i], cur);
        rc = run_op(o.kind, o.desc.data(), cur);
        (void)hipEventRecord(ev[2 * i + 1], cur);
    }
    {
        hipError_t e = hipDeviceSynchronize();   // also after a failure: the side lanes may still run
        if (rc == 0 && e != hipSuccess) rc = ou_fail(-100, "trace sync: %s", hipGetErrorString(e));
    }
    for (size_t i = 0; i < n && rc == 0; ++i) {
        float a = -1.f, b = -1.f;
        if (!is_sync(p->ops[i].kind)) {
            (void)hipEventElapsedTime(&a, ev[2 * n], ev[2 * i]);
            (void)hipEventElapsedTime(&b, ev[2 * n], ev[2 * i + 1]);
        }
        t0[i] = a, t1[i] = b;
    }
    for (auto& e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

int ou_program_profile(ou_program* p, void* stream, float* ms)
{
    if (!p || !ms) return ou_fail(-1, "program_profile: null");
    hipStream_t s = (hipStream_t)stream;
    const size_t n = p->ops.size();
    std::vector<hipEvent_t> ev(n + 1, nullptr);
    int rc = 0;
    for (auto& e : ev)
        if (rc == 0 && hipEventCreate(&e) != hipSuccess) rc = ou_fail(-100, "program_profile: event create");
    if (rc == 0) (void)hipEventRecord(ev[0], s);
    // lanes are ignored here: the op list in order is a valid serial schedule
    for (size_t i = 0; i < n && rc == 0; ++i) {
        if (!is_sync(p->ops[i].kind)) rc = run_op(p->ops[i].kind, p->ops[i].desc.data(), s);
        (void)hipEventRecord(ev[i + 1], s);
    }
    {
        hipError_t e = hipStreamSynchronize(s);   // also after a failure
        if (rc == 0 && e != hipSuccess) rc = ou_fail(-100, "profile sync: %s", hipGetErrorString(e));
    }
    for (size_t i = 0; i < n && rc == 0; ++i) {
        float t = 0.f;
        (void)hipEventElapsedTime(&t, ev[i], ev[i + 1]);
        ms[i] = t;
    }
    for (auto& e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

}  // extern "C"
