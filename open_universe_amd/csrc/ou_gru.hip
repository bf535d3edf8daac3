// ou_gru.hip -- bidirectional GRU recurrence for gfx950.
//
// Replaces the recurrent half of torch.nn.GRU(batch_first, bidirectional) in
// ScoreEncoder (networks/universe/score.py:84-90,117-118) and
// ConditionerEncoder (networks/universe/condition.py:173-179,212-215).  The
// input projection gi = W_ih x + b_ih is one dense GEMM over all frames and is
// done beforehand by ou_conv (1x1); this kernel runs the serial part:
//   r = sig(gi_r + W_hr h + b_hr), z = sig(gi_z + W_hz h + b_hz)
//   n = tanh(gi_n + r * (W_hn h + b_hn)),  h' = (1 - z) n + z h      (torch order)
//
// MI355X mapping.  W_hh is 3H x H fp32 = 786 KB per direction for H = 256 --
// more than one CU's register file + LDS (512 KB + 160 KB).  So each direction
// is split over G = H/32 workgroups ("a chain"); a workgroup owns 32 hidden
// units, i.e. 96 rows of W_hh, held in VGPRs for the whole sequence (96 fp32
// per lane at H = 256).  Per time step every workgroup needs the full h_{t-1}:
// it is exchanged through 8-byte {tag = step + 1, value} granules written with
// agent-scope relaxed (sc1) stores and polled with sc1 loads -- the payload is
// its own flag, so no fence is needed (cdna_hip_programming.md Guideline 16,
// recipe R2).  Granules are double-buffered by step parity, which is enough
// because no workgroup can publish step t+2 before every workgroup has read
// step t.  Spins are bounded; on timeout the kernel sets *status and exits.
//
// Lane layout inside a wave: lane = u*8 + kg: u = one of the wave's 8 hidden
// units, kg = which H/8 slice of the dot product the lane owns.  The 3 partial
// dot products are reduced across the 8 kg lanes with xor-shuffles.
#include <hip/hip_runtime.h>

#include "../../include/ouhip.h"
#include "ou_common.h"

namespace {

constexpr int kMaxBatchPerWG = 4;

// workspace after the granules: one XCC-id slot per (item, direction, member)
__host__ __device__ constexpr int64_t xcc_slot_base(int batch, int hidden) { return (int64_t)batch * 4 * hidden; }
__host__ __device__ constexpr int64_t xcc_slot_count(int batch, int hidden) { return (int64_t)batch * hidden / 4; }

// Diagnostic build only (-DOU_GRU_STAMPS, tools/gru_bench.py): thread 0 of
// every workgroup sums s_memtime deltas per phase of the step loop and writes
// them after the granules (5 phases + step count per workgroup).
#ifdef OU_GRU_STAMPS
constexpr int kStampSlots = 8;
#define OU_STAMP_INIT uint64_t st_[5] = {0, 0, 0, 0, 0}; uint64_t tp_ = __builtin_amdgcn_s_memtime();
#define OU_STAMP(i) do { const uint64_t n_ = __builtin_amdgcn_s_memtime(); st_[i] += n_ - tp_; tp_ = n_; } while (0)
#else
constexpr int kStampSlots = 0;
#define OU_STAMP_INIT
#define OU_STAMP(i) do { } while (0)
#endif

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Sum over the 8 consecutive lanes of a group with DPP (no LDS round trip):
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], then row_half_mirror (i <-> 7-i)
// adds the other quad.  Every lane of the group ends with the total.
#define OU_DPP(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, (v)), (ctrl), 0xF, 0xF, true))
__device__ __forceinline__ float sum8(float v)
{
    v += OU_DPP(v, 0xB1);
    v += OU_DPP(v, 0x4E);
    v += OU_DPP(v, 0x141);
    return v;
}

// One "chain" = one (batch group, direction): G = H/U workgroups of 8*U
// threads, each owning U hidden units.  Chains are independent; a workgroup
// of a chain only talks to the other members of the same chain.
//
// Placement (flags & 1): block ids are laid out so that the G members of a
// chain share blockIdx % 8 -- observed to put them on one XCD (one L2), which
// shortens every hand-off.  Speed only: correctness never depends on where
// a block runs (the hand-off is agent-scope sc1 granules).
template <int H, int NB, int U>
__global__ __launch_bounds__(8 * U) void gru_kernel(ou_gru_desc d, int nb, int nchains, int flags)
{
    constexpr int G = H / U;             // workgroups per chain
    constexpr int NT = 8 * U;            // threads
    constexpr int KPL = H / 8;           // k-slice per lane
    constexpr int SEG = KPL + 4;         // padded LDS segment (bank spread)
    __shared__ __attribute__((aligned(16))) float hs[NB][8 * SEG];
    __shared__ int abort_flag;

    const int bid = blockIdx.x;
    int chain, member;
    if (flags & 1) {   // bits 12-14: chain c on blockIdx % 8 == (c + offset) % 8
        const int c8 = bid & 7, rest = bid >> 3;
        member = rest % G;
        chain = (rest / G) * 8 + ((c8 - (flags >> 12)) & 7);
    } else {
        chain = bid / G;
        member = bid % G;
    }
    if (chain >= nchains) return;        // padding block of the XCD layout
    const int dir = chain & 1;
    const int b0 = (chain >> 1) * nb;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int kg = lane & 7;
    const int u = lane >> 3;
    const int j = member * U + wave * 8 + u;   // hidden unit
    const int nbh = min(nb, d.batch - b0);
    const int T = d.steps;
    const bool sleep_poll = !(flags & 2);
    const bool nowait = flags & 16;      // timing diagnostic only: results are wrong
    if (tid == 0) abort_flag = 0;

    // W_hh rows of this unit (gates r, z, n), k-slice of this lane, in VGPRs
    const float* wbase = d.w_hh + (int64_t)dir * 3 * H * H;
    float wr[KPL], wz[KPL], wn[KPL];
#pragma unroll
    for (int k = 0; k < KPL; k += 4) {
        const float4 a = *(const float4*)(wbase + (int64_t)(0 * H + j) * H + kg * KPL + k);
        const float4 bq = *(const float4*)(wbase + (int64_t)(1 * H + j) * H + kg * KPL + k);
        const float4 c = *(const float4*)(wbase + (int64_t)(2 * H + j) * H + kg * KPL + k);
        wr[k] = a.x; wr[k + 1] = a.y; wr[k + 2] = a.z; wr[k + 3] = a.w;
        wz[k] = bq.x; wz[k + 1] = bq.y; wz[k + 2] = bq.z; wz[k + 3] = bq.w;
        wn[k] = c.x; wn[k + 1] = c.y; wn[k + 2] = c.z; wn[k + 3] = c.w;
    }
    const float bhr = d.b_hh[dir * 3 * H + 0 * H + j];
    const float bhz = d.b_hh[dir * 3 * H + 1 * H + j];
    const float bhn = d.b_hh[dir * 3 * H + 2 * H + j];

    uint64_t* gran = d.granules;   // [B][2 dir][2 parity][H]
    auto gidx = [&](int b, int par, int k) -> int64_t {
        return (((int64_t)b * 2 + dir) * 2 + par) * H + k;
    };

    // per-step operands of this lane's unit: gi (3 gates) and the optional
    // output residual, prefetched one step ahead (issued right after the
    // gather barrier, so they are never queued in front of the next poll)
    float gir[NB], giz[NB], gin[NB], rsd[NB];
    auto prefetch = [&](int step, float* pr, float* pz, float* pn, float* pres) {
        const int tm = dir == 0 ? step : T - 1 - step;
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            if (bb < nbh && kg == 0) {
                const float* g = d.gi + (int64_t)(b0 + bb) * d.gi_bstride +
                                 (int64_t)(dir * 3 * H) * T + tm;
                pr[bb] = g[(int64_t)(0 * H + j) * T];
                pz[bb] = g[(int64_t)(1 * H + j) * T];
                pn[bb] = g[(int64_t)(2 * H + j) * T];
                pres[bb] = d.res ? d.res[(int64_t)(b0 + bb) * d.res_bstride +
                                         (int64_t)(dir * H + j) * d.res_cstride + tm]
                                 : 0.f;
            }
        }
    };
    prefetch(0, gir, giz, gin, rsd);
    OU_STAMP_INIT

    for (int t = 0; t < T; ++t) {
        const int time = dir == 0 ? t : T - 1 - t;
        // gather h_{t-1}
        if (t == 0) {
            for (int i = tid; i < nbh * H; i += NT) {
                const int bb = i / H, k = i - bb * H;
                hs[bb][(k / KPL) * SEG + (k % KPL)] = 0.f;
            }
        } else {
            // all of this thread's granules are requested at once; only the
            // stale ones are re-polled (one L2 round trip per pass, not per granule)
            const uint32_t want = (uint32_t)t;   // tag of h_{t-1}
            const int par = (t - 1) & 1;
            constexpr int NPER = (NB * H + NT - 1) / NT;
            uint64_t v[NPER];
            uint64_t* pp[NPER];
#pragma unroll
            for (int e = 0; e < NPER; ++e) {
                const int i = tid + e * NT;
                const int bb = i / H, k = i - bb * H;
                pp[e] = gran + gidx(b0 + min(bb, nbh - 1), par, k);
                v[e] = (i < nbh * H) ? __hip_atomic_load(pp[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : ((uint64_t)want << 32);
            }
            uint32_t spins = 0;
            while (true) {
                bool ok = true;
                if (nowait) break;
#pragma unroll
                for (int e = 0; e < NPER; ++e) ok &= (uint32_t)(v[e] >> 32) == want;
                if (ok) break;
                if (sleep_poll) __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 23)) {   // ~seconds: the chain is dead
                    atomicExch(d.status, 1);
                    abort_flag = 1;
                    break;
                }
#pragma unroll
                for (int e = 0; e < NPER; ++e)
                    if ((uint32_t)(v[e] >> 32) != want)
                        v[e] = __hip_atomic_load(pp[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            OU_STAMP(0);
#pragma unroll
            for (int e = 0; e < NPER; ++e) {
                const int i = tid + e * NT;
                if (i < nbh * H) {
                    const int bb = i / H, k = i - bb * H;
                    hs[bb][(k / KPL) * SEG + (k % KPL)] = __uint_as_float((uint32_t)v[e]);
                }
            }
        }
        __syncthreads();
        if (abort_flag) return;   // uniform across the workgroup
        OU_STAMP(1);

        float cr[NB], cz[NB], cn[NB], cres[NB];
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            cr[bb] = gir[bb]; cz[bb] = giz[bb]; cn[bb] = gin[bb]; cres[bb] = rsd[bb];
        }
        if (t + 1 < T) prefetch(t + 1, gir, giz, gin, rsd);

#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            if (bb >= nbh) break;
            const float* hv = &hs[bb][kg * SEG];
            float sr = 0.f, sz = 0.f, sn = 0.f;
#pragma unroll
            for (int k = 0; k < KPL; k += 4) {
                const float4 hq = *(const float4*)(hv + k);
                sr = fmaf(wr[k], hq.x, sr); sz = fmaf(wz[k], hq.x, sz); sn = fmaf(wn[k], hq.x, sn);
                sr = fmaf(wr[k + 1], hq.y, sr); sz = fmaf(wz[k + 1], hq.y, sz); sn = fmaf(wn[k + 1], hq.y, sn);
                sr = fmaf(wr[k + 2], hq.z, sr); sz = fmaf(wz[k + 2], hq.z, sz); sn = fmaf(wn[k + 2], hq.z, sn);
                sr = fmaf(wr[k + 3], hq.w, sr); sz = fmaf(wz[k + 3], hq.w, sz); sn = fmaf(wn[k + 3], hq.w, sn);
            }
            sr = sum8(sr);
            sz = sum8(sz);
            sn = sum8(sn);
            OU_STAMP(2);
            if (kg == 0) {
                const float hprev = hs[bb][(j / KPL) * SEG + (j % KPL)];
                const float r = sigmoidf_(cr[bb] + (sr + bhr));
                const float z = sigmoidf_(cz[bb] + (sz + bhz));
                const float n = tanhf(cn[bb] + r * (sn + bhn));
                const float hn = (1.0f - z) * n + z * hprev;
                const int b = b0 + bb;
                if (t + 1 < T) {
                    const uint64_t g = ((uint64_t)(uint32_t)(t + 1) << 32) | __float_as_uint(hn);
                    __hip_atomic_store(gran + gidx(b, t & 1, j), g, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
                const int64_t c = (int64_t)(dir * H + j);
                const float out = d.res ? (hn + cres[bb]) * d.res_scale : hn;
                d.y[(int64_t)b * d.y_bstride + c * d.y_cstride + time] = out;
            }
        }
        OU_STAMP(3);
        __syncthreads();
        OU_STAMP(4);
    }
#ifdef OU_GRU_STAMPS
    if (tid == 0) {
        uint64_t* o = gran + xcc_slot_base(d.batch, H) + xcc_slot_count(d.batch, H) + (int64_t)bid * kStampSlots;
        for (int i = 0; i < 5; ++i) o[i] = st_[i];
        o[5] = T;
    }
#endif
}


// ---------------------------------------------------------------------------
// k-split recurrence (default for H % 64 == 0).
//
// Lane L of a wave owns the k-slice [L*KPL, (L+1)*KPL) of h (KPL = H/64) for
// ALL 8 hidden units of its wave: W_hh[g*H + j][k-slice] for 8 units x 3
// gates sits in 24*KPL VGPRs.  Every wave is self-contained: it polls the
// granules of its own k-slice (16-byte sc1 loads, two granules each), so
// there is no LDS staging and no workgroup barrier in the step loop.  The 24
// per-lane partial sums are reduced with a reduce-scatter -- permlane32_swap,
// permlane16_swap, DPP row_ror:8 (each halves the values a lane carries),
// then an 8-lane DPP sum -- which leaves lane L with the r/z/n sums of unit
// L >> 3 (replicated on 8 lanes).  Each lane keeps its unit's h_{t-1} in a
// register; one lane per unit publishes h_t.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float fast_sigmoid(float x)
{
    // 1 / (1 + 2^(-x log2 e)): v_exp_f32 + v_rcp_f32 (~1 ulp each)
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}
__device__ __forceinline__ float fast_tanh(float x)
{
    // 2 sigmoid(2x) - 1: absolute error ~1e-7 around 0, relative ~1e-7 elsewhere
    return fmaf(2.0f, fast_sigmoid(2.0f * x), -1.0f);
}

__device__ __forceinline__ void swap32(float& x, float& y)
{
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]);
    y = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& x, float& y)
{
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]);
    y = __uint_as_float(r[1]);
}

constexpr int kKsWaves = 4;   // waves per workgroup


template <int H, int NB, int UW>
__global__ __launch_bounds__(64 * kKsWaves) void gru_ks_kernel(ou_gru_desc d, int nb, int nchains, int flags,
                                                               int bofs)
{
    constexpr int KPL = H / 64;
    constexpr int G = H / (UW * kKsWaves);   // workgroups per chain
    constexpr int NV = UW * 3 * NB;          // partial sums per lane
    constexpr int NG = 3 * NB;               // sums left per lane after the scatter
    constexpr int USH = UW == 8 ? 3 : 4;     // unit of lane L = L >> USH
    static_assert(H % 64 == 0 && G >= 1 && (UW == 4 || UW == 8), "k-split GRU: H % 64 == 0, UW 4 or 8");

    const int bid = blockIdx.x;
    int chain, member;
    if (flags & 1) {   // bits 12-14: chain c on blockIdx % 8 == (c + offset) % 8
        const int c8 = bid & 7, rest = bid >> 3;
        member = rest % G;
        chain = (rest / G) * 8 + ((c8 - (flags >> 12)) & 7);
    } else {
        chain = bid / G;
        member = bid % G;
    }
    if (chain >= nchains) return;            // padding block of the XCD layout
    const int dir = chain & 1;
    const int b0 = bofs + (chain >> 1) * nb;
    const int nbh = min(nb, d.batch - b0);
    const int T = d.steps;
    const bool sleep_poll = !(flags & 2);

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int ubase = (member * kKsWaves + wave) * UW;
    const int j = ubase + (lane >> USH);     // unit whose gates this lane computes
    const bool writer = (lane & ((1 << USH) - 1)) == 0;

    float w[UW][3][KPL];
    const float* wbase = d.w_hh + (int64_t)dir * 3 * H * H + lane * KPL;
#pragma unroll
    for (int u = 0; u < UW; ++u)
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
            for (int k = 0; k < KPL; ++k) w[u][g][k] = wbase[(int64_t)(g * H + ubase + u) * H + k];
    const float bhr = d.b_hh[dir * 3 * H + 0 * H + j];
    const float bhz = d.b_hh[dir * 3 * H + 1 * H + j];
    const float bhn = d.b_hh[dir * 3 * H + 2 * H + j];

    // granules [B][2 dir][2 parity][H]; this lane reads KPL consecutive ones
    uint64_t* gran = d.granules;

    // Same-XCD fast path.  Consumers always load granules sc1 (served by the
    // L2, never by a stale L1).  A producer normally stores sc1 (write-
    // through, which drops the line from its L2, so every consumer load goes
    // out to the Infinity Cache).  When every workgroup of this chain runs on
    // one XCD -- checked here at run time, never assumed -- the chain shares
    // one L2 and a plain store (kept in that L2) is visible to the sc1 loads.
    // Either way every granule is tag-checked.
    bool local_l2 = false;
    if (!(flags & 64)) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        uint64_t* xs = gran + xcc_slot_base(d.batch, H) + ((int64_t)b0 * 2 + dir) * G;
        if (threadIdx.x == 0)
            __hip_atomic_store(xs + member, (1ull << 32) | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t v = 0;
        for (uint32_t spins = 0;; ++spins) {
            v = lane < G ? __hip_atomic_load(xs + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : ((1ull << 32) | xcc);
            if (__all((uint32_t)(v >> 32) == 1u)) break;
            if (spins > (1u << 23)) {
                if (lane == 0) atomicExch(d.status, 1);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        local_l2 = __all((uint32_t)v == xcc);
    }
    const int64_t gran_bytes = (int64_t)d.batch * 2 * 2 * H * 8;
    const __amdgpu_buffer_rsrc_t grsrc =
        ou_rsrc(gran, gran_bytes);
    auto goff = [&](int b, int par) -> int {   // byte offset of this lane's slice
        return (int)(((((int64_t)b * 2 + dir) * 2 + par) * H + lane * KPL) * 8);
    };

    // steps [tb, te) of this launch (the recurrence may be split over
    // launches: h of the step before tb comes from d.hstate)
    const int tb = d.t_begin, te = d.t_end > 0 ? min(d.t_end, T) : T;
    float hp[NB];                            // h_{t-1} of unit j
    float gir[NB], giz[NB], gin[NB], rsd[NB];
    auto prefetch = [&](int step) {
        const int tm = dir == 0 ? step : T - 1 - step;
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            if (bb < nbh) {
                const float* g = d.gi + (int64_t)(b0 + bb) * d.gi_bstride + (int64_t)(dir * 3 * H) * T + tm;
                gir[bb] = g[(int64_t)(0 * H + j) * T];
                giz[bb] = g[(int64_t)(1 * H + j) * T];
                gin[bb] = g[(int64_t)(2 * H + j) * T];
                rsd[bb] = d.res ? d.res[(int64_t)(b0 + bb) * d.res_bstride +
                                        (int64_t)(dir * H + j) * d.res_cstride + tm]
                                : 0.f;
            }
        }
    };
    // One item per chain (NB == 1, the batch-1 case): gi and the residual of
    // the wave's UW units are staged through LDS in chunks of CS steps
    // instead of prefetched one step ahead.  Vector loads retire in order, so
    // the poll loop's vmcnt wait also waited for the previous step's gi
    // prefetch (~0.07 us of a 0.8 us step, measured with a build that skipped
    // the gi loads);
    // a chunk load pays that latency once per CS steps.  Per wave and chunk
    // the 4 UW rows (3 gates x UW units of gi, UW residual rows) x CS steps
    // are loaded coalesced along time and written as [step][unit][r z n res],
    // so a step reads its four values with one ds_read_b128 issued before
    // the hand-off wait.  flags bit8 keeps the per-step prefetch (A/B runs).
    constexpr int CS = UW == 4 ? 128 : 64;   // steps per chunk (4 UW x CS x 4 B = 8 KB per wave)
    const bool stage = NB == 1 && !(flags & 256);
    float4* gst = nullptr;
    if constexpr (NB == 1) {
        __shared__ float4 gst_all[kKsWaves][CS * UW];
        gst = gst_all[wave];
    }
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    auto stage_chunk = [&](int c0) {   // steps [c0, c0 + CS) (clamped to te - 1) -> LDS
        constexpr int NV4 = 4 * UW * CS / 64;   // values per lane
        const int ub = (member * kKsWaves + wv) * UW;
        float v[NV4];
#pragma unroll
        for (int i = 0; i < NV4; ++i) {
            const int e = lane + 64 * i, row = e / CS, st = min(c0 + e % CS, te - 1);
            const int tm = dir == 0 ? st : T - 1 - st;
            if (row < 3 * UW) {
                const int g = row / UW, u = row % UW;
                v[i] = d.gi[(int64_t)b0 * d.gi_bstride + (int64_t)(dir * 3 * H + g * H + ub + u) * T + tm];
            } else {
                const int u = row - 3 * UW;
                v[i] = d.res ? d.res[(int64_t)b0 * d.res_bstride + (int64_t)(dir * H + ub + u) * d.res_cstride + tm]
                             : 0.f;
            }
        }
#pragma unroll
        for (int i = 0; i < NV4; ++i) {
            const int e = lane + 64 * i, row = e / CS, sc = e % CS;
            const int comp = row < 3 * UW ? row / UW : 3, u = row < 3 * UW ? row % UW : row - 3 * UW;
            ((float*)gst)[(sc * UW + u) * 4 + comp] = v[i];
        }
    };
    auto hs_at = [&](int b, int u) -> float {   // h of unit u before step tb (written by the previous launch)
        return tb > 0 ? d.hstate[((int64_t)b * 2 + dir) * H + u] : 0.f;
    };
    // h before step tb, loaded ahead of the loop: a load inside the loop's
    // first-step branch made the compiler drain every outstanding load at the
    // branch join (the gi prefetch included): 0.73 -> 1.0 us per step
    float h0[NB][KPL];
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        hp[bb] = hs_at(b0 + min(bb, nbh - 1), j);
#pragma unroll
        for (int k = 0; k < KPL; ++k) h0[bb][k] = hs_at(b0 + min(bb, nbh - 1), lane * KPL + k);
    }
    if (stage) stage_chunk(tb);
    else prefetch(tb);
    OU_STAMP_INIT

    for (int t = tb; t < te; ++t) {
        const int time = dir == 0 ? t : T - 1 - t;
        float h[NB][KPL];
        // this step's staged gi / residual (LDS read in flight during the wait)
        float4 gv{};
        if (stage) {
            if (t > tb && (t - tb) % CS == 0) stage_chunk(t);
            gv = gst[((t - tb) % CS) * UW + (lane >> USH)];
        }
        if (t == tb) {
#pragma unroll
            for (int bb = 0; bb < NB; ++bb)
#pragma unroll
                for (int k = 0; k < KPL; ++k) h[bb][k] = h0[bb][k];
        } else {
            const uint32_t want = (uint32_t)t;   // tag of h_{t-1}
            const int par = (t - 1) & 1;
            for (uint32_t spins = 0;; ++spins) {
                bool ok = true;
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) {
                    const int b = b0 + min(bb, nbh - 1);
                    if constexpr (KPL % 2 == 0) {
#pragma unroll
                        for (int q = 0; q < KPL / 2; ++q) {
                            // aux 16 = sc1: served by L2, never by this CU's L1
                            const auto v = __builtin_amdgcn_raw_buffer_load_b128(grsrc, goff(b, par) + 16 * q, 0, 16);
                            h[bb][2 * q] = __uint_as_float(v[0]);
                            h[bb][2 * q + 1] = __uint_as_float(v[2]);
                            ok &= bb >= nbh || (v[1] == want && v[3] == want);
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < KPL; ++k) {
                            const uint64_t v = __hip_atomic_load(
                                gran + ((((int64_t)b * 2 + dir) * 2 + par) * H + lane * KPL + k),
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            h[bb][k] = __uint_as_float((uint32_t)v);
                            ok &= bb >= nbh || (uint32_t)(v >> 32) == want;
                        }
                    }
                }
                if (__all(ok)) break;
                if (sleep_poll) __builtin_amdgcn_s_sleep(1);
                if (spins > (1u << 23)) {        // ~seconds: the chain is dead
                    if (lane == 0) atomicExch(d.status, 1);
                    return;
                }
                asm volatile("" ::: "memory");   // re-load every pass
            }
        }
        OU_STAMP(0);

        float cr[NB], cz[NB], cn[NB], cres[NB];
        if (stage) {
            cr[0] = gv.x, cz[0] = gv.y, cn[0] = gv.z, cres[0] = gv.w;
        } else {
#pragma unroll
            for (int bb = 0; bb < NB; ++bb) {
                cr[bb] = gir[bb]; cz[bb] = giz[bb]; cn[bb] = gin[bb]; cres[bb] = rsd[bb];
            }
            if (t + 1 < te) prefetch(t + 1);
        }

        // partial dot products, value index (u * NB + b) * 3 + g
        float acc[NV];
#pragma unroll
        for (int u = 0; u < UW; ++u)
#pragma unroll
            for (int bb = 0; bb < NB; ++bb)
#pragma unroll
                for (int g = 0; g < 3; ++g) {
                    float a = 0.f;
#pragma unroll
                    for (int k = 0; k < KPL; ++k) a = fmaf(w[u][g][k], h[bb][k], a);
                    acc[(u * NB + bb) * 3 + g] = a;
                }
        OU_STAMP(1);

        // reduce-scatter over the 64 lanes: the top unit bit <-> lane bit 5,
        // the next <-> lane bit 4 (and for UW = 8 the last <-> lane bit 3);
        // then sum over the 2^USH lanes left
#pragma unroll
        for (int i = 0; i < NV / 2; ++i) {
            swap32(acc[i], acc[i + NV / 2]);
            acc[i] += acc[i + NV / 2];
        }
#pragma unroll
        for (int i = 0; i < NV / 4; ++i) {
            swap16(acc[i], acc[i + NV / 4]);
            acc[i] += acc[i + NV / 4];
        }
        if constexpr (UW == 8) {
            const bool hi8 = lane & 8;
#pragma unroll
            for (int i = 0; i < NG; ++i) {
                const float send = hi8 ? acc[i] : acc[i + NG];
                const float keep = hi8 ? acc[i + NG] : acc[i];
                acc[i] = keep + OU_DPP(send, 0x128);   // row_ror:8 == lane ^ 8
            }
        } else {
#pragma unroll
            for (int i = 0; i < NG; ++i) acc[i] += OU_DPP(acc[i], 0x128);
        }
#pragma unroll
        for (int i = 0; i < NG; ++i) acc[i] = sum8(acc[i]);
        OU_STAMP(2);

#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            if (bb >= nbh) break;
            const float r = fast_sigmoid(cr[bb] + (acc[bb * 3 + 0] + bhr));
            const float z = fast_sigmoid(cz[bb] + (acc[bb * 3 + 1] + bhz));
            const float n = fast_tanh(cn[bb] + r * (acc[bb * 3 + 2] + bhn));
            const float hn = (1.0f - z) * n + z * hp[bb];
            hp[bb] = hn;
            if (writer) {
                const int b = b0 + bb;
                if (t + 1 < T) {
                    const uint64_t gv = ((uint64_t)(uint32_t)(t + 1) << 32) | __float_as_uint(hn);
                    uint64_t* gp = gran + ((((int64_t)b * 2 + dir) * 2 + (t & 1)) * H + j);
                    if (local_l2)   // plain 8-byte store: stays in the shared L2
                        __hip_atomic_store(gp, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    else            // sc1 write-through
                        __hip_atomic_store(gp, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                const float out = d.res ? (hn + cres[bb]) * d.res_scale : hn;
                d.y[(int64_t)b * d.y_bstride + (int64_t)(dir * H + j) * d.y_cstride + time] = out;
            }
        }
        OU_STAMP(3);
    }
    // h of the last step, for a launch that continues the recurrence
    if (d.hstate && writer) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb)
            if (bb < nbh) d.hstate[((int64_t)(b0 + bb) * 2 + dir) * H + j] = hp[bb];
    }
    // leave the placement slot zeroed for the next launch on this workspace:
    // every member of the chain has passed the placement handshake by now
    // (none can finish step 1 before all have published step 0)
    if (!(flags & 64) && threadIdx.x == 0)
        __hip_atomic_store(gran + xcc_slot_base(d.batch, H) + ((int64_t)b0 * 2 + dir) * G + member, (uint64_t)0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef OU_GRU_STAMPS
    if (lane == 0 && wave == 0) {
        uint64_t* o = gran + xcc_slot_base(d.batch, H) + xcc_slot_count(d.batch, H) + (int64_t)bid * kStampSlots;
        for (int i = 0; i < 4; ++i) o[i] = st_[i];
        o[4] = local_l2;
        o[5] = T;
    }
#endif
}

template <int H, int NB, int UW>
void launch_ks(const ou_gru_desc& d, int nb, int nchains, int flags, int bofs, hipStream_t s)
{
    constexpr int G = H / (UW * kKsWaves);
    const int grid = (flags & 1) ? 8 * G * ((nchains + 7) / 8) : nchains * G;
    hipLaunchKernelGGL((gru_ks_kernel<H, NB, UW>), dim3(grid), dim3(64 * kKsWaves), 0, s, d, nb, nchains, flags,
                       bofs);
}

// items per launch of the k-split kernel: every workgroup of every chain must
// be resident at once (one 256-thread workgroup per CU is always possible)
constexpr int kKsMaxWGs = 256;

template <int H, int UW>
int launch_ks_uw(const ou_gru_desc& d, int flags, hipStream_t s)
{
    constexpr int G = H / (UW * kKsWaves);
    constexpr int kMaxNb = H >= 512 ? 2 : 4;   // 4 items at H = 512 would spill
    // one item per chain while the chip has room, else 2 or 4
    int nb = 1;
    while (nb < kMaxNb && 2 * ((d.batch + nb - 1) / nb) * G > kKsMaxWGs) nb *= 2;
    const int per_launch = (kKsMaxWGs / (2 * G)) * nb;
    for (int b = 0; b < d.batch; b += per_launch) {
        const int items = min(per_launch, d.batch - b);
        const int nchains = 2 * ((items + nb - 1) / nb);
        if (nb == 1) launch_ks<H, 1, UW>(d, nb, nchains, flags, b, s);
        else if (nb == 2 || kMaxNb == 2) launch_ks<H, 2, UW>(d, nb, nchains, flags, b, s);
        else launch_ks<H, kMaxNb, UW>(d, nb, nchains, flags, b, s);
    }
    return 0;
}

template <int H>
int launch_ks_all(const ou_gru_desc& d, int flags, hipStream_t s)
{
    // 4 units per wave (half the per-wave dot product, twice the CUs) while
    // one item per chain fits; 8 units per wave otherwise (or flags bit7)
    constexpr int G4 = H / (4 * kKsWaves);
    if (!(flags & 128) && 2 * d.batch * G4 <= kKsMaxWGs) return launch_ks_uw<H, 4>(d, flags, s);
    return launch_ks_uw<H, 8>(d, flags, s);
}

template <int H, int NB, int U>
void launch_u(const ou_gru_desc& d, int nb, int nchains, int flags, hipStream_t s)
{
    constexpr int G = H / U;
    const int grid = (flags & 1) ? 8 * G * ((nchains + 7) / 8) : nchains * G;
    hipLaunchKernelGGL((gru_kernel<H, NB, U>), dim3(grid), dim3(8 * U), 0, s, d, nb, nchains, flags);
}

template <int H, int NB>
void launch_nb(const ou_gru_desc& d, int nb, int nchains, int flags, hipStream_t s)
{
    if ((flags & 8) && H >= 128 && H % 128 == 0)
        launch_u<H, NB, (H >= 128 ? 128 : 32)>(d, nb, nchains, flags, s);
    else if ((flags & 4) && H >= 64 && H % 64 == 0)
        launch_u<H, NB, (H >= 64 ? 64 : 32)>(d, nb, nchains, flags, s);
    else
        launch_u<H, NB, 32>(d, nb, nchains, flags, s);
}

template <int H>
void launch_h(const ou_gru_desc& d, int nb, int nchains, int flags, hipStream_t s)
{
    if (nb == 1) launch_nb<H, 1>(d, nb, nchains, flags, s);
    else if (nb == 2) launch_nb<H, 2>(d, nb, nchains, flags, s);
    else launch_nb<H, 4>(d, nb, nchains, flags, s);
}

}  // namespace

extern "C" int64_t ou_gru_workspace_bytes(int hidden, int batch)
{
    return (xcc_slot_base(batch, hidden) + xcc_slot_count(batch, hidden) + (int64_t)kStampSlots * 1024) *
           (int64_t)sizeof(uint64_t);
}

// after a launch: a short one (steps < 5) on a ws_zeroed workspace leaves it
// zeroed for the next launch on it, whatever that one's T
static int gru_after(const ou_gru_desc& d, hipStream_t s)
{
    const int rc = ou_check_launch("gru");
    if (rc == 0 && d.ws_zeroed && d.steps < 5)
        OU_HIP_CHECK(hipMemsetAsync(d.granules, 0, ou_gru_workspace_bytes(d.hidden, d.batch), s), "gru: memset");
    return rc;
}

extern "C" int ou_gru(const ou_gru_desc* dp, void* stream)
{
    if (!dp) return ou_fail(-1, "gru: null descriptor");
    const ou_gru_desc& d = *dp;
    if (!d.gi || !d.b_hh || !d.y || d.steps <= 0 || d.batch <= 0 || d.batch > 32768)
        return ou_fail(-1, "gru: invalid descriptor");
    hipStream_t s = (hipStream_t)stream;
    const bool split = d.t_begin != 0 || (d.t_end != 0 && d.t_end != d.steps);
    // flags: bits 0-11 as documented (or the defaults: d.flags < 0, or bit 15
    // set), bits 12-14 the XCD offset of the chain layout (bit 0)
    const bool dflt = d.flags < 0 || (d.flags & 0x8000);
    const int fbits = dflt ? -1 : (d.flags & 0xfff), fofs = d.flags >= 0 ? (d.flags & 0x7000) : 0;
    if (d.t_begin < 0 || (d.t_end != 0 && (d.t_end <= d.t_begin || d.t_end > d.steps)) || (split && !d.hstate))
        return ou_fail(-1, "gru: bad step range [%d, %d) of %d (hstate %p)", d.t_begin, d.t_end, d.steps,
                       (const void*)d.hstate);
    if (split && (d.hidden % 64 || (fbits >= 0 && (fbits & 32))))
        return ou_fail(-2, "gru: a step range needs the k-split kernel (hidden %% 64 == 0)");
    if (!d.w_hh || !d.granules || !d.status) return ou_fail(-1, "gru: invalid descriptor");
    // the k-split kernel clears its placement slots when it exits.  A launch
    // of T steps leaves the tags T - 1 and T - 2 in the two parity slots (it
    // writes tag t + 1 for t + 1 < T); a new launch's first polls look for
    // tags 1 and 2, and every later poll of a slot follows one that already
    // saw this launch's tag there.  So with T - 2 >= 3 (T >= 5) a workspace
    // zeroed once per replay serves every launch of it (ws_zeroed); shorter
    // launches clear it themselves, before they run and again after (their
    // tags T - 1, T - 2 are < 3: a following launch could match them).
    // a launch continuing a split recurrence (t_begin > 0) starts from hstate:
    // the tags the previous launches left are all older than the ones it polls
    if ((!d.ws_zeroed && d.t_begin == 0) || d.steps < 5)
        OU_HIP_CHECK(hipMemsetAsync(d.granules, 0, ou_gru_workspace_bytes(d.hidden, d.batch), s), "gru: memset");
    // k-split kernel (default for H % 64 == 0; flags bit5 selects the
    // workgroup-gather kernel below)
    if (d.hidden % 64 == 0 && !(fbits >= 0 && (fbits & 32))) {
        const int kflags = (fbits >= 0 ? fbits : 1) | fofs;
        switch (d.hidden) {
        case 64: launch_ks_all<64>(d, kflags, s); break;
        case 128: launch_ks_all<128>(d, kflags, s); break;
        case 256: launch_ks_all<256>(d, kflags, s); break;
        case 384: launch_ks_all<384>(d, kflags, s); break;
        case 512: launch_ks_all<512>(d, kflags, s); break;
        default: return ou_fail(-1, "gru: unsupported hidden size %d", d.hidden);
        }
        return gru_after(d, s);
    }
    const int nb = d.batch >= kMaxBatchPerWG ? kMaxBatchPerWG : (d.batch >= 2 ? 2 : 1);
    const int nchains = 2 * ((d.batch + nb - 1) / nb);
    // default: XCD-local chains; 64-unit workgroups (fewer producers per
    // hand-off) for one item per chain, 32-unit ones when a workgroup carries
    // several items (measured: tools/gru_bench.py)
    const int flags = (fbits >= 0 ? fbits : (nb == 1 ? 5 : 1)) | fofs;
    // every workgroup of a chain must be resident at once: a few hundred
    // workgroups at most, far below 256 CUs x 4
    if (nchains * (d.hidden / 32) > 512) return ou_fail(-2, "gru: grid too large for residency");
    switch (d.hidden) {
    case 32: launch_h<32>(d, nb, nchains, flags, s); break;
    case 64: launch_h<64>(d, nb, nchains, flags, s); break;
    case 128: launch_h<128>(d, nb, nchains, flags, s); break;
    case 256: launch_h<256>(d, nb, nchains, flags, s); break;
    case 384: launch_h<384>(d, nb, nchains, flags, s); break;
    default: return ou_fail(-1, "gru: unsupported hidden size %d", d.hidden);
    }
    return gru_after(d, s);
}
